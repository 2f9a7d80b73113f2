"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import milwrm_oracle as O


def _nan_i8(a):
    a = a.astype(np.float64)
    a[a < 0] = np.nan
    return a


def test_non_zero_mean_and_batch_means(golden):
    g = golden("mxif_small")
    ests, pix = zip(*[O.non_zero_mean(r) for r in g["raw"]])
    np.testing.assert_array_equal(np.array(ests), g["mean_estimators"])
    np.testing.assert_array_equal(np.array(pix), g["pixels"])
    bm = O.batch_means(ests, pix, list(g["batch_names"]))
    np.testing.assert_array_equal(bm["b1"], g["batch_mean_b1"])
    np.testing.assert_array_equal(bm["b2"], g["batch_mean_b2"])


def test_lognorm_blur_matches_reference(golden):
    g = golden("mxif_small")
    bm = g["batch_mean_b1"]
    x = O.gaussian_blur(O.log_normalize(g["raw"][0], bm), 2.0)
    np.testing.assert_allclose(x, g["preprocessed0"], rtol=1e-12, atol=1e-14)
    x2 = O.gaussian_blur(O.log_normalize(g["raw"][2], g["batch_mean_b2"]), 2.0)
    np.testing.assert_allclose(x2, g["preprocessed2"], rtol=1e-12, atol=1e-14)


def test_subsample_and_scaler(golden):
    g = golden("mxif_small")
    subs = []
    for i, b in enumerate(["b1", "b1", "b2"]):
        bm = g["batch_mean_b1"] if b == "b1" else g["batch_mean_b2"]
        x = O.gaussian_blur(O.log_normalize(g["raw"][i], bm), 2.0)
        s, idx = O.subsample_pixels(x, g["masks"][i], list(range(8)), 0.2)
        subs.append(s)
        if i == 0:
            np.testing.assert_array_equal(idx, g["sub_idx0"])
    X = np.vstack(subs)
    mean, scale, _ = O.scaler_fit(X)
    np.testing.assert_allclose(mean, g["scaler_mean"], rtol=1e-13)
    np.testing.assert_allclose(scale, g["scaler_scale"], rtol=1e-13)
    np.testing.assert_allclose(O.scaler_transform(X, mean, scale), g["cluster_data"], rtol=1e-11, atol=1e-12)


def test_legacy_randint_restatement():
    for M, fr in [(6540, 0.2), (1000, 0.5), (2**20, 0.01), (2**20 + 1, 0.01), (123457, 0.3)]:
        np.random.seed(16)
        ref = np.random.choice(M, int(M * fr))
        mine = O.legacy_randint_masked(16, M, int(M * fr))
        np.testing.assert_array_equal(mine, ref)


def test_kmeans_plusplus_indices(golden):
    g = golden("mxif_small")
    X = g["cluster_data"]
    Xc = X - X.mean(axis=0)
    for k in (2, 3, 8, 13, 20):
        _, idx = O.kmeans_plusplus(Xc, k, 18)
        np.testing.assert_array_equal(idx, g["kpp_indices"][k, :k])


def _kpp_margins(X, k, seed=18):
    """Per k-means++ step (sklearn _kmeans.py:225-272 on centered X): the
    relative distance of every target u * pot to the cumulative-sum
    boundaries around the row it selects, and the relative gap between the
    best and second-best trial potentials (distinct candidates)."""
    n = X.shape[0]
    rs = np.random.RandomState(seed)
    T = 2 + int(np.log(k))
    x_sq = np.einsum("ij,ij->i", X, X)
    closest = O._sq_dist_gemm(X, X[[rs.choice(n, p=np.ones(n) / n)]], x_sq)[:, 0]
    pot = closest.sum()
    out = []
    for _ in range(1, k):
        rv = rs.uniform(size=T) * pot
        cum = np.cumsum(closest)
        cand = np.minimum(np.searchsorted(cum, rv), n - 1)
        lo = np.where(cand > 0, cum[cand - 1], 0.0)
        cmarg = float((np.minimum(np.abs(cum[cand] - rv), np.abs(rv - lo)) / pot).min())
        d = O._sq_dist_gemm(X, X[cand], x_sq).T
        np.minimum(closest, d, out=d)
        pots = d.sum(axis=1)
        o = np.argsort(pots, kind="stable")
        gap = float((pots[o[1]] - pots[o[0]]) / pots[o[0]]) if cand[o[1]] != cand[o[0]] else np.inf
        out.append((cmarg, gap))
        b = int(np.argmin(pots))
        pot, closest = pots[b], d[b]
    return out


def test_kpp_decision_margins(golden):
    """Round-2 DESIGN recorded a reverted k-means++ variant whose golden
    indices changed at k = 12 (cause not found) and the verdict asked whether
    index parity hangs on fp64 summation order.  It does not on this fixture:
    every decision of every k = 2..20 seeding sits >= 1.7e-6 relative from its
    boundary (target vs cumulative sum) and >= 4.7e-4 between the best two
    trial potentials -- ten orders of magnitude above any reordering of fp64
    sums (~1e-15), so a flip there means different distances (a defect of
    that variant), not rounding.  What the margins are comparable to is the
    fp32 storage of the clustering rows (~6e-8 per element, the design's
    documented precision): at n rows a target's margin scales like 1/n."""
    g = golden("mxif_small")
    X = g["cluster_data"]
    Xc = X - X.mean(axis=0)
    cm, sg = np.inf, np.inf
    for k in range(2, 21):
        for c, s in _kpp_margins(Xc, k):
            cm, sg = min(cm, c), min(sg, s)
    assert cm > 1e-6 and sg > 4e-4, (cm, sg)


def test_first_center_closed_form_vs_numpy():
    for n in (1, 7, 6297, 100003, 2**20):
        rs = np.random.RandomState(18)
        ref = rs.choice(n, p=np.ones(n) / n)
        u = np.random.RandomState(18).random_sample()
        assert O.first_center_index(n, u) == ref


def test_single_lloyd_step(golden):
    g = golden("mxif_small")
    X = g["cluster_data"]
    Xc = X - X.mean(axis=0)
    labels, cn, w, shift = O.lloyd_iter(Xc, g["lloyd1_centers_in"])
    np.testing.assert_array_equal(labels, g["lloyd1_labels"])
    np.testing.assert_allclose(cn, g["lloyd1_centers_out"], rtol=1e-12, atol=1e-13)
    np.testing.assert_array_equal(w, g["lloyd1_weights"])
    np.testing.assert_allclose(shift, g["lloyd1_shift"], rtol=1e-11)


def test_kmeans_fit_and_sweep(golden):
    g = golden("mxif_small")
    X = g["cluster_data"]
    best_k, curve = O.choose_best_k(X, range(2, 21), 0.05, 18)
    assert best_k == int(g["best_k"])
    np.testing.assert_allclose([curve[k] for k in range(2, 21)], g["sweep_scaled_inertia"], rtol=1e-10)
    r = O.kmeans_fit(X, int(g["k"]), 18)
    np.testing.assert_array_equal(r["labels_"], g["labels"])
    np.testing.assert_allclose(r["cluster_centers_"], g["centers"], rtol=1e-10, atol=1e-12)
    assert r["n_iter_"] == int(g["n_iter"])
    np.testing.assert_allclose(r["inertia_"], float(g["inertia"]), rtol=1e-10)


def test_tissue_ids_and_confidence(golden):
    g = golden("mxif_small")
    centers, mean, scale = g["centers"], g["scaler_mean"], g["scaler_scale"]
    for i, b in enumerate(["b1", "b1", "b2"]):
        bm = g["batch_mean_b1"] if b == "b1" else g["batch_mean_b2"]
        x = O.gaussian_blur(O.log_normalize(g["raw"][i], bm), 2.0)
        t = O.tissue_ids(x, g["masks"][i], list(range(8)), centers, mean, scale)
        np.testing.assert_array_equal(np.nan_to_num(t, nan=-1), np.nan_to_num(_nan_i8(g["tissue_IDs"][i]), nan=-1))
        c, cm = O.confidence_mxif(x, g["masks"][i], list(range(8)), centers, mean, scale, t)
        np.testing.assert_allclose(c, g["confidence_IDs"][i], rtol=1e-9, atol=1e-12, equal_nan=True)
        np.testing.assert_allclose([cm[j] for j in range(len(centers))], g["confidence_score_df"][i],
                                   rtol=1e-9, equal_nan=True)


def test_pipeline_hard256(golden):
    g = golden("mxif_hard256")
    r = O.mxif_pipeline([g["raw"]], [g["mask"]], ["b"], list(range(30)), k=8)
    np.testing.assert_allclose(r["kmeans"]["cluster_centers_"], g["centers"], rtol=1e-9, atol=1e-11)
    assert r["kmeans"]["n_iter_"] == int(g["n_iter"])
    np.testing.assert_allclose(r["kmeans"]["inertia_"], float(g["inertia"]), rtol=1e-10)
    t = np.nan_to_num(r["tissue_IDs"][0], nan=-1).astype(np.int8)
    np.testing.assert_array_equal(t, g["tissue_IDs"])
    np.testing.assert_allclose(r["confidence_IDs"][0], g["confidence_IDs"], rtol=1e-6, equal_nan=True)


def test_gaussian_edges_and_downsample(golden):
    g = golden("preproc_edges")
    for i in range(5):
        out = O.gaussian_blur(g[f"gauss{i}_in"], float(g[f"gauss{i}_sigma"]))
        np.testing.assert_allclose(out, g[f"gauss{i}_out"], rtol=1e-12, atol=1e-14)
    for i in range(3):
        f = int(g[f"down{i}_fact"])
        np.testing.assert_allclose(O.block_reduce_mean(g[f"down{i}_in"], f), g[f"down{i}_out"], rtol=1e-14)
        np.testing.assert_allclose(O.block_reduce_mean(g[f"down{i}_mask"], f), g[f"down{i}_mask_out"], rtol=1e-14)
    np.testing.assert_allclose(O.log_normalize(g["lognorm_none_in"]), g["lognorm_none_out"], rtol=1e-14)


def test_st_plumbing(golden):
    import scipy.sparse as sp

    g = golden("st_hex")
    feats = []
    for s in range(2):
        n = g[f"pcs{s}"].shape[0]
        A = sp.csr_matrix((np.ones(len(g[f"adj{s}_indices"])), g[f"adj{s}_indices"], g[f"adj{s}_indptr"]), shape=(n, n))
        feats.append(O.blur_features_st(g[f"pcs{s}"], A))
    X = np.vstack(feats)
    mean, scale, _ = O.scaler_fit(X)
    Xs = O.scaler_transform(X, mean, scale)
    np.testing.assert_allclose(Xs, g["cluster_data"], rtol=1e-10, atol=1e-12)
    r = O.kmeans_fit(Xs, int(g["k"]), 18)
    np.testing.assert_array_equal(r["labels_"], g["labels"])
    n0 = g["pcs0"].shape[0]
    c0, _ = O.confidence_st(Xs[:n0], r["cluster_centers_"], r["labels_"][:n0])
    np.testing.assert_allclose(c0, g["conf0"], rtol=1e-9)


# ---- QC estimators, proportions, tissue masks (tests/golden/qc_small.npz) ----

def _qc_images(g):
    """The mxif_small slides preprocessed as the reference does before QC
    (batch means, log-normalise, Gaussian) -> host float64 HWC."""
    raw, masks = g["raw"], g["masks"]
    ests, pix = zip(*[O.non_zero_mean(r) for r in raw])
    means = O.batch_means(ests, pix, ["b1", "b1", "b2"])
    out = []
    for r, b in zip(raw, ["b1", "b1", "b2"]):
        out.append(O.gaussian_blur(O.log_normalize(r, means[b]), 2.0))
    return out


@pytest.mark.parametrize("k", [4, 24])
def test_qc_mxif_oracle(golden, k):
    g = golden("qc_small")
    imgs = _qc_images(g)
    cents, mean, scale = g[f"k{k}_centers"], g[f"k{k}_scaler_mean"], g[f"k{k}_scaler_scale"]
    tids = [np.where(t < 0, np.nan, t.astype(np.float64)) for t in g[f"k{k}_tissue_IDs"]]
    pv = [O.percentage_variance_mxif(im, list(range(8)), cents, mean, scale, t)
          for im, t in zip(imgs, tids)]
    np.testing.assert_allclose(pv, g[f"k{k}_pct_variance"], rtol=1e-10)
    mse = O.mse_mxif(imgs, tids, list(range(8)), cents, mean, scale, k)
    np.testing.assert_allclose(np.array([mse[i] for i in range(k)]), g[f"k{k}_mse"], rtol=1e-10,
                               atol=1e-14)
    np.testing.assert_allclose(O.tissue_id_proportions(g[f"k{k}_tissue_IDs"], k),
                               g[f"k{k}_proportions"], rtol=1e-12)


def test_qc_st_oracle(golden):
    g = golden("qc_small")
    X, cents, labels = g["st_cluster_data"], g["st_centers"], g["st_labels"]
    n_obs = [g[f"st_pcs{s}"].shape[0] for s in range(3)]
    offs = np.concatenate([[0], np.cumsum(n_obs)])
    labs = [labels[offs[s]:offs[s + 1]] for s in range(3)]
    pv = [O.percentage_variance_st(X[offs[s]:offs[s + 1]], cents, labs[s]) for s in range(3)]
    np.testing.assert_allclose(pv, g["st_pct_variance"], rtol=1e-10)
    mse = O.mse_st(X, labs, n_obs, cents, 5)
    np.testing.assert_allclose(np.array([mse[i] for i in range(5)]), g["st_mse"], rtol=1e-10)
    props = np.stack([np.bincount(l, minlength=5) / len(l) for l in labs])
    np.testing.assert_allclose(props, g["st_proportions"], rtol=1e-12)


def test_create_tissue_mask_oracle(golden):
    g = golden("qc_small")
    for r, ref in zip(g["raw"][:2], g["tissue_mask"]):
        np.testing.assert_array_equal(O.create_tissue_mask(r), ref)


def test_st_k8_oracle(golden):
    """The oracle's KMeans on the st_hex rows at config 1's k = 8 reproduces
    the reference run at k = 8 (st_hex_k8.npz)."""
    g, g8 = golden("st_hex"), golden("st_hex_k8")
    km = O.kmeans_fit(g["cluster_data"], 8, random_state=18)
    np.testing.assert_array_equal(km["labels_"], g8["labels"])
    assert km["n_iter_"] == int(g8["n_iter"])
    np.testing.assert_allclose(km["cluster_centers_"], g8["centers"], rtol=1e-10, atol=1e-12)
