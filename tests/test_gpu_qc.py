"""GPU parity of the clustering QC estimators, tissue-domain proportions,
tissue masks, the ST feature blur and the use_paths npz round trip, against
values the reference's own functions produced (tests/golden/qc_small.npz,
make_golden.py make_qc) and the oracle.

Tolerances: the device slides and rows are fp32 (the reference float64) with
fp64 accumulation: sums of squares within 1e-5 relative."""
import numpy as np
import pandas as pd
import pytest

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu
FEATS = list(range(8))
TAU = 1e-5  # near-tie: relative top-2 gap of the squared distances


def _preprocessed_imgs(g):
    """Our img objects for the qc_small slides, log-normalised with the batch
    means and blurred, as prep_cluster_data leaves them."""
    import milwrm_amd as M

    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in zip(g["raw"], g["masks"])]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    means = O.batch_means(ests, pix, ["b1", "b1", "b2"])
    for im, b in zip(imgs, ["b1", "b1", "b2"]):
        im.log_normalize(mean=means[b])
        im.blurring("gaussian", sigma=2)
    return imgs


def _scaler(mean, scale):
    from milwrm_amd.kmeans import StandardScaler

    s = StandardScaler()
    s.mean_, s.scale_ = np.asarray(mean, dtype=np.float64), np.asarray(scale, dtype=np.float64)
    return s


@pytest.mark.parametrize("k", [4, 24])
def test_qc_mxif_vs_reference(gpu, golden, k, monkeypatch):
    """estimate_percentage_variance_mxif / estimate_mse_mxif (MILWRM.py:280-333,
    453-515) on the reference's own labelling; k = 24 takes two 20-domain
    passes.  Both blur modes (materialised, and deferred: the QC pass blurs
    band by band -- 13-row bands here -- into a reused buffer and leaves the
    img's raw slide in place); the exact fixed-point sums make the two modes
    BITWISE equal."""
    from milwrm_amd import MILWRM as MW

    g = golden("qc_small")
    cents = g[f"k{k}_centers"]
    sc = _scaler(g[f"k{k}_scaler_mean"], g[f"k{k}_scaler_scale"])
    tids = [np.where(t < 0, np.nan, t.astype(np.float64)) for t in g[f"k{k}_tissue_IDs"]]
    got = {}
    monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", "13")
    for mode in ("0", "1"):
        monkeypatch.setenv("MW_FUSED_BLUR", mode)
        imgs = _preprocessed_imgs(g)
        pv = [MW.estimate_percentage_variance_mxif(im, False, sc, cents, FEATS, t)
              for im, t in zip(imgs, tids)]
        np.testing.assert_allclose(pv, g[f"k{k}_pct_variance"], rtol=1e-5)
        mse = MW.estimate_mse_mxif(imgs, False, tids, sc, cents, FEATS, k)
        mse = np.array([mse[i] for i in range(k)])
        np.testing.assert_allclose(mse, g[f"k{k}_mse"], rtol=2e-5, atol=1e-9)
        got[mode] = (np.array(pv), mse)
        if mode == "1":
            assert all(im._pending_blur is not None for im in imgs)  # nothing materialised
    np.testing.assert_array_equal(got["0"][0], got["1"][0])
    np.testing.assert_array_equal(got["0"][1], got["1"][1])


def test_qc_deferred_50ch_bitwise(gpu, monkeypatch):
    """50-channel slides (the config-5 channel count): the QC estimators on a
    deferred-blur slide (band by band, never a full fp32 copy) are bitwise the
    materialised slide's, and match the oracle's fp64 restatement."""
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW

    raw, mask = O.synth_slide(150, 124, 50, seed=905, mode="hard")
    rng = np.random.default_rng(3)
    k = 6
    mean = raw.reshape(-1, 50).mean(0) + 1.0
    cents = rng.normal(0, 1, size=(k, 50))
    sc = _scaler(rng.normal(0.3, 0.05, 50), rng.uniform(0.05, 0.2, 50))
    tid = rng.integers(-1, k, size=(150, 124)).astype(np.float64)
    tid[tid < 0] = np.nan
    res = {}
    monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", "21")
    for mode in ("0", "1"):
        monkeypatch.setenv("MW_FUSED_BLUR", mode)
        ims = []
        for j in range(2):
            im = M.img(raw.copy(), mask=mask.copy())
            im.log_normalize(mean=mean * (1 + 0.1 * j))
            im.blurring("gaussian", sigma=2)
            ims.append(im)
        assert (ims[0]._pending_blur is not None) == (mode == "1")
        pv = MW.estimate_percentage_variance_mxif(ims[0], False, sc, cents, list(range(50)), tid)
        mse = MW.estimate_mse_mxif(ims, False, [tid, tid], sc, cents, list(range(50)), k)
        res[mode] = (pv, np.array([mse[i] for i in range(k)]))
    assert res["0"][0] == res["1"][0]
    np.testing.assert_array_equal(res["0"][1], res["1"][1])
    pre = O.gaussian_blur(O.log_normalize(raw, mean))
    ref = O.percentage_variance_mxif(pre, list(range(50)), cents, sc.mean_, sc.scale_, tid)
    assert abs(res["0"][0] - ref) <= 1e-5 * abs(ref)


def test_qc_int8_device_labels_and_single_feature(gpu, golden):
    """The labeler's own int8 device label maps as tissue_ID, and a single
    feature (the largest per-lane LDS footprint) against the oracle."""
    import torch

    from milwrm_amd import MILWRM as MW

    g = golden("qc_small")
    imgs = _preprocessed_imgs(g)
    cents = g["k4_centers"]
    sc = _scaler(g["k4_scaler_mean"], g["k4_scaler_scale"])
    t8 = torch.from_numpy(g["k4_tissue_IDs"][0].copy()).cuda()
    pv = MW.estimate_percentage_variance_mxif(imgs[0], False, sc, cents, FEATS, t8)
    np.testing.assert_allclose(pv, g["k4_pct_variance"][0], rtol=1e-5)
    host = imgs[0].img
    tid = np.where(g["k4_tissue_IDs"][0] < 0, np.nan, g["k4_tissue_IDs"][0].astype(float))
    sc1 = _scaler(g["k4_scaler_mean"][[3]], g["k4_scaler_scale"][[3]])
    c1 = cents[:, [3]]
    got = MW.estimate_percentage_variance_mxif(imgs[0], False, sc1, c1, [3], tid)
    ref = O.percentage_variance_mxif(host, [3], c1, sc1.mean_, sc1.scale_, tid)
    np.testing.assert_allclose(got, ref, rtol=1e-5)


def test_qc_constant_feature_and_zero_denominator(gpu):
    """A near-constant feature keeps its digits (shifted sums), and a constant
    slide gives the reference's numpy nan (0/0) rather than an exception."""
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW

    rng = np.random.default_rng(5)
    a = np.empty((64, 80, 2))
    a[:, :, 0] = 1000.0 + rng.normal(0, 1e-3, size=(64, 80))
    a[:, :, 1] = rng.uniform(0, 5, size=(64, 80))
    im = M.img(a.astype(np.float32).astype(np.float64), mask=np.ones((64, 80)))
    tid = (a[:, :, 1] > 2.5).astype(float)
    cents = np.array([[1000.0, 1.25], [1000.0, 3.75]])
    sc = _scaler([0.0, 0.0], [1.0, 1.0])
    got = MW.estimate_percentage_variance_mxif(im, False, sc, cents, [0, 1], tid)
    ref = O.percentage_variance_mxif(im.img, [0, 1], cents, sc.mean_, sc.scale_, tid)
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    flat = M.img(np.full((8, 8, 2), 3.0), mask=np.ones((8, 8)))
    with np.errstate(invalid="ignore", divide="ignore"):
        v = MW.estimate_percentage_variance_mxif(flat, False, sc, np.array([[3.0, 3.0]]), [0, 1],
                                                 np.zeros((8, 8)))
    assert np.isnan(v)


def test_tissue_id_proportions_mxif(gpu, golden):
    """plot_tissue_ID_proportions_mxif (MILWRM.py:2013-2073): the per-image
    domain shares from the label pass's counts; the plot is drawn (Agg)."""
    import matplotlib

    matplotlib.use("Agg")
    import milwrm_amd as M

    g = golden("qc_small")
    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in zip(g["raw"], g["masks"])]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b1", "b1", "b2"],
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=FEATS, sigma=2, fract=0.2)
    lab.label_tissue_regions(k=4, plot_out=False, random_state=18)
    ax = lab.plot_tissue_ID_proportions_mxif()
    assert ax is not None
    tids = [np.nan_to_num(t, nan=-1) for t in lab.tissue_IDs]
    own = O.tissue_id_proportions(tids, 4)
    np.testing.assert_allclose(lab.tissue_ID_proportion.values, own, rtol=1e-12)
    # against the reference: every label equal except near-ties (the
    # reference's own confidence < TAU), and the proportions move by exactly
    # those pixels
    ref_t = [np.nan_to_num(t, nan=-1) for t in g["k4_tissue_IDs"]]
    batches = ["b1", "b1", "b2"]
    e_p = [O.non_zero_mean(r) for r in g["raw"]]
    bm = O.batch_means([e for e, _ in e_p], [p for _, p in e_p], batches)
    moved = 0
    for i, (r, m, t, tr) in enumerate(zip(g["raw"], g["masks"], tids, ref_t)):
        pre = O.gaussian_blur(O.log_normalize(r, bm[batches[i]]))
        cid = O.confidence_mxif(pre, m, FEATS, g["k4_centers"], g["k4_scaler_mean"],
                                g["k4_scaler_scale"], tr)[0]
        diff = t != tr
        assert not (diff & ~(np.nan_to_num(cid, nan=1.0) < TAU)).any(), f"image {i}"
        moved = max(moved, int(diff.sum()))
    n_lab = min(int((t >= 0).sum()) for t in ref_t)
    np.testing.assert_allclose(lab.tissue_ID_proportion.values, g["k4_proportions"],
                               atol=moved / n_lab + 1e-12)


def test_create_tissue_mask_vs_reference(gpu, golden):
    """img.create_tissue_mask (MxIF.py:543-589) against the reference's masks
    (labels equal except at near-ties of the 2-means), and the reference's
    feature-count error for a feature subset."""
    import milwrm_amd as M

    g = golden("qc_small")
    for r, ref in zip(g["raw"][:2], g["tissue_mask"]):
        im = M.img(r.copy())
        im.create_tissue_mask()
        got = np.asarray(im.mask, dtype=np.float64)
        assert got.shape == ref.shape
        # mismatches only where the 2-means gap of the (pinned) oracle is a
        # near-tie: relative gap of the squared distances < TAU
        own, gap = O.create_tissue_mask(r, return_gap=True)
        np.testing.assert_array_equal(own, ref)  # the oracle reproduces the reference here
        bad = (got != ref) & ~(np.nan_to_num(gap, nan=0.0) < TAU)
        assert not bad.any(), f"{int(bad.sum())} mask pixels differ outside near-ties"
    im = M.img(g["raw"][0].copy())
    with pytest.raises(ValueError, match="features"):
        im.create_tissue_mask(features=[0, 1, 2])


class _Duck:
    def __init__(self, n, labels=None, categories=None):
        self.n_obs = n
        self.obs = pd.DataFrame(index=[str(i) for i in range(n)])
        if labels is not None:  # as st_labeler.label_tissue_regions sets it (MILWRM.py:1080-1089)
            self.obs["tissue_ID"] = pd.Categorical(labels, categories=categories)


def test_qc_st_vs_reference(gpu, golden):
    """estimate_percentage_variance_st / estimate_mse_st (MILWRM.py:518-554,
    601-644, including the reference's section offsets) and the ST domain
    proportions (plot_tissue_ID_proportions_st, MILWRM.py:1400-1452)."""
    import matplotlib

    matplotlib.use("Agg")
    from milwrm_amd import MILWRM as MW

    g = golden("qc_small")
    X, cents, labels = g["st_cluster_data"], g["st_centers"], g["st_labels"]
    n_obs = [g[f"st_pcs{s}"].shape[0] for s in range(3)]
    offs = np.concatenate([[0], np.cumsum(n_obs)])
    ads = [_Duck(n_obs[s], labels[offs[s]:offs[s + 1]], np.unique(labels)) for s in range(3)]
    pv = [MW.estimate_percentage_variance_st(X[offs[s]:offs[s + 1]], ads[s], cents) for s in range(3)]
    # fp64 rows (mw_domain_sse_f64) and two-level fixed-point sums: fp64-grade
    # against the reference's numpy float64 sums
    np.testing.assert_allclose(pv, g["st_pct_variance"], rtol=1e-11)
    mse = MW.estimate_mse_st(X, ads, cents, 5)
    np.testing.assert_allclose(np.array([mse[i] for i in range(5)]), g["st_mse"], rtol=1e-11, atol=1e-15)
    st = MW.st_labeler.__new__(MW.st_labeler)
    st.adatas = ads
    st.plot_tissue_ID_proportions_st()
    np.testing.assert_allclose(st.tissue_ID_proportion.values, g["st_proportions"], rtol=1e-12)


def test_blur_features_st_device_vs_oracle(gpu, golden):
    """blur_features_st (ST.py:25-77) on the device CSR neighbour mean: the
    oracle's neighbour mean on the golden hex graph, a self-loop counted twice,
    and NaN features skipped as pandas' mean does."""
    import scipy.sparse as sp

    import milwrm_amd as M

    g = golden("st_hex")
    n = g["pcs0"].shape[0]
    A = sp.csr_matrix((np.ones(len(g["adj0_indices"])), g["adj0_indices"], g["adj0_indptr"]),
                      shape=(n, n)).tolil()
    A[5, 5] = 1.0  # self-loop
    A = A.tocsr()
    X = g["pcs0"].copy()
    X[7, 2] = np.nan
    ad = _Duck(n)
    ad.obsp = {"g": A}
    tmp = pd.DataFrame(X, columns=[f"X_pca_{i}" for i in range(X.shape[1])])
    got = M.blur_features_st(ad, tmp, spatial_graph_key="g").values
    ref = np.empty_like(X)
    for x in range(n):
        nb = list(A.indices[A.indptr[x]:A.indptr[x + 1]]) + [x]
        ref[x] = pd.DataFrame(X[nb]).mean().values
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(ad.obs["blur_X_pca_0"].values, ref[:, 0], rtol=1e-12)


def test_use_paths_npz_round_trip(gpu, golden, tmp_path):
    """mxif_labeler with image paths (MILWRM.py:205-233, 258-260): npz in,
    preprocessed npz out under _final_preprocessed_images, labels and
    confidences equal to the in-memory run."""
    import milwrm_amd as M

    g = golden("mxif_small")
    paths = []
    for i in range(3):
        p = str(tmp_path / f"slide{i}")
        M.img(g["raw"][i].copy(), mask=g["masks"][i].copy()).to_npz(p)
        paths.append(p)
    ests, pix = zip(*[M.img.from_npz(p + ".npz").calculate_non_zero_mean() for p in paths])
    df = pd.DataFrame({"Img": paths, "batch_names": ["b1", "b1", "b2"],
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    assert lab.use_paths
    with pytest.raises(Exception, match="requird"):
        lab.prep_cluster_data(features=FEATS, sigma=2, fract=0.2)
    lab.prep_cluster_data(features=FEATS, sigma=2, fract=0.2, path_save=str(tmp_path))
    saved = list(lab.image_df["Img"])
    assert all(p.endswith("_final_preprocessed") for p in saved)
    assert all((tmp_path / "_final_preprocessed_images" / (p.split("/")[-1] + ".npz")).exists()
               for p in saved)
    lab.label_tissue_regions(k=4, plot_out=False, random_state=18)
    lab.confidence_score_images()
    imgs = [M.img(g["raw"][i].copy(), mask=g["masks"][i].copy()) for i in range(3)]
    ests2, pix2 = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df2 = pd.DataFrame({"Img": imgs, "batch_names": ["b1", "b1", "b2"],
                        "mean estimators": list(ests2), "pixels": list(pix2)})
    mem = M.mxif_labeler(df2)
    mem.prep_cluster_data(features=FEATS, sigma=2, fract=0.2)
    mem.label_tissue_regions(k=4, plot_out=False, random_state=18)
    mem.confidence_score_images()
    np.testing.assert_array_equal(lab.kmeans.cluster_centers_, mem.kmeans.cluster_centers_)
    for i in range(3):
        np.testing.assert_array_equal(np.nan_to_num(lab.tissue_IDs[i], nan=-1),
                                      np.nan_to_num(mem.tissue_IDs[i], nan=-1))
    np.testing.assert_array_equal(lab.confidence_score_df.values, mem.confidence_score_df.values)


def test_qc_nonfinite_feature_gives_nan(gpu):
    """A non-finite value in a slide (fp32 input) has no fixed point in the
    exact QC sums: the quantities of its feature are NaN, as the reference's
    numpy sums are; the other features keep their values."""
    from milwrm_amd import MILWRM as MW
    import milwrm_amd as M

    raw, mask = O.synth_slide(64, 80, 4, seed=5, mode="hard")
    x = raw.astype(np.float32)
    tid = np.where(mask != 0, (np.arange(64 * 80).reshape(64, 80) % 3).astype(np.float64), np.nan)
    cents = np.random.RandomState(0).normal(size=(3, 4))
    sc = _scaler(np.zeros(4), np.full(4, 100.0))
    clean = MW.estimate_mse_mxif([M.img(x.copy(), mask=mask.copy())], False, [tid], sc, cents,
                                 list(range(4)), 3)
    x[10, 20, 2] = np.nan
    im = M.img(x, mask=mask.copy())
    pv = MW.estimate_percentage_variance_mxif(im, False, sc, cents, list(range(4)), tid)
    assert np.isnan(pv)
    mse = MW.estimate_mse_mxif([M.img(x.copy(), mask=mask.copy())], False, [tid], sc, cents,
                               list(range(4)), 3)
    for d in range(3):
        assert np.isnan(mse[d][0][2])
        np.testing.assert_array_equal(np.delete(mse[d][0], 2), np.delete(clean[d][0], 2))


@pytest.mark.parametrize("mode", ["materialised", "banded", "fused"])
def test_label_pass_qc_equals_estimators(gpu, golden, monkeypatch, mode):
    """label_tissue_regions(qc=True): the QC sums behind
    plot_percentage_variance_explained / plot_mse_mxif (MILWRM.py:1796-2011)
    taken as extra outputs of the label pass -- the resident slide whole, a
    deferred-blur slide band by band from the label pass's own fp32 bands
    (21-row bands: no second blur) -- are bitwise the estimators' own passes
    (fixed point from the raw slide's bound, img._blur_bound, in both).  The
    fused label epilogue has no fp32 band: the estimators run their pass and
    give the same bits.  S^2 against the oracle's fp64 restatement on the same
    labels."""
    import matplotlib

    matplotlib.use("Agg")
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW

    g = golden("qc_small")
    monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", "21")
    monkeypatch.setenv("MW_FUSED_BLUR", "0" if mode == "materialised" else "1")
    monkeypatch.setenv("MW_DEFERRED_ASSIGN", "fused" if mode == "fused" else "band")
    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in zip(g["raw"], g["masks"])]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    batches = ["b1", "b1", "b2"]
    df = pd.DataFrame({"Img": imgs, "batch_names": batches,
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=FEATS, sigma=2, fract=0.2)
    assert all((im._pending_blur is not None) == (mode != "materialised") for im in imgs)
    assert all(im._xbound is not None for im in imgs)
    lab.label_tissue_regions(k=4, plot_out=False, random_state=18, qc=True)
    taken = [s is not None for s in lab._qc_stats]
    assert all(taken) if mode != "fused" else not any(taken)
    pv = lab.percentage_variance_images()
    mse = lab.mse_images()
    cents = lab.kmeans.cluster_centers_
    tids = list(lab.tissue_IDs)
    est_pv = [MW.estimate_percentage_variance_mxif(im, False, lab.scaler, cents, FEATS, t)
              for im, t in zip(imgs, tids)]
    est_mse = MW.estimate_mse_mxif(imgs, False, tids, lab.scaler, cents, FEATS, 4)
    np.testing.assert_array_equal(pv, est_pv)
    for i in range(4):
        np.testing.assert_array_equal(np.array(mse[i]), np.array(est_mse[i]))
    assert lab.plot_percentage_variance_explained(R_square=True) is not None
    assert lab.plot_mse_mxif() is not None
    e_p = [O.non_zero_mean(r) for r in g["raw"]]
    bm = O.batch_means([e for e, _ in e_p], [p for _, p in e_p], batches)
    for i, r in enumerate(g["raw"]):
        pre = O.gaussian_blur(O.log_normalize(r, bm[batches[i]]))
        ref = O.percentage_variance_mxif(pre, FEATS, cents, lab.scaler.mean_, lab.scaler.scale_, tids[i])
        assert abs(pv[i] - ref) <= 1e-5 * abs(ref), f"image {i}"
