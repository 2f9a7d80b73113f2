"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-generated golden vectors.

Tolerances (north_star): labels bit-exact except near-ties (oracle cID <
TAU), centers / inertia / confidence within 1e-4 relative (fp32 storage,
fp64 accumulation), best_k identical."""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu
TAU = 1e-5
RTOL = 1e-4


def _nan_i8(a):
    a = a.astype(np.float64)
    a[a < 0] = np.nan
    return a


def _labels_match(got, ref, cid_ref):
    """Equal except at near-ties (reference cID < TAU)."""
    got = np.nan_to_num(np.asarray(got, dtype=np.float64), nan=-1)
    ref = np.nan_to_num(np.asarray(ref, dtype=np.float64), nan=-1)
    diff = got != ref
    near = np.nan_to_num(cid_ref, nan=1.0) < TAU
    assert not np.any(diff & ~near), f"{int((diff & ~near).sum())} non-tie label mismatches"


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_nz_stats(gpu, golden):
    import milwrm_amd as M

    g = golden("mxif_small")
    for i in range(3):
        im = M.img(g["raw"][i].copy(), mask=g["masks"][i].copy())
        est, pix = im.calculate_non_zero_mean()
        assert pix == int(g["pixels"][i])
        np.testing.assert_array_equal(np.array(est), g["mean_estimators"][i])


def test_lognorm_blur(gpu, golden):
    import milwrm_amd as M

    g = golden("mxif_small")
    for i, key, bm in [(0, "preprocessed0", g["batch_mean_b1"]), (2, "preprocessed2", g["batch_mean_b2"])]:
        im = M.img(g["raw"][i].copy(), mask=g["masks"][i].copy())
        im.log_normalize(mean=bm)
        im.blurring("gaussian", sigma=2)
        np.testing.assert_allclose(im.img, g[key], rtol=2e-6, atol=2e-6)


def test_lognorm_standalone_and_mean_none(gpu, golden):
    import milwrm_amd as M

    g = golden("preproc_edges")
    im = M.img(g["lognorm_none_in"].copy(), mask=np.ones(g["lognorm_none_in"].shape[:2]))
    im.log_normalize()
    np.testing.assert_allclose(im.img, g["lognorm_none_out"], rtol=2e-6, atol=1e-6)


def test_blur_edges_and_fallback_radius(gpu, golden):
    import milwrm_amd as M

    g = golden("preproc_edges")
    for i in range(5):
        a = g[f"gauss{i}_in"]
        im = M.img(a.copy(), mask=np.ones(a.shape[:2]))
        im.blurring("gaussian", sigma=float(g[f"gauss{i}_sigma"]))
        np.testing.assert_allclose(im.img, g[f"gauss{i}_out"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.float32])
@pytest.mark.parametrize("shape,sigma", [((70, 131, 30), 2.0), ((37, 64, 16), 1.0),
                                         ((20, 200, 8), 0.5), ((300, 67, 64), 2.0),
                                         ((9, 5, 2), 2.0), ((40, 72, 6), 1.5)])
def test_fused_lognorm_blur_kernels(gpu, dtype, shape, sigma):
    """Fused log-normalise + blur (matrix-core and VALU fast paths) against the
    fp64 oracle over input dtypes, channel counts (pad channels, 1-4 channel
    tiles), radii and band geometries (edge bands, partial last band, images
    narrower than one band).  Tolerance: fp32 rounding of ~2r+1 products."""
    import os

    import torch

    from milwrm_amd import device as D

    import zlib

    rng = np.random.default_rng(zlib.crc32(repr((shape, sigma, np.dtype(dtype).str)).encode()))
    hi = 255 if dtype == np.uint8 else 4000
    a = rng.integers(0, hi, size=shape).astype(dtype)
    a[rng.random(shape) < 0.05] = 0
    inv = (1.0 / rng.uniform(50, 500, size=shape[2])).astype(np.float32)
    ref = O.gaussian_blur(O.log_normalize(a.astype(np.float64), mean=1.0 / inv.astype(np.float64)),
                          sigma=sigma)
    x = D.to_device_image(a)
    inv_d = torch.from_numpy(inv).cuda()
    for impl in ("mfma", "valu"):
        if impl == "valu":
            os.environ["MW_BLUR_IMPL"] = "valu"
        try:
            got = D.blur(x, sigma, inv_mean=inv_d).cpu().numpy()
        finally:
            os.environ.pop("MW_BLUR_IMPL", None)
        np.testing.assert_allclose(got, ref, rtol=2e-6, atol=2e-7, err_msg=impl)


def test_downsample(gpu, golden):
    import milwrm_amd as M

    g = golden("preproc_edges")
    for i in range(3):
        im = M.img(g[f"down{i}_in"].copy(), mask=g[f"down{i}_mask"].copy())
        im.downsample(int(g[f"down{i}_fact"]))
        np.testing.assert_allclose(im.img, g[f"down{i}_out"], rtol=1e-6)
        np.testing.assert_allclose(im.mask, g[f"down{i}_mask_out"], rtol=1e-6)


def test_subsample_gather(gpu, golden):
    import milwrm_amd as M

    g = golden("mxif_small")
    im = M.img(g["raw"][0].copy(), mask=g["masks"][0].copy())
    im.log_normalize(mean=g["batch_mean_b1"])
    im.blurring("gaussian", sigma=2)
    X = im.subsample_pixels(list(range(8)), 0.2)
    ref, idx = O.subsample_pixels(g["preprocessed0"], g["masks"][0], list(range(8)), 0.2)
    np.testing.assert_array_equal(idx, g["sub_idx0"])
    assert X.shape == ref.shape
    np.testing.assert_allclose(X, ref, rtol=2e-6, atol=2e-6)
    # feature subset and order
    X2 = im.subsample_pixels([5, 1, 3], 0.2)
    np.testing.assert_allclose(X2, ref[:, [5, 1, 3]], rtol=2e-6, atol=2e-6)


def test_kmeans_plusplus_indices(gpu, golden):
    from milwrm_amd.kmeans import DeviceRows, _kmeans_plusplus_device

    g = golden("mxif_small")
    rows = DeviceRows.from_host(g["cluster_data"])
    for k in range(2, 21):
        _, idx = _kmeans_plusplus_device(rows, k, np.random.RandomState(18))
        np.testing.assert_array_equal(idx, g["kpp_indices"][k, :k], err_msg=f"k={k}")


def test_single_lloyd_step(gpu, golden):
    """One Lloyd iteration from the golden centers (lloyd_iter_chunked_dense):
    labels bitwise (outside reference near-ties), cluster sizes exactly,
    averaged centers and center shift against the reference's step."""
    from milwrm_amd.kmeans import DeviceRows, lloyd_step_device

    g = golden("mxif_small")
    X = g["cluster_data"]
    Xc = X - X.mean(axis=0)
    cin = g["lloyd1_centers_in"]
    rows = DeviceRows.from_host(Xc)
    lab, sums, w = lloyd_step_device(rows, cin)
    lab = lab.cpu().numpy().astype(np.int32)
    d = np.sort(((Xc[:, None, :] - cin[None]) ** 2).sum(-1), axis=1)
    near = (d[:, 1] - d[:, 0]) / d[:, 1] < TAU
    ref_lab = g["lloyd1_labels"]
    moved = lab != ref_lab
    assert not np.any(moved & ~near)
    # cluster sizes, always checked: ours are the counts of our labels, and
    # they differ from the reference's exactly by the near-tie rows that moved
    k = len(w)
    np.testing.assert_array_equal(w, np.bincount(lab, minlength=k))
    delta = np.bincount(lab[moved], minlength=k) - np.bincount(ref_lab[moved], minlength=k)
    np.testing.assert_array_equal(w, g["lloyd1_weights"] + delta)
    assert np.all(w > 0)
    centers = sums / w[:, None]
    np.testing.assert_allclose(centers, g["lloyd1_centers_out"], rtol=RTOL, atol=1e-6)
    shift = np.sqrt(((centers - cin) ** 2).sum(axis=1))
    np.testing.assert_allclose(shift, g["lloyd1_shift"], rtol=1e-3, atol=1e-6)


def test_bounded_lloyd_labels_are_argmin(gpu, monkeypatch):
    """The bound-pruned E-step (rows whose bounds prove their label skip the
    distances) gives every row the label of the plain fp32 argmin: after a
    fit, one full E-step (mode 1) with the final centers changes nothing on a
    strictly converged fit, and the labels equal a brute-force argmin."""
    from milwrm_amd import kmeans as KM
    from milwrm_amd.kmeans import DeviceRows, KMeans, LAST_STATS

    # the Python Lloyd loop records the per-pass statistics read below (the
    # C driver does not); start from none so no earlier fit's stats leak in
    monkeypatch.setattr(KM, "USE_C_FIT", False)
    LAST_STATS.clear()
    rng = np.random.default_rng(3)
    X = np.concatenate([rng.normal(m, 1.0, size=(4000, 12)) for m in (-2, 0, 2, 4)])
    X = (X - X.mean(0)) / X.std(0)
    rows = DeviceRows.from_host(X)
    km = KMeans(n_clusters=6, random_state=18, tol=0.0).fit(rows)
    assert sum(LAST_STATS["recomputed"]) < km.n_iter_ * X.shape[0]  # the bounds pruned work
    c32 = km.cluster_centers_.astype(np.float32).astype(np.float64)
    x32 = X.astype(np.float32).astype(np.float64)
    d = ((x32[:, None, :] - c32[None]) ** 2).sum(-1)
    ds = np.sort(d, axis=1)
    near = (ds[:, 1] - ds[:, 0]) / ds[:, 1] < TAU
    lab = km.labels_
    assert not np.any((lab != np.argmin(d, axis=1)) & ~near)


def test_kmeans_fit_matches_reference(gpu, golden):
    import milwrm_amd as M

    g = golden("mxif_small")
    km = M.KMeans(n_clusters=int(g["k"]), random_state=18).fit(g["cluster_data"])
    assert km.n_iter_ == int(g["n_iter"])
    np.testing.assert_array_equal(km.labels_, g["labels"])
    assert _rel(km.cluster_centers_, g["centers"]) < RTOL
    assert abs(km.inertia_ - float(g["inertia"])) / float(g["inertia"]) < RTOL
    np.testing.assert_array_equal(km.predict(g["cluster_data"]), g["labels"])


def test_sweep_best_k(gpu, golden):
    import milwrm_amd as M

    g = golden("mxif_small")
    best_k, res = M.chooseBestKforKMeansParallel(g["cluster_data"], range(2, 21), random_state=18,
                                                 alpha_k=0.05)
    assert best_k == int(g["best_k"])
    np.testing.assert_allclose(res["Scaled Inertia"].values, g["sweep_scaled_inertia"], rtol=RTOL)


def _sweep_rows(golden, which):
    from milwrm_amd.kmeans import DeviceRows

    if which == "mxif_small":
        return DeviceRows.from_host(golden("mxif_small")["cluster_data"])
    if which == "noise":  # unstructured: long, uneven convergence across k
        X = np.random.default_rng(7).standard_normal((20000, 8))
        return DeviceRows.from_host(X)
    import milwrm_amd as M

    g = golden("mxif_hard256")
    im = M.img(g["raw"].copy(), mask=g["mask"].copy())
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                       "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(g["raw"].shape[2])), sigma=2, fract=0.2)
    return lab._device_rows()


@pytest.mark.parametrize("which", ["mxif_small", "hard256", "noise"])
def test_batched_sweep_equals_separate_fits(gpu, golden, which):
    """find_optimal_k's batched Lloyd (all k in one pass per iteration,
    mw_lloyd_pass with every running fit) returns exactly what separate KMeans fits return:
    same k-means++ indices, n_iter, labels, and bitwise equal centers and
    inertia for k = 2..20 (both M-step classes, k <= 16 and 17..20)."""
    from milwrm_amd.kmeans import KMeans, fit_many

    rows = _sweep_rows(golden, which)
    ks = list(range(2, 21))
    many = fit_many(rows, ks, random_state=18)
    for k, b in zip(ks, many):
        a = KMeans(n_clusters=k, random_state=18).fit(rows)
        np.testing.assert_array_equal(a.init_indices_, b.init_indices_)
        assert a.n_iter_ == b.n_iter_, (k, a.n_iter_, b.n_iter_)
        assert a.inertia_ == b.inertia_, (k, a.inertia_, b.inertia_)
        np.testing.assert_array_equal(a.cluster_centers_, b.cluster_centers_)
        np.testing.assert_array_equal(a.labels_, b.labels_)


def test_batched_sweep_matches_sequential_sweep(gpu, golden, monkeypatch):
    import milwrm_amd as M

    X = _sweep_rows(golden, "hard256")
    bk1, r1 = M.chooseBestKforKMeansParallel(X, range(2, 21), random_state=18, alpha_k=0.05)
    monkeypatch.setenv("MW_SWEEP_BATCH", "0")
    bk0, r0 = M.chooseBestKforKMeansParallel(X, range(2, 21), random_state=18, alpha_k=0.05)
    assert bk1 == bk0
    np.testing.assert_array_equal(r1["Scaled Inertia"].values, r0["Scaled Inertia"].values)


def _mxif_labeler_from(g, n):
    import milwrm_amd as M

    imgs = [M.img(g["raw"][i].copy(), mask=g["masks"][i].copy()) for i in range(n)]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    names = list(g["batch_names"][:n]) if "batch_names" in g else ["b"] * n
    df = pd.DataFrame({"Img": imgs, "batch_names": names, "mean estimators": list(ests),
                       "pixels": list(pix)})
    return M.mxif_labeler(df)


@pytest.fixture(params=["0", "fused", "band"], ids=["materialised", "fused", "banded"])
def blur_mode(request, monkeypatch):
    """Run a pipeline test with the blurred slide materialised and with the
    blur deferred (MW_FUSED_BLUR=1): into the fused sample / assign epilogues,
    or with the label pass over 40-row bands blurred one at a time; the
    deferred paths must actually have run."""
    from milwrm_amd import device as D

    deferred = request.param != "0"
    monkeypatch.setenv("MW_FUSED_BLUR", "1" if deferred else "0")
    if deferred:
        monkeypatch.setenv("MW_DEFERRED_ASSIGN", request.param)
        monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", "40")
    before = dict(D.FUSED_USED)
    yield request.param
    if deferred:
        assert D.FUSED_USED["sample"] > before["sample"], "fused sample epilogue not taken"
        key = "assign" if request.param == "fused" else "assign_banded"
        assert D.FUSED_USED[key] > before[key], f"deferred label pass ({key}) not taken"


def test_mxif_labeler_end_to_end_small(gpu, golden, blur_mode):
    g = golden("mxif_small")
    lab = _mxif_labeler_from(g, 3)
    lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2)
    np.testing.assert_allclose(lab.scaler.mean_, g["scaler_mean"], rtol=1e-5)
    np.testing.assert_allclose(lab.scaler.scale_, g["scaler_scale"], rtol=1e-5)
    np.testing.assert_allclose(lab.cluster_data, g["cluster_data"], rtol=1e-4, atol=2e-5)
    assert lab.merged_batch_labels == list(g["merged_batch_labels"])
    lab.label_tissue_regions(k=None, alpha=0.05, plot_out=False, random_state=18)
    assert lab.k == int(g["k"])
    assert lab.kmeans.n_iter_ == int(g["n_iter"])
    assert _rel(lab.kmeans.cluster_centers_, g["centers"]) < RTOL
    lab.confidence_score_images()
    for i in range(3):
        cid_ref = g["confidence_IDs"][i]
        _labels_match(lab.tissue_IDs[i], _nan_i8(g["tissue_IDs"][i]), cid_ref)
        ok = ~np.isnan(cid_ref)
        np.testing.assert_array_equal(np.isnan(lab.confidence_IDs[i]), np.isnan(cid_ref))
        np.testing.assert_allclose(lab.confidence_IDs[i][ok], cid_ref[ok], rtol=RTOL, atol=RTOL)
    np.testing.assert_allclose(lab.confidence_score_df.values, g["confidence_score_df"], rtol=RTOL,
                               atol=1e-6)


def test_mxif_labeler_hard256(gpu, golden, blur_mode):
    import milwrm_amd as M

    g = golden("mxif_hard256")
    im = M.img(g["raw"].copy(), mask=g["mask"].copy())
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(30)), sigma=2, fract=0.2)
    assert lab.cluster_data.shape[0] == int(g["n_samples"])
    lab.label_tissue_regions(k=8, plot_out=False, random_state=18)
    assert _rel(lab.kmeans.cluster_centers_, g["centers"]) < RTOL
    assert abs(lab.kmeans.inertia_ - float(g["inertia"])) / float(g["inertia"]) < RTOL
    lab.confidence_score_images()
    _labels_match(lab.tissue_IDs[0], _nan_i8(g["tissue_IDs"]), g["confidence_IDs"].astype(np.float64))
    ok = ~np.isnan(g["confidence_IDs"])
    np.testing.assert_allclose(lab.confidence_IDs[0][ok], g["confidence_IDs"][ok], rtol=RTOL, atol=RTOL)


class _Duck:
    def __init__(self, pcs, adj):
        self.obsm = {"X_pca": pcs}
        self.obsp = {"spatial_connectivities": adj}
        self.obs = pd.DataFrame(index=[str(i) for i in range(pcs.shape[0])])
        self.n_obs = pcs.shape[0]


def test_st_labeler(gpu, golden):
    import scipy.sparse as sp

    import milwrm_amd as M

    g = golden("st_hex")
    ads = []
    for s in range(2):
        n = g[f"pcs{s}"].shape[0]
        A = sp.csr_matrix((np.ones(len(g[f"adj{s}_indices"])), g[f"adj{s}_indices"], g[f"adj{s}_indptr"]),
                          shape=(n, n))
        ads.append(_Duck(g[f"pcs{s}"], A))
    lab = M.st_labeler(ads)
    lab.prep_cluster_data(use_rep="X_pca", n_rings=1, spatial_graph_key="spatial_connectivities")
    np.testing.assert_allclose(lab.cluster_data, g["cluster_data"], rtol=1e-10, atol=1e-12)
    lab.label_tissue_regions(k=None, plot_out=False, random_state=18)
    assert lab.k == int(g["k"])
    np.testing.assert_array_equal(lab.kmeans.labels_, g["labels"])
    assert _rel(lab.kmeans.cluster_centers_, g["centers"]) < RTOL
    lab.confidence_score()
    np.testing.assert_allclose(ads[0].obs["confidence_score"].values, g["conf0"], rtol=RTOL, atol=RTOL)
    np.testing.assert_allclose(lab.confidence_score_df.values, g["confidence_score_df"], rtol=RTOL)


def test_large_properties(gpu):
    """4096^2 x 30 device-generated slide: determinism (bitwise repeat),
    confidence in [0,1], labels = argmin recomputed in fp64 on sampled pixels
    (except near ties), shard-free invariants."""
    from milwrm_amd import device as D
    from milwrm_amd.assign import assign_image

    raw, mask = D.synth_slide(4096, 4096, 30, seed=7, mode="hard")
    mean = np.full(30, 50.0)
    inv = torch.from_numpy((1 / mean).astype(np.float32)).cuda()
    b1 = D.blur(raw, 2.0, inv_mean=inv)
    b2 = D.blur(raw, 2.0, inv_mean=inv)
    assert torch.equal(b1, b2)
    rng = np.random.default_rng(0)
    centers = rng.normal(0, 1, size=(8, 30))
    mu = b1.double().mean(dim=(0, 1)).cpu().numpy()
    sd = b1.double().std(dim=(0, 1)).cpu().numpy()
    lab, conf, dom = assign_image(b1, np.arange(30), mu, 1 / sd, centers, mask)
    lab2, conf2, dom2 = assign_image(b1, np.arange(30), mu, 1 / sd, centers, mask)
    assert torch.equal(lab, lab2) and torch.equal(dom, dom2)
    m = mask.cpu().numpy().astype(bool)
    L = lab.cpu().numpy()
    Cf = conf.cpu().numpy()
    assert np.all(L[~m] == -1) and np.all(np.isnan(Cf[~m]))
    assert np.nanmin(Cf[m]) >= 0 and np.nanmax(Cf[m]) <= 1
    ys = rng.integers(0, 4096, 20000)
    xs = rng.integers(0, 4096, 20000)
    sel = m[ys, xs]
    x = b1[torch.as_tensor(ys), torch.as_tensor(xs)].double().cpu().numpy()[sel]
    xs_ = (x - mu) / sd
    d = ((xs_[:, None, :] - centers[None]) ** 2).sum(-1)
    ref = d.argmin(1)
    srt = np.sort(d, 1)
    cid = (srt[:, 1] - srt[:, 0]) / srt[:, 1]
    _labels_match(L[ys, xs][sel], ref, cid)
    np.testing.assert_allclose(Cf[ys, xs][sel], cid, rtol=RTOL, atol=RTOL)
    # per-domain sums are the sums of the per-pixel outputs: exactly the sum of
    # the fixed-point confidences rint(conf * 2^32), split in two 32-bit limbs
    from milwrm_amd.assign import dom_sums

    dm = dom.cpu().numpy()
    s, cnt = dom_sums(dm, 8)
    for j in range(8):
        sel_j = L == j
        assert cnt[j] == sel_j.sum()
        q = np.rint(Cf[sel_j].astype(np.float64) * 2.0 ** 32).astype(np.uint64).sum(dtype=np.uint64)
        assert dm[j] == float(int(q) >> 32) and dm[8 + j] == float(int(q) & 0xFFFFFFFF)
        np.testing.assert_allclose(s[j], np.nansum(Cf[sel_j].astype(np.float64)), rtol=1e-9)


def test_device_mt19937_subsample_indices_bit_exact(gpu):
    from milwrm_amd.rng import subsample_indices_device

    for M, fr in [(6540, 0.2), (1, 0.9), (2, 0.5), (1000, 0.5), (2**20, 0.01), (2**20 + 1, 0.3),
                  (123457, 0.3), (2**31 - 1, 1e-5), (85_000_000, 0.2)]:
        np.random.seed(16)
        ref = np.random.choice(M, int(M * fr))
        got, tot = subsample_indices_device(M, fr, 16)
        assert int(tot.item()) >= ref.shape[0]
        np.testing.assert_array_equal(got.cpu().numpy(), ref, err_msg=f"M={M}")
    for seed in (0, 18, 2**32 - 1):
        np.random.seed(seed)
        ref = np.random.choice(777_777, 300_000)
        got, _ = subsample_indices_device(777_777, 300_000 / 777_777 + 1e-12, seed)
        np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_global_rng_state_after_subsample(gpu, golden):
    """subsample_pixels leaves NumPy's global RandomState where the
    reference's np.random.seed(16); np.random.choice(M, S) leaves it
    (MxIF.py:484-490), for the golden slide and for a draw spanning many
    generator segments."""
    import milwrm_amd as M
    from milwrm_amd.rng import set_global_state_after_draws, subsample_indices_device

    def same(a, b):
        return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2]

    g = golden("mxif_small")
    im = M.img(g["raw"][0].copy(), mask=g["masks"][0].copy())
    im.log_normalize(mean=g["batch_mean_b1"])
    im.blurring("gaussian", sigma=2)
    np.random.seed(123)
    im.subsample_pixels(list(range(8)), 0.2)
    got = np.random.get_state()
    Mpx = int((g["masks"][0] != 0).sum())
    np.random.seed(16)
    np.random.choice(Mpx, int(Mpx * 0.2))
    assert same(got, np.random.get_state())
    for Mpx, fr in [(85_000_000, 0.2), (2**20 + 1, 0.3), (1000, 0.5)]:
        np.random.seed(5)
        idx, tot = subsample_indices_device(Mpx, fr, 16)
        assert int(tot.item()) >= int(Mpx * fr)
        set_global_state_after_draws()
        got = np.random.get_state()
        np.random.seed(16)
        np.random.choice(Mpx, int(Mpx * fr))
        assert same(got, np.random.get_state()), Mpx


def _same_bits(a, b):
    return bool(torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8)))


@pytest.mark.parametrize("H,W,C,k,feats", [
    (300, 260, 30, 8, None), (130, 64, 30, 16, None), (190, 210, 30, 8, [3, 1, 4, 15, 9, 2, 6]),
    (200, 200, 16, 8, None), (160, 96, 64, 12, None), (1031, 778, 30, 8, None),
    (150, 130, 50, 8, None), (120, 100, 45, 6, list(range(44, 4, -1)))])
def test_fused_epilogues_match_materialised(gpu, H, W, C, k, feats):
    """Blur with the sample / assign epilogue (blurred slide never stored) is
    bit-identical to blur → gather and blur → assign: same X rows, column
    statistics, labels, confidences and per-domain sums.  Parity of the
    materialised path itself with the oracle is pinned by the tests above."""
    from milwrm_amd import device as D
    from milwrm_amd.assign import assign_image, blur_assign_image

    raw, mask = D.synth_slide(H, W, C, seed=7, mode="hard")
    mask = D.padded_mask(mask)
    s, c = D.nz_stats(raw)
    inv = (c.double() / s).float()
    blurred = D.blur(raw, 2.0, inv_mean=inv)
    r2p, M = D.mask_rank(mask.reshape(-1))
    S = int(0.2 * M)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    idx = torch.randint(0, M, (S,), device="cuda", generator=g, dtype=torch.int32)
    feats = list(range(C)) if feats is None else feats
    F = len(feats)
    feat = torch.tensor(feats, dtype=torch.int32, device="cuda")
    X0 = torch.empty((S, F), dtype=torch.float32, device="cuda")
    st0 = torch.zeros(2 * F + 1, dtype=torch.float64, device="cuda")
    D.gather_rows(blurred, feat, idx, r2p, X0, st0, False)
    X1 = torch.full((S, F), float("nan"), dtype=torch.float32, device="cuda")
    assert D.blur_gather_fused(raw, 2.0, inv, 1.0, feat, idx, r2p, X1)
    st1 = torch.zeros(2 * F + 1, dtype=torch.float64, device="cuda")
    D.col_stats_rows(X1, st1, False)
    assert _same_bits(X0, X1)
    assert _same_bits(st0, st1)
    if feats != list(range(C)):
        return
    mu = st0[1:1 + F].cpu().numpy()
    invs = 1.0 / np.sqrt(st0[1 + F:].cpu().numpy() / st0[0].item())
    rows = X0[torch.arange(0, S, max(1, S // k), device="cuda")[:k]].double().cpu().numpy()
    centers = (rows - mu) * invs
    l0, c0, d0 = assign_image(blurred, feats, mu, invs, centers, mask)
    out = blur_assign_image(raw, 2.0, inv, 1.0, mu, invs, centers, mask)
    assert out is not None
    l1, c1, d1 = out
    assert _same_bits(l0, l1) and _same_bits(c0, c1) and _same_bits(d0, d1)


class _Scaler:
    def __init__(self, mean, scale):
        self.mean_, self.scale_ = mean, scale

    def affine(self):
        return self.mean_.copy(), 1.0 / self.scale_


@pytest.mark.parametrize("H,W,C,k,feats", [(64, 48, 8, 5, None), (97, 131, 30, 8, [0, 3, 5, 7, 11, 29]),
                                           (33, 17, 12, 20, [2, -1])])
def test_qc_estimators(gpu, H, W, C, k, feats):
    """estimate_percentage_variance_mxif / estimate_mse_mxif (MILWRM.py:280-333,
    453-515) through mw_domain_sse against the oracle's restatement: masked
    (NaN) pixels, an empty domain, a feature subset and k at the kernel's limit.
    fp64 sums over fp32 pixels: rtol 1e-8."""
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW

    rng = np.random.default_rng(H * W + C)
    fidx = list(range(C)) if feats is None else [f % C for f in feats]
    F = len(fidx)
    arrs, tids = [], []
    mean = rng.random(F) * 1.5
    scale = 0.5 + rng.random(F)
    centers = rng.standard_normal((k, F))
    for j in range(2):
        arr = (rng.random((H, W, C)) * 3).astype(np.float32)
        mask = (rng.random((H, W)) > 0.2).astype(np.uint8)
        tid = O.tissue_ids(arr, mask, fidx, centers, mean, scale)
        tid[tid == 1] = 0  # domain 1 empty: MSE row of zeros
        arrs.append(arr)
        tids.append(tid)
    ims = [M.img(a.copy(), mask=np.ones((H, W), dtype=np.uint8)) for a in arrs]
    sc = _Scaler(mean, scale)
    for im, a, t in zip(ims, arrs, tids):
        got = MW.estimate_percentage_variance_mxif(im, False, sc, centers, feats, t)
        ref = O.percentage_variance_mxif(a, fidx, centers, mean, scale, t)
        assert abs(got - ref) <= 1e-8 * abs(ref), (got, ref)
    got = MW.estimate_mse_mxif(ims, False, tids, sc, centers, feats, k)
    ref = O.mse_mxif(arrs, tids, fidx, centers, mean, scale, k)
    assert sorted(got) == sorted(ref) == list(range(k))
    for i in range(k):
        for g_, r_ in zip(got[i], ref[i]):
            np.testing.assert_allclose(g_, r_, rtol=1e-8, atol=1e-12)
    assert all(np.all(v == 0) for v in got[1])


def test_st_labeler_k8(gpu, golden):
    """Config 1 at its own k (BASELINE.json: st_labeler, k = 8) against the
    reference run at k = 8 on the st_hex sections (st_hex_k8.npz)."""
    import scipy.sparse as sp

    import milwrm_amd as M

    g, g8 = golden("st_hex"), golden("st_hex_k8")
    np.testing.assert_array_equal(g8["pcs0"], g["pcs0"])  # same inputs
    ads = []
    for s in range(2):
        n = g[f"pcs{s}"].shape[0]
        A = sp.csr_matrix((np.ones(len(g[f"adj{s}_indices"])), g[f"adj{s}_indices"], g[f"adj{s}_indptr"]),
                          shape=(n, n))
        ads.append(_Duck(g[f"pcs{s}"], A))
    lab = M.st_labeler(ads)
    lab.prep_cluster_data(use_rep="X_pca", n_rings=1, spatial_graph_key="spatial_connectivities")
    lab.label_tissue_regions(k=8, plot_out=False, random_state=18)
    assert lab.kmeans.n_iter_ == int(g8["n_iter"])
    np.testing.assert_array_equal(lab.kmeans.labels_, g8["labels"])
    assert _rel(lab.kmeans.cluster_centers_, g8["centers"]) < RTOL
    assert abs(lab.kmeans.inertia_ - float(g8["inertia"])) / float(g8["inertia"]) < RTOL
    np.testing.assert_array_equal(np.asarray(ads[1].obs["tissue_ID"].astype(int)), g8["tissue_ID1"])
    lab.confidence_score()
    for s in range(2):
        np.testing.assert_allclose(ads[s].obs["confidence_score"].values, g8[f"conf{s}"], rtol=RTOL,
                                   atol=RTOL)
    np.testing.assert_allclose(lab.confidence_score_df.values, g8["confidence_score_df"], rtol=RTOL)


@pytest.mark.parametrize("n,density", [(64, 1.0), (65, 0.5), (4097, 0.85), (100_003, 0.01), (262_144, 1.0),
                                       (1_000_000, 0.85)])
def test_rank_index_gather_equals_table(gpu, n, density):
    """The compact rank index (mw_mask_rank_index: per 64-pixel word its mask
    bits and prefix, per 64 ranks a word) maps every draw to the pixel the
    rank -> pixel table gives: rows, column statistics and the sample slots
    bitwise equal; partial last words, empty words, M a multiple of 64."""
    import torch

    from milwrm_amd import _native as N
    from milwrm_amd import device as D
    from milwrm_amd.rng import subsample_indices_device

    rs = np.random.RandomState(n)
    C = 6
    mask = (rs.random_sample(n) < density).astype(np.uint8)
    if n == 4097:
        mask[128:640] = 0  # whole empty words
    img = torch.from_numpy(rs.random_sample((n, 1, C)).astype(np.float32)).cuda()
    m = D.padded_mask(torch.from_numpy(mask).cuda())
    M = int(mask.sum())
    cnt = torch.empty(1, dtype=torch.int64, device="cuda")
    ws = D.WS.get("mrank", N.query("mw_mask_rank_ws_bytes", n))
    r2p = torch.empty(n, dtype=torch.int32, device="cuda")
    N.call("mw_mask_rank", D.P(m), n, D.P(r2p), D.P(cnt), D.P(ws), D.stream())
    assert int(cnt.item()) == M
    ix = torch.empty(N.query("mw_rank_index_bytes", n), dtype=torch.uint8, device="cuda")
    N.call("mw_mask_rank_index", D.P(m), n, D.P(ix), D.P(cnt), D.P(ws), D.stream())
    assert int(cnt.item()) == M
    ri = D.RankIndex(ix, n)
    np.random.seed(16)
    idx, _ = subsample_indices_device(M, 0.9, 16, torch.device("cuda"))
    S = int(idx.shape[0])
    feat = torch.arange(C, dtype=torch.int32, device="cuda")
    out = []
    for table in (r2p, ri):
        X = torch.empty((S, C), dtype=torch.float32, device="cuda")
        st = torch.zeros(1 + 2 * C, dtype=torch.float64, device="cuda")
        D.gather_rows(img, feat, idx, table, X, st, accumulate=False)
        out.append((X.cpu().numpy(), st.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    np.testing.assert_array_equal(out[1][0], img.reshape(n, C).cpu().numpy()[np.nonzero(mask)[0][idx.cpu().numpy()]])
