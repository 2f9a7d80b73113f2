"""BASELINE configs 2 and 5 at full size, pinned by size-independent checks.

The oracle cannot run the whole 10k^2 or 40k^2 pipeline in a test, so each
stage is checked against an fp64 recompute of exactly what it claims:

* scaler: mean / ddof-0 variance of the gathered rows, recomputed in fp64;
* k-means++ (config 2): the oracle's sklearn restatement (_kmeans.py:174-272,
  GEMM-form fp64 distances, sequential cumsum) run on the full 1.7e7 x 30
  scaled and centered rows on the host: identical indices;
* the fit: inertia recomputed in fp64 from the rows, labels and centers; every
  row's fit label the fp64 argmin under the final centers except near-ties;
* the label + confidence pass: 1e5 sampled pixels (masked and background),
  their log-normalised + Gaussian-blurred features recomputed in fp64 from
  the raw slide (17 x 17 patches, edge-replicated: scipy's mode='nearest'),
  scaled by the fitted scaler; labels equal the fp64 argmin except near-ties
  (relative top-2 gap < TAU), confidences within 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu
TAU = 1e-5
RTOL = 1e-4


def _run(size, C, k, seed):
    import pandas as pd

    import milwrm_amd as M
    from milwrm_amd import device as D

    raw, mask = D.synth_slide(size, size, C, seed=seed, mode="hard")
    im = M.img.from_device(raw, mask)
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=k, plot_out=False, random_state=18)
    lab.confidence_score_images()
    mean = np.asarray(est, dtype=np.float64) / pix
    return raw, mask, lab, mean


def _chunks(n, step):
    for a in range(0, n, step):
        yield a, min(n, a + step)


def _check_scaler_fit(lab, k, step=1_000_000):
    """Scaler, inertia and fit labels against fp64 recomputes over the rows."""
    rows = lab._rows
    S, F = rows.S, rows.F
    dev = rows.X.device
    s1 = torch.zeros(F, dtype=torch.float64, device=dev)
    for a, b in _chunks(S, step):
        s1 += rows.X[a:b].double().sum(0)
    mu = s1 / S
    s2 = torch.zeros(F, dtype=torch.float64, device=dev)
    for a, b in _chunks(S, step):
        s2 += ((rows.X[a:b].double() - mu) ** 2).sum(0)
    var = (s2 / S).cpu().numpy()
    np.testing.assert_allclose(lab.scaler.mean_, mu.cpu().numpy(), rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(lab.scaler.var_, var, rtol=1e-9)
    km = lab.kmeans
    smu = torch.from_numpy(lab.scaler.mean_).to(dev)
    sinv = torch.from_numpy(1.0 / lab.scaler.scale_).to(dev)
    C = torch.from_numpy(km.cluster_centers_).to(dev)
    labels = km._labels_dev.long()
    inertia = 0.0
    bad = 0
    for a, b in _chunks(S, step):
        xs = (rows.X[a:b].double() - smu) * sinv
        inertia += float(((xs - C[labels[a:b]]) ** 2).sum())
        d = ((xs[:, None, :] - C[None]) ** 2).sum(-1)
        top = torch.topk(d, 2, dim=1, largest=False).values
        gap = (top[:, 1] - top[:, 0]) / top[:, 1]
        bad += int(((d.argmin(1) != labels[a:b]) & ~(gap < TAU)).sum())
    assert abs(km.inertia_ - inertia) <= 1e-6 * inertia, (km.inertia_, inertia)
    assert bad == 0, f"{bad} fit labels differ from the fp64 argmin outside near-ties"
    return smu, sinv


def _blur64_at(raw, mean, ys, xs, sigma=2.0):
    """fp64 log10(x/mean + 1) then the scipy Gaussian (taps of the oracle,
    mode='nearest') evaluated at pixels (ys, xs): n x C."""
    H, W, _ = raw.shape
    w = torch.from_numpy(O.gaussian_kernel1d(sigma)).to(raw.device)
    r = (w.numel() - 1) // 2
    off = torch.arange(-r, r + 1, device=raw.device)
    yy = (ys[:, None] + off[None]).clamp(0, H - 1)
    xx = (xs[:, None] + off[None]).clamp(0, W - 1)
    p = raw[yy[:, :, None], xx[:, None, :]]  # n x (2r+1) x (2r+1) x C, int16 bits of uint16
    p = (p.to(torch.int32) & 0xFFFF).double() if p.dtype == torch.int16 else p.double()
    inv = torch.from_numpy(1.0 / mean).to(raw.device)
    p = torch.log10(p * inv + 1.0)
    # correlate1d(weights[::-1]) == convolution with w: taps symmetric
    v = (p * w[None, :, None, None]).sum(1)
    return (v * w[None, :, None]).sum(1)


def _check_label_pass(raw, mask, lab, mean, smu, sinv, n=100_000, seed=0, step=5_000):
    dev = raw.device
    H, W, C = raw.shape
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    ys = torch.randint(0, H, (n,), generator=g).to(dev)
    xs = torch.randint(0, W, (n,), generator=g).to(dev)
    cen = torch.from_numpy(lab.kmeans.cluster_centers_).to(dev)
    L = lab._labels_dev[0]
    Cf = lab._conf_dev[0]
    m = mask[ys, xs] != 0
    assert bool((L[ys, xs][~m] == -1).all()) and bool(torch.isnan(Cf[ys, xs][~m]).all())
    bad = 0
    worst = 0.0
    for a, b in _chunks(n, step):
        sel = m[a:b]
        yb, xb = ys[a:b][sel], xs[a:b][sel]
        f = (_blur64_at(raw, mean, yb, xb) - smu) * sinv
        d = ((f[:, None, :] - cen[None]) ** 2).sum(-1)
        srt = torch.sort(d, dim=1).values
        cid = (srt[:, 1] - srt[:, 0]) / srt[:, 1]
        got = L[yb, xb].long()
        bad += int(((got != d.argmin(1)) & ~(cid < TAU)).sum())
        gc = Cf[yb, xb].double()
        worst = max(worst, float(((gc - cid).abs() / torch.clamp(cid.abs(), min=1.0)).max()))
    assert bad == 0, f"{bad} sampled pixel labels differ from the fp64 argmin outside near-ties"
    assert worst < RTOL, worst


def _label_sums(labels, xs, k):
    """Per-label fp64 sums of the rows (a one-hot GEMM: no atomics)."""
    onehot = torch.nn.functional.one_hot(labels, k).double()
    return onehot.T @ xs


def _lloyd64(lab, smu, sinv, step=2_000_000):
    """Test infrastructure: sklearn's ``_kmeans_single_lloyd`` (_kmeans.py:
    624-752, as oracle.lloyd) in fp64 torch on the device, from the fit's own
    k-means++ indices over the same fp32 rows (direct-difference distances,
    lowest index wins ties, strict label convergence or the center-shift
    tolerance, the extra E-step when not strict).  Returns (labels int64,
    centers fp64, n_iter, strict, gap) with gap = the relative top-2 distance
    gap of every row under the final centers."""
    rows = lab._rows
    S, F = rows.S, rows.F
    km = lab.kmeans
    k = km.cluster_centers_.shape[0]
    dev = rows.X.device
    idx = torch.from_numpy(np.asarray(km.init_indices_, dtype=np.int64)).to(dev)
    centers = (rows.X.index_select(0, idx).double() - smu) * sinv
    tol = float(np.mean(lab.scaler.var_ / lab.scaler.scale_ ** 2)) * km.tol
    labels_old = torch.full((S,), -1, dtype=torch.int64, device=dev)

    def estep(C, want_gap=False):
        lab_ = torch.empty(S, dtype=torch.int64, device=dev)
        gap = torch.empty(S, dtype=torch.float64, device=dev) if want_gap else None
        sums = torch.zeros((k, F), dtype=torch.float64, device=dev)
        for a, b in _chunks(S, step):
            xs = (rows.X[a:b].double() - smu) * sinv
            d = torch.stack([((xs - C[j]) ** 2).sum(1) for j in range(k)], 1)
            lab_[a:b] = d.argmin(1)
            if want_gap:
                top = torch.topk(d, 2, dim=1, largest=False).values
                gap[a:b] = (top[:, 1] - top[:, 0]) / top[:, 1]
            sums += _label_sums(lab_[a:b], xs, k)
        cnt = torch.bincount(lab_, minlength=k).double()
        return lab_, sums, cnt, gap

    strict = False
    for it in range(km.max_iter):
        print(f"fp64 Lloyd iteration {it}", flush=True)
        labels, sums, cnt, _ = estep(centers)
        assert bool((cnt > 0).all()), "empty cluster: relocation is outside this check"
        new = sums / cnt[:, None]
        shift = float(((new - centers) ** 2).sum())
        centers = new
        if torch.equal(labels, labels_old):
            strict = True
            break
        if shift <= tol:
            break
        labels_old = labels
    labels, _, _, gap = estep(centers, want_gap=True)
    return labels, centers, it + 1, strict, gap


def _check_mstep(lab, smu, sinv):
    """The fit against the fp64 Lloyd from the same k-means++ indices: the same
    n_iter, labels equal outside near-ties, centers within 1e-4."""
    km = lab.kmeans
    labels, centers, n_iter, strict, gap = _lloyd64(lab, smu, sinv)
    assert n_iter == km.n_iter_, (n_iter, km.n_iter_, strict)
    diff = (labels != km._labels_dev.long()) & ~(gap < TAU)
    assert int(diff.sum()) == 0, f"{int(diff.sum())} fit labels differ from the fp64 Lloyd outside near-ties"
    c = centers.cpu().numpy()
    scale = np.abs(c).max()
    np.testing.assert_allclose(km.cluster_centers_, c, rtol=1e-4, atol=1e-4 * scale)


def _check_centers_are_means(lab, smu, sinv, step=2_000_000):
    """At the Lloyd fixed point the centers are the per-label means of the
    scaled rows: within 1e-4 (strict convergence), else within the fit's
    center-shift tolerance."""
    rows = lab._rows
    S, F = rows.S, rows.F
    km = lab.kmeans
    k = km.cluster_centers_.shape[0]
    labels = km._labels_dev.long()
    sums = torch.zeros((k, F), dtype=torch.float64, device=rows.X.device)
    for a, b in _chunks(S, step):
        sums += _label_sums(labels[a:b], (rows.X[a:b].double() - smu) * sinv, k)
    cnt = torch.bincount(labels, minlength=k).double()
    means = (sums / cnt[:, None]).cpu().numpy()
    c = km.cluster_centers_
    if np.abs(c - means).max() <= 1e-4 * np.abs(means).max():
        return
    tol = float(np.mean(lab.scaler.var_ / lab.scaler.scale_ ** 2)) * km.tol
    assert ((c - means) ** 2).sum() <= tol, (np.abs(c - means).max(), tol)


@pytest.mark.timeout(900)
def test_config2_full_size(gpu):
    """Config 2: one 10k x 10k x 30 hard slide, k = 8 (the bench workload)."""
    raw, mask, lab, mean = _run(10_000, 30, 8, 20251015)
    smu, sinv = _check_scaler_fit(lab, 8)
    _check_mstep(lab, smu, sinv)
    _check_centers_are_means(lab, smu, sinv)
    # k-means++ at the bench's size: the oracle on the full row set
    rows = lab._rows
    Xs = ((rows.X.double() - smu) * sinv).cpu().numpy()
    Xs -= Xs.mean(axis=0)  # KMeans.fit centers X before seeding (_kmeans.py:1477-1481)
    _, idx = O.kmeans_plusplus(Xs, 8, np.random.RandomState(18))
    del Xs
    np.testing.assert_array_equal(lab.kmeans.init_indices_, idx)
    _check_label_pass(raw, mask, lab, mean, smu, sinv)


@pytest.mark.timeout(900)
def test_config5_slide_full_size(gpu):
    """Config 5's slide: 40k x 40k x 50 (deferred blur: fused sample epilogue
    and banded label pass), k = 8."""
    from milwrm_amd import device as D

    D.WS.clear()  # earlier tests' scratch and torch's cache: this slide needs most of the HBM
    torch.cuda.empty_cache()
    used = dict(D.FUSED_USED)
    raw, mask, lab, mean = _run(40_000, 50, 8, 20251016)
    assert D.FUSED_USED["sample"] > used["sample"]  # the 320 GB fp32 slide was never stored
    smu, sinv = _check_scaler_fit(lab, 8)
    _check_centers_are_means(lab, smu, sinv)
    from milwrm_amd.rng import first_center_index, kpp_draws

    u0, _ = kpp_draws(18, 8, 2 + int(np.log(8)))
    assert int(lab.kmeans.init_indices_[0]) == first_center_index(lab._rows.S, u0)
    _check_label_pass(raw, mask, lab, mean, smu, sinv, step=2_000)
