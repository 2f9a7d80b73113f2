"""Slide residency and streaming (milwrm_amd.stream; SURVEY §7 step 8,
BASELINE config 5: more slides per GPU than HBM holds).

* An HBM budget cap (``MW_HBM_BUDGET``) forces every host-backed slide to be
  streamed in row bands (non-zero statistics, blur + subsample epilogue over
  output-row windows, banded blur + label pass, QC sums); the results must be
  BITWISE those of the resident run: scaler, k-means++ indices, n_iter,
  centers, inertia, every row label, every pixel's label and confidence, the
  confidence frame, the QC estimators.  Shapes cover the matrix-core
  epilogues (C = 8, 50) and the slot-gather fallback (odd C), odd band sizes.
* A budget that holds one slide at a time: the LRU evicts, results unchanged.
* The synthetic source's bands are bit for bit the whole generated slide.
* Two 40k x 40k x 50 slides on one GPU (config 5's two slides per GPU of an
  8-GPU node), streamed from the device generator: property checks as
  tests/test_gpu_fullsize.py (scaler, first k-means++ index, fit labels and
  inertia against fp64 recomputes, sampled pixels' labels / confidences
  against an fp64 blur of regenerated raw rows).
"""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu
TAU = 1e-5


def _slides(C, n=3, seed=900, dtype=np.uint16):
    out = []
    for i in range(n):
        raw, mask = O.synth_slide(150 + 17 * i, 176 + 32 * i, C, seed=seed + i, mode="hard")
        out.append((np.minimum(raw, 255).astype(dtype) if dtype != np.uint16 else raw, mask))
    return out


def _pipeline(slides, k=5, qc=True):
    import milwrm_amd as M
    from milwrm_amd.MILWRM import estimate_mse_mxif, estimate_percentage_variance_mxif

    C = slides[0][0].shape[2]
    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in slides]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b1", "b1", "b2"][:len(imgs)],
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=k, plot_out=False, random_state=18)
    lab.confidence_score_images()
    out = dict(est=np.asarray(ests), pix=np.asarray(pix), mean=lab.scaler.mean_,
               scale=lab.scaler.scale_, idx=lab.kmeans.init_indices_, n_iter=lab.kmeans.n_iter_,
               centers=lab.kmeans.cluster_centers_, inertia=lab.kmeans.inertia_,
               rows=lab.kmeans.labels_, conf_df=lab.confidence_score_df.values,
               tid=[np.nan_to_num(t, nan=-1) for t in lab.tissue_IDs],
               cid=[np.nan_to_num(c, nan=-1) for c in lab.confidence_IDs],
               dom=[d.cpu().numpy() for d in lab._dom_dev],
               np_state=np.random.get_state()[1].copy())
    if qc:
        feats = list(range(C))
        out["pv"] = [estimate_percentage_variance_mxif(im, False, lab.scaler, lab.kmeans.cluster_centers_,
                                                       feats, t) for im, t in zip(imgs, lab.tissue_IDs)]
        mse = estimate_mse_mxif(imgs, False, list(lab.tissue_IDs), lab.scaler, lab.kmeans.cluster_centers_,
                                feats, k)
        out["mse"] = np.array([mse[i] for i in range(k)])
    out["resident"] = [im._dev is not None for im in imgs]
    return out


def _assert_same(a, b):
    for key in ("est", "pix", "mean", "scale", "idx", "centers", "rows", "conf_df", "np_state"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
    assert a["n_iter"] == b["n_iter"]
    assert a["inertia"] == b["inertia"]
    for x, y in zip(a["tid"], b["tid"]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a["cid"], b["cid"]):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(a["dom"], b["dom"]):  # exact domain records: any band split
        np.testing.assert_array_equal(x, y)
    if "pv" in a:
        np.testing.assert_array_equal(a["pv"], b["pv"])
        np.testing.assert_array_equal(a["mse"], b["mse"])


@pytest.mark.parametrize("C,dtype,band,rank", [(8, np.uint16, "37", "table"), (8, np.uint16, "37", "index"),
                                               (50, np.uint16, "61", "index"), (7, np.uint16, "29", "table"),
                                               (8, np.uint8, "200", "index")])
def test_streamed_equals_resident(gpu, monkeypatch, C, dtype, band, rank):
    """Streamed == resident, bitwise; the streamed run draws through the rank
    table or the compact rank index (the resident one through the table)."""
    from milwrm_amd import device as D

    slides = _slides(C, dtype=dtype)
    monkeypatch.delenv("MW_HBM_BUDGET", raising=False)
    monkeypatch.setattr(D, "RANK_TABLE_MAX_PIX", 1 << 62)
    ref = _pipeline(slides)
    assert all(ref["resident"])
    monkeypatch.setattr(D, "RANK_TABLE_MAX_PIX", 1 << 62 if rank == "table" else 0)
    monkeypatch.setenv("MW_HBM_BUDGET", "1")       # nothing may stay resident: every pass streams
    monkeypatch.setenv("MW_STREAM_BAND_ROWS", band)
    before = dict(D.FUSED_USED)
    got = _pipeline(slides)
    assert not any(got["resident"])
    for key in ("nz_streamed", "sample_streamed", "assign_streamed"):
        assert D.FUSED_USED[key] > before[key], key
    _assert_same(got, ref)


def test_fused_assign_streamed(gpu, monkeypatch):
    """The fused blur + label epilogue over streamed bands (mw_blur_assign_rows)
    gives the banded path's bits."""
    from milwrm_amd import device as D

    slides = _slides(8)
    monkeypatch.setenv("MW_HBM_BUDGET", "1")
    monkeypatch.setenv("MW_STREAM_BAND_ROWS", "45")
    ref = _pipeline(slides, qc=False)
    monkeypatch.setenv("MW_DEFERRED_ASSIGN", "fused")
    before = dict(D.FUSED_USED)
    got = _pipeline(slides, qc=False)
    assert D.FUSED_USED["assign"] > before["assign"]
    _assert_same(got, ref)


def test_lru_eviction(gpu, monkeypatch):
    """A budget that holds about one slide: uploads evict the least recently
    used copy (host arrays stay), the fit releases what it needs; the results
    do not change."""
    from milwrm_amd.stream import RESIDENCY

    slides = _slides(8)
    ref = _pipeline(slides)
    one = max(r.shape[0] * r.shape[1] * r.shape[2] * 4 for r, _ in slides)  # an fp32 blurred copy
    monkeypatch.setenv("MW_HBM_BUDGET", str(int(one * 1.2)))
    ev = RESIDENCY.evictions
    got = _pipeline(slides)
    assert RESIDENCY.evictions > ev
    assert RESIDENCY.used() <= one * 1.2
    _assert_same(got, ref)


def test_synth_source_bands_bitwise(gpu):
    from milwrm_amd import device as D
    from milwrm_amd import stream

    H, W, C = 301, 208, 50
    raw, mask = D.synth_slide(H, W, C, seed=77)
    src = stream.SynthSource(H, W, C, 77)
    whole = src.materialize()
    assert torch.equal(whole, raw)
    assert torch.equal(src.mask_device(), mask)
    got = torch.empty_like(raw)
    for y0, y1, a, rb in stream.bands(src, 23, 8):
        got[a:a + rb.shape[0]] = rb
    assert torch.equal(got, raw)


@pytest.mark.parametrize("second", ["granted", "oom"])
def test_bands_shrunk_buffer_no_overlap(gpu, monkeypatch, second):
    """HBM short on the first band buffer (stream.alloc_rows handing back fewer
    rows than a one-band plan asked for): the plan becomes several bands, and
    the reads must not overwrite a band before its consumer is done -- with a
    second buffer (granted) or, when that allocation fails, with one buffer
    whose next read waits for the band before it.  Every band, and the
    non-zero statistics, equal the resident slide bit for bit."""
    from milwrm_amd import device as D
    from milwrm_amd import stream

    H, W, C = 301, 208, 8
    raw, _ = D.synth_slide(H, W, C, seed=78)
    src = stream.SynthSource(H, W, C, 78)
    real = stream.alloc_rows
    calls = []

    def short(rows, row_shape, dtype, min_rows=1, dev=None):
        calls.append(rows)
        if len(calls) == 1:
            return real(40, row_shape, dtype, min_rows=1, dev=dev)  # "halved" twice and more
        if second == "oom":
            raise torch.OutOfMemoryError("test: no second buffer")
        return real(rows, row_shape, dtype, min_rows=min_rows, dev=dev)

    monkeypatch.setattr(stream, "alloc_rows", short)
    got = torch.zeros_like(raw)
    n = 0
    for y0, y1, a, rb in stream.bands(src, H, 8):
        # slow consumer on the main stream: a read racing ahead would land here
        acc = rb.to(torch.float32)
        for _ in range(20):
            acc = acc * 1.0
        got[y0:y1] = acc[y0 - a:y1 - a].to(raw.dtype)
        n += 1
    assert n > 1 and len(calls) == 2
    assert torch.equal(got, raw)
    monkeypatch.setenv("MW_STREAM_BAND_ROWS", str(H))
    calls.clear()
    s1, c1 = stream.nz_stats(src)
    assert len(calls) == 2
    s0, c0 = D.nz_stats(raw)
    assert torch.equal(s1, s0) and torch.equal(c1, c0)


# ------------------------------------------------- two config-5 slides / GPU

def _chunks(n, step):
    for a in range(0, n, step):
        yield a, min(n, a + step)


def _blur64_rows(src, mean, ys, xs, sigma=2.0):
    """fp64 log10(x/mean + 1) + the scipy Gaussian (mode='nearest') at pixels
    (ys, xs), from raw rows the source regenerates."""
    H, W, C = src.shape
    w = torch.from_numpy(O.gaussian_kernel1d(sigma)).cuda()
    r = (w.numel() - 1) // 2
    y0, y1 = max(0, int(ys.min()) - r), min(H, int(ys.max()) + r + 1)
    rows = torch.empty((y1 - y0, W, C), dtype=src.dtype, device="cuda")
    src.read(y0, y1, rows)
    off = torch.arange(-r, r + 1, device="cuda")
    yy = (ys[:, None] + off[None]).clamp(0, H - 1) - y0
    xx = (xs[:, None] + off[None]).clamp(0, W - 1)
    p = rows[yy[:, :, None], xx[:, None, :]]
    p = (p.to(torch.int32) & 0xFFFF).double()
    inv = torch.from_numpy(1.0 / mean).cuda()
    p = torch.log10(p * inv + 1.0)
    v = (p * w[None, :, None, None]).sum(1)
    return (v * w[None, :, None]).sum(1)


def _config5_slides_streamed(n_slides):
    """``n_slides`` 40k x 40k x 50 slides on one GPU (160 GB of uint16 each:
    at most one could be resident), streamed band by band from the device
    generator, k = 8, with the full-size property checks."""
    import milwrm_amd as M
    from milwrm_amd import device as D
    from milwrm_amd import stream
    from milwrm_amd.rng import first_center_index, kpp_draws

    D.WS.clear()
    torch.cuda.empty_cache()
    H = W = 40_000
    C = 50
    srcs = [stream.SynthSource(H, W, C, 20251016 + i) for i in range(n_slides)]
    imgs = [M.img.from_source(s) for s in srcs]
    before = dict(D.FUSED_USED)
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b"] * n_slides, "mean estimators": list(ests),
                       "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=8, plot_out=False, random_state=18)
    lab.confidence_score_images()
    assert all(im._dev is None for im in imgs)  # never resident
    for key in ("nz_streamed", "sample_streamed", "assign_streamed"):
        assert D.FUSED_USED[key] >= before[key] + n_slides, key
    mean = np.sum([np.asarray(e) for e in ests], axis=0) / np.sum(pix)
    # scaler against an fp64 recompute of the gathered rows
    rows = lab._rows
    S, F = rows.S, rows.F
    assert S == sum(lab._batch_counts)
    step = 2_000_000
    s1 = torch.zeros(F, dtype=torch.float64, device="cuda")
    for a, b in _chunks(S, step):
        s1 += rows.X[a:b].double().sum(0)
    mu = s1 / S
    s2 = torch.zeros(F, dtype=torch.float64, device="cuda")
    for a, b in _chunks(S, step):
        s2 += ((rows.X[a:b].double() - mu) ** 2).sum(0)
    np.testing.assert_allclose(lab.scaler.mean_, mu.cpu().numpy(), rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(lab.scaler.var_, (s2 / S).cpu().numpy(), rtol=1e-9)
    # first k-means++ center (sklearn's sequential cumsum of 1/n, rng.first_center_index)
    u0, _ = kpp_draws(18, 8, 2 + int(np.log(8)))
    assert int(lab.kmeans.init_indices_[0]) == first_center_index(S, u0)
    # fit labels = fp64 argmin under the final centers (near-ties aside), inertia
    km = lab.kmeans
    smu = torch.from_numpy(lab.scaler.mean_).cuda()
    sinv = torch.from_numpy(1.0 / lab.scaler.scale_).cuda()
    Cn = torch.from_numpy(km.cluster_centers_).cuda()
    labels = km._labels_dev.long()
    inertia, bad = 0.0, 0
    for a, b in _chunks(S, step):
        xs = (rows.X[a:b].double() - smu) * sinv
        inertia += float(((xs - Cn[labels[a:b]]) ** 2).sum())
        d = ((xs[:, None, :] - Cn[None]) ** 2).sum(-1)
        top = torch.topk(d, 2, dim=1, largest=False).values
        gap = (top[:, 1] - top[:, 0]) / top[:, 1]
        bad += int(((d.argmin(1) != labels[a:b]) & ~(gap < TAU)).sum())
    assert abs(km.inertia_ - inertia) <= 1e-6 * inertia, (km.inertia_, inertia)
    assert bad == 0
    # label pass: sampled pixels in a few row windows (top edge, interior, bottom edge)
    g = torch.Generator().manual_seed(5)
    for s, (src, im) in enumerate(zip(srcs, imgs)):
        L, Cf = lab._labels_dev[s], lab._conf_dev[s]
        mask = src.mask_device()
        nbad, worst = 0, 0.0
        for wy in (0, 5_003, 19_990, 39_800):
            ys = torch.randint(wy, min(H, wy + 200), (4000,), generator=g).cuda()
            xs = torch.randint(0, W, (4000,), generator=g).cuda()
            m = mask[ys, xs] != 0
            assert bool((L[ys, xs][~m] == -1).all()) and bool(torch.isnan(Cf[ys, xs][~m]).all())
            yb, xb = ys[m], xs[m]
            if yb.numel() == 0:
                continue
            f = (_blur64_rows(src, mean, yb, xb) - smu) * sinv
            d = ((f[:, None, :] - Cn[None]) ** 2).sum(-1)
            srt = torch.sort(d, dim=1).values
            cid = (srt[:, 1] - srt[:, 0]) / srt[:, 1]
            nbad += int(((L[yb, xb].long() != d.argmin(1)) & ~(cid < TAU)).sum())
            worst = max(worst, float(((Cf[yb, xb].double() - cid).abs() / cid.abs().clamp(min=1.0)).max()))
        assert nbad == 0, f"slide {s}: {nbad} sampled labels differ from the fp64 argmin"
        assert worst < 1e-4, worst


@pytest.mark.timeout(1200)
def test_two_config5_slides_streamed(gpu):
    """Config 5's per-GPU share on an 8-GPU node (16 slides / 8 GPUs)."""
    _config5_slides_streamed(2)


@pytest.mark.timeout(1200)
def test_four_config5_slides_streamed(gpu):
    """Config 5's per-GPU share on a 4-GPU node (16 slides / 4 GPUs): four
    40k x 40k x 50 slides, 4 x 54.4 GB = 217.6 GB of clustering rows beside
    the fit state (~23 GB) and the label outputs (4 x 8 GB) on one 288 GB
    MI355X (DESIGN.md section 10 feasibility table).  It runs, with the same
    property checks as the 8-GPU share."""
    _config5_slides_streamed(4)


@pytest.mark.timeout(600)
def test_label_pass_twice_config5_resident(gpu):
    """A 40k x 40k x 50 slide resident in HBM (deferred blur: its fp32 blur,
    320 GB, is never stored), labelled twice while the first result is kept:
    the second pass takes the QC sums too (label_tissue_regions(qc=True)).
    Round 4's banded label pass sized its fp32 band from free + cached HBM
    and failed one 28.7 GiB allocation here; the band buffer is now sized
    from what one allocation can get and halved on an allocation failure.
    Labels and confidences are bitwise those of the first pass."""
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW
    from milwrm_amd import device as D

    D.WS.clear()
    torch.cuda.empty_cache()
    H = W = 40_000
    C = 50
    raw, mask = D.synth_slide(H, W, C, seed=20251015, mode="hard")
    im = M.img.from_device(raw, mask)
    feats = list(range(C))
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=feats, sigma=2, fract=0.2)
    lab.find_tissue_regions(k=8, random_state=18)
    assert im._pending_blur is not None  # deferred: the banded label pass
    cents = lab.kmeans.cluster_centers_
    r1 = MW._assign_img(im, feats, cents, lab.scaler)
    r2 = MW._assign_img(im, feats, cents, lab.scaler, qc=True)
    assert torch.equal(r1[0], r2[0])
    assert torch.equal(r1[1].view(torch.int32), r2[1].view(torch.int32))
    # per-domain confidence sums: exact fixed-point limbs, so the second pass
    # (less free HBM: other band heights) gives the same bits
    assert torch.equal(r1[2], r2[2])
    assert r2[3] is not None and int(r2[3]["n"]) == H * W


def test_domain_sums_band_invariant(gpu, monkeypatch):
    """confidence_score_df and the label pass's domain records do not depend
    on how the slide is cut: the resident (materialised) label pass and the
    banded pass of a deferred-blur slide at two band heights give the same
    bits (exact fixed-point confidence sums, MILWRM.py:447-449)."""
    slides = _slides(8)
    monkeypatch.setenv("MW_FUSED_BLUR", "0")
    ref = _pipeline(slides, qc=False)
    for band in ("23", "61"):
        monkeypatch.setenv("MW_FUSED_BLUR", "1")
        monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", band)
        got = _pipeline(slides, qc=False)
        _assert_same(got, ref)  # conf_df and the domain records included
