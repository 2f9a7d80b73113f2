"""Label + confidence pass (KMeans.predict on every pixel fused with
``estimate_confidence_score_mxif``, MILWRM.py:237-277 and 389-450) on device."""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native as N
from . import device as D
from . import profiling


def assign_image(img_f32: torch.Tensor, feat_idx, mu, inv, centers: np.ndarray,
                 mask_u8: torch.Tensor, out_lab=None, out_conf=None):
    """One streaming pass over an HWC fp32 image.

    Returns (labels int8 [H,W] with -1 outside the mask, conf fp32 [H,W] with
    NaN outside the mask, dom fp64 [3k] = the per-label sums of confidences
    as exact fixed-point limbs, then per-label pixel counts, both over mask
    != 0: ``dom_sums`` reads them; records of several bands or ranks add
    exactly)."""
    H, W, C = img_f32.shape
    k, F = centers.shape
    dev = img_f32.device
    feat, a, b, c32 = D.h2d_many(
        [np.asarray(feat_idx, dtype=np.int32),
         np.asarray(inv, dtype=np.float64).astype(np.float32),
         (-np.asarray(mu, dtype=np.float64) * np.asarray(inv, dtype=np.float64)).astype(np.float32),
         np.asarray(centers, dtype=np.float32)], dev)
    n = H * W
    lab = torch.empty((H, W), dtype=torch.int8, device=dev) if out_lab is None else out_lab
    conf = torch.empty((H, W), dtype=torch.float32, device=dev) if out_conf is None else out_conf
    assert lab.is_contiguous() and conf.is_contiguous() and lab.numel() == n and conf.numel() == n
    dom = torch.empty(DOM_REC * k, dtype=torch.float64, device=dev)
    ws = D.WS.get("assign", N.query("mw_assign_ws_bytes", n, k))
    st = D.stream()
    with profiling.timed("assign_conf", n * (C * 4 + 1 + 5)):
        N.call("mw_assign_conf", D.P(img_f32), C, D.P(feat), F, D.P(a), D.P(b), D.P(c32), k,
               D.P(mask_u8), n, D.P(lab), D.P(conf), D.P(ws), st)
    N.call("mw_assign_reduce", D.P(ws), n, k, D.P(dom), st)
    return lab, conf, dom


def blur_assign_image(raw, sigma: float, inv_mean, pseudoval: float, mu, inv,
                      centers: np.ndarray, mask_u8: torch.Tensor, truncate: float = 4.0, band_rows=None):
    """``assign_image(blur(lognorm(raw)), all channels, ...)`` with the label
    pass as the blur's epilogue (the blurred slide is never stored), then the
    same per-block domain records.  ``raw``: a resident slide (one launch) or
    a ``stream.RowSource`` (one launch per band of output rows,
    mw_blur_assign_rows, which is bit for bit the whole-slide launch).  None
    when the fused kernel does not take this shape (the caller materialises
    the blur)."""
    from .stream import as_source, band_rows_for, bands

    src = as_source(raw)
    H, W, C = src.shape
    k, F = centers.shape
    if F != C or inv_mean is None:
        return None
    dev = D.device()
    a, b, c32 = D.h2d_many([np.asarray(inv, dtype=np.float64).astype(np.float32),
                            (-np.asarray(mu, dtype=np.float64) * np.asarray(inv, dtype=np.float64))
                            .astype(np.float32), np.asarray(centers, dtype=np.float32)], dev)
    w = D.gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    n = H * W
    lab = torch.empty((H, W), dtype=torch.int8, device=dev)
    conf = torch.empty((H, W), dtype=torch.float32, device=dev)
    mask_u8 = D.padded_mask(mask_u8)
    if band_rows is None:
        band_rows = H if src.zero_copy else band_rows_for(src)
    elem = torch.empty(0, dtype=src.dtype).element_size()
    for y0, y1, a0, rb in bands(src, band_rows, r):
        with profiling.timed("blur_assign", (y1 - y0) * W * (C * elem + 5)):
            ok = N.try_call("mw_blur_assign_rows", D.P(rb), D.dtype_code(rb), int(rb.shape[0]), W, C, a0,
                            y0 - a0, y1 - a0, D.P(inv_mean), float(pseudoval), w.ctypes.data, r, D.P(a),
                            D.P(b), D.P(c32), k, D.P(mask_u8), D.P(lab), D.P(conf), D.stream())
        if not ok:  # shape-determined: decided by the first band
            return None
    D.FUSED_USED["assign"] += 1
    if not src.zero_copy:
        D.FUSED_USED["assign_streamed"] += 1
    dom = torch.empty(DOM_REC * k, dtype=torch.float64, device=dev)
    ws = D.WS.get("assign", N.query("mw_assign_ws_bytes", n, k))
    st = D.stream()
    with profiling.timed("domain_records", n * 5):
        N.call("mw_domain_records", D.P(lab), D.P(conf), n, C, k, D.P(ws), st)
    N.call("mw_assign_reduce", D.P(ws), n, k, D.P(dom), st)
    return lab, conf, dom


def _assign_band_rows(src, r, extra_per_row, band_rows):
    """Output rows per band of the banded label / QC passes: ``band_rows``,
    else ``MW_ASSIGN_BAND_ROWS``, else (resident slide) what half the free
    HBM holds as fp32 (what one allocation can get: ``stream.alloc_bytes``),
    (streamed slide) ``stream.band_rows_for``."""
    from .stream import alloc_bytes, band_rows_for

    if band_rows is not None:
        return int(band_rows)
    env = os.environ.get("MW_ASSIGN_BAND_ROWS")
    if env:
        return int(env)
    if src.zero_copy:
        return int(alloc_bytes() // 2 // extra_per_row) - 2 * r
    return band_rows_for(src, extra_per_row)


def _band_buffer(H, W, C, r, band_rows, min_band=16):
    """The reused fp32 band buffer of the banded passes and the band height it
    holds: ``band_rows`` output rows + 2r halo rows, lower if that one
    allocation fails (``stream.alloc_rows`` halves it on an out-of-memory
    error, down to ``min_band`` output rows)."""
    from .stream import alloc_rows

    want = min(H, band_rows + 2 * r)
    buf = alloc_rows(want, (W, C), torch.float32, min_rows=min(want, min_band + 2 * r))
    got = int(buf.shape[0])
    return buf, (band_rows if got >= want else got - 2 * r)


def banded_assign_image(raw, sigma: float, inv_mean, pseudoval: float, feat_idx, mu,
                        inv, centers: np.ndarray, mask_u8: torch.Tensor, truncate: float = 4.0,
                        band_rows=None, out_rows=None, qc: LabelPassQC | None = None):
    """``assign_image(blur(lognorm(raw)))`` for a slide whose fp32 blurred copy
    does not fit HBM: the blur is materialised one band of rows at a time
    (band plus r halo rows of input; the kernel's arithmetic per output value
    does not depend on the band, so labels and confidences are bitwise those
    of the whole-slide blur) into one reused buffer, and each band goes
    through the label pass.  The per-domain sums are added band after band.
    ``raw``: a resident slide or a ``stream.RowSource`` (a slide that is not
    resident: its bands are read as they are needed, the next one while this
    one is labelled).  None when not even a 16-row band fits in half the
    free HBM.  ``out_rows`` = (r0, r1): label only those rows of ``raw`` (a
    slide band's own rows inside its halo'd array, milwrm_amd.bands); outputs
    are (r1 - r0) x W.  ``qc``: a ``LabelPassQC`` that takes every labelled
    band (whole slides only: ``out_rows`` None)."""
    from .stream import as_source, bands

    src = as_source(raw)
    H, W, C = src.shape
    r0, r1 = (0, H) if out_rows is None else (int(out_rows[0]), int(out_rows[1]))
    k, F = centers.shape
    w = D.gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    row_bytes = W * C * 4
    from .stream import RESIDENCY

    # the outputs (5 bytes per pixel) and a minimal band must fit: cached
    # scratch of earlier passes and resident copies of other slides go first
    RESIDENCY.release((r1 - r0) * W * 5 + (16 + 2 * r) * row_bytes + (256 << 20))
    band_rows = _assign_band_rows(src, r, row_bytes, band_rows)
    if band_rows < 16:
        return None
    band_rows = min(band_rows, r1 - r0)
    dev = D.device()
    lab = torch.empty((r1 - r0, W), dtype=torch.int8, device=dev)
    conf = torch.empty((r1 - r0, W), dtype=torch.float32, device=dev)
    dom = torch.zeros(DOM_REC * k, dtype=torch.float64, device=dev)  # exact limbs: any band split, same bits
    buf, band_rows = _band_buffer(H, W, C, r, band_rows)
    for y0, y1, a, rb in bands(src, band_rows, r, r0, r1):
        out = buf[:rb.shape[0]]
        D.blur(rb, sigma, inv_mean=inv_mean, pseudoval=pseudoval, out=out, truncate=truncate)
        _, _, d = assign_image(out[y0 - a:y1 - a], feat_idx, mu, inv, centers,
                               D.padded_mask(mask_u8[y0:y1].contiguous()),
                               out_lab=lab[y0 - r0:y1 - r0], out_conf=conf[y0 - r0:y1 - r0])
        dom_add_(dom, d)
        if qc is not None:  # the band is still in the buffer: its QC sums now
            qc.band(out[y0 - a:y1 - a], lab[y0 - r0:y1 - r0])
    D.FUSED_USED["assign_banded"] += 1
    if not src.zero_copy:
        D.FUSED_USED["assign_streamed"] += 1
    return lab, conf, dom


def _labels_i8(tissue_id, n, k, dev) -> torch.Tensor:
    """tissue_ID as the kernels read it: int8 per pixel, -1 = no domain."""
    if isinstance(tissue_id, torch.Tensor) and tissue_id.dtype == torch.int8:
        return tissue_id.to(dev).reshape(n).contiguous()
    t = np.asarray(tissue_id, dtype=np.float64).reshape(-1)
    if t.size != n:
        raise ValueError(f"tissue_ID has {t.size} pixels, image has {n}")
    ok = np.isfinite(t) & (t >= 0) & (t < k) & (t == np.floor(t))
    return D.h2d(np.where(ok, t, -1).astype(np.int8), dev)


def _exp38(bound) -> np.ndarray:
    """Per-entry e with bound * 2^e < 2^38 (the fixed point of mw_domain_sse)."""
    bound = np.asarray(bound, dtype=np.float64)
    e = np.zeros(bound.shape, dtype=np.int32)
    pos = np.isfinite(bound) & (bound > 0)
    e[pos] = 38 - np.frexp(bound[pos])[1]
    return e


class _DomainSSE:
    """Exact per-domain QC sums of one slide (mw_domain_sse), accumulated over
    any number of pixel ranges (the whole slide, or band after band): the
    fixed point of every feature comes from the slide's column maxima, the
    scaler, the centers and the pivot, so the sums are the same bits however
    the pixels are split."""

    def __init__(self, feat, F, mu, inv, centers, pivot, colmax, dev):
        k = centers.shape[0]
        if not 1 <= k <= 127:
            raise ValueError(f"domain statistics support 1 <= k <= 127 domains, got {k}")
        mu = np.asarray(mu, dtype=np.float64)
        inv = np.asarray(inv, dtype=np.float64)
        self.k, self.F, self.dev = k, F, dev
        b = -mu * inv
        cen = np.ascontiguousarray(centers, dtype=np.float64)
        pivot = np.asarray(pivot, dtype=np.float64)
        # |x'_f| <= |a_f| max|x| + |b_f| (slack for the fp64 rounding of x')
        xs = (np.abs(inv) * np.asarray(colmax, dtype=np.float64)[feat] + np.abs(b)) * (1 + 1e-12)
        cm = np.abs(cen).max(axis=0)
        y = xs + np.abs(pivot)
        self.exps = np.concatenate([_exp38((xs + cm) ** 2), _exp38(y), _exp38(y * y)]).astype(np.int32)
        self.pivot = pivot
        # a non-finite value in a feature's column (maximum), its pivot or a
        # center column has no fixed point: the reference's numpy sums give NaN
        # there, so every quantity of that feature is NaN (conservatively: all
        # domains of the feature, not only those holding the value)
        self.nonfinite = ~(np.isfinite(xs) & np.isfinite(pivot) & np.isfinite(cm))
        self.chunks = [(d0, min(20, k - d0)) for d0 in range(0, k, 20)]
        self.feat_d, self.a_d, self.b_d, self.pv_d, self.qe_d = D.h2d_many(
            [np.asarray(feat, dtype=np.int32), inv, b, pivot, self.exps], dev)
        self.c_d = [D.h2d(cen[d0:d0 + kc], dev) for d0, kc in self.chunks]
        self.out = [torch.zeros(N.query("mw_domain_sse_out_len", kc, F), dtype=torch.float64,
                                device=dev) for _, kc in self.chunks]
        self.n = 0
        self.n_adds = 0

    def add(self, img_f32: torch.Tensor, labels_i8: torch.Tensor):
        """Add the pixels of an HWC fp32 range (or fp64 rows as an S x 1 x F
        image) and its int8 labels."""
        H, W, C = img_f32.shape
        n = H * W
        if n == 0:
            return
        self.n_adds += 1
        if self.n_adds >= 1 << 10:  # every add puts < 2^43 into a limb: exact below 2^53
            raise MemoryError("QC sums over 1023 pixel ranges or more would leave the exact limbs: "
                              "the bands are too low for the HBM this slide needs")
        st = D.stream()
        f64 = img_f32.dtype == torch.float64
        for (d0, kc), c_d, out in zip(self.chunks, self.c_d, self.out):
            ws = D.WS.get("domain_sse", N.query("mw_domain_sse_ws_bytes", n, kc, self.F))
            with profiling.timed("domain_sse", n * (C * img_f32.element_size() + 1)):
                N.call("mw_domain_sse_f64" if f64 else "mw_domain_sse", D.P(img_f32), C, D.P(self.feat_d),
                       self.F, D.P(self.a_d),
                       D.P(self.b_d), D.P(self.pv_d), D.P(c_d), D.P(self.qe_d), kc, d0,
                       D.P(labels_i8), n, D.P(out), 1, D.P(ws), st)
        self.n += n

    def result(self) -> dict:
        F, k = self.F, self.k
        e = self.exps.astype(np.int64)
        sse = np.zeros((k, F))
        count = np.zeros(k)
        sums = None
        for (d0, kc), o in zip(self.chunks, D.d2h(*self.out) if len(self.out) > 1 else [D.d2h(self.out[0])]):
            NQ = kc * F + 2 * F
            # two-level fixed point: (hi + lo 2^-38) 2^-e, each level as 32-bit limbs
            hi = o[:NQ] * 4294967296.0 + o[NQ:2 * NQ]
            lo = o[2 * NQ:3 * NQ] * 4294967296.0 + o[3 * NQ:4 * NQ]
            scale = np.ldexp(1.0, -np.concatenate([np.tile(e[:F], kc), e[F:2 * F], e[2 * F:]]))
            v = (hi + np.ldexp(lo, -38)) * scale
            sse[d0:d0 + kc] = v[:kc * F].reshape(kc, F)
            count[d0:d0 + kc] = o[4 * NQ:]
            if sums is None:
                sums = (v[kc * F:kc * F + F], v[kc * F + F:])
        s1, s2 = sums
        if self.nonfinite.any():
            sse[:, self.nonfinite] = np.nan
            s1, s2 = s1.copy(), s2.copy()
            s1[self.nonfinite] = np.nan
            s2[self.nonfinite] = np.nan
        return {"sse": sse, "sum": s1, "sumsq": s2, "count": count, "n": self.n,
                "pivot": self.pivot}


def _colmax(img_f32: torch.Tensor, out=None, accumulate=False) -> torch.Tensor:
    H, W, C = img_f32.shape
    if out is None:
        out = torch.zeros(C, dtype=torch.float32, device=img_f32.device)
    if H * W:
        N.call("mw_col_absmax_acc" if accumulate else "mw_col_absmax", D.P(img_f32), H * W, C,
               D.P(out), D.stream())
    return out


def domain_sse_image(img_f32: torch.Tensor, feat_idx, mu, inv, centers: np.ndarray,
                     tissue_id, pivot=None, colmax=None) -> dict:
    """Per-domain squared error and whole-slide scaled sums (``mw_domain_sse``;
    the sums behind ``estimate_percentage_variance_mxif`` MILWRM.py:280-333,
    ``estimate_mse_mxif`` :453-515 and the ST twins :518-554, :601-644), one
    pass per 20 domains, exact (fixed point from the slide's column maxima).

    ``tissue_id``: H x W labels as the reference holds them (float, NaN outside
    the mask) or an int8 device map with -1 outside the mask.  ``pivot``: the
    shift of the whole-slide sums (default: the scaled features of the first
    pixel, which keeps a near-constant feature free of cancellation).  Returns
    fp64 host arrays: sse (k x F), sum / sumsq of x' - pivot (F), count (k),
    n (pixels), pivot (F).  ``colmax``: the per-channel max |x| (default: a
    device pass over the fp32 slide)."""
    H, W, C = img_f32.shape
    k, F = centers.shape
    img_f32 = img_f32.contiguous()
    feat = _check_feats(feat_idx, F, C)
    dev = img_f32.device
    n = H * W
    lab = _labels_i8(tissue_id, n, k, dev)
    if pivot is None:
        pivot = _first_pixel_scaled(img_f32, feat, mu, inv)
    if colmax is None:  # (mw_col_absmax takes up to 16384 channels)
        colmax = D.d2h(_colmax(img_f32))
    acc = _DomainSSE(feat, F, mu, inv, centers, pivot, colmax, dev)
    acc.add(img_f32, lab)
    return acc.result()


def _check_feats(feat_idx, F, C) -> np.ndarray:
    feat = np.asarray(feat_idx, dtype=np.int32)
    feat = np.where(feat < 0, feat + C, feat).astype(np.int32)
    if feat.shape != (F,) or feat.min() < 0 or feat.max() >= C:
        raise ValueError(f"features {feat_idx} do not match {F} centroid columns / {C} channels")
    return feat


def _first_pixel_scaled(img_f32, feat, mu, inv) -> np.ndarray:
    x0 = D.d2h(img_f32.reshape(-1, img_f32.shape[2])[0]).astype(np.float64)[feat]
    return x0 * np.asarray(inv, dtype=np.float64) - np.asarray(mu, dtype=np.float64) * np.asarray(
        inv, dtype=np.float64)


def domain_sse_deferred(raw, sigma: float, inv_mean, pseudoval: float, feat_idx, mu,
                        inv, centers: np.ndarray, tissue_id, truncate: float = 4.0,
                        band_rows=None, colmax=None) -> dict:
    """``domain_sse_image(blur(lognorm(raw)), ...)`` for a slide whose fp32
    blurred copy does not fit HBM (the deferred-blur mode): the blur is
    materialised band by band (band + r halo rows of input) into one reused
    buffer, twice -- once for the column maxima that fix the fixed point,
    once for the sums -- or once when ``colmax`` (a per-channel bound on |x|,
    ``img._blur_bound``) is given.  The sums are exact, so the result is
    bitwise the materialised slide's given the same bound
    (tests/test_gpu_qc.py).  ``raw``: a resident slide or a
    ``stream.RowSource`` (read band by band)."""
    from .stream import as_source
    from .stream import bands as read_bands

    src = as_source(raw)
    H, W, C = src.shape
    k, F = centers.shape
    feat = _check_feats(feat_idx, F, C)
    w = D.gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    band_rows = _assign_band_rows(src, r, W * C * 4, band_rows)
    if band_rows < 1:
        raise MemoryError("not even one row band of the blurred slide fits in half the free HBM")
    band_rows = min(band_rows, H)
    # exact limbs: every band adds < 2^43 per quantity, the fp64 sums stay exact below 2^53
    if -(-H // band_rows) >= 1 << 10:
        band_rows = -(-H // ((1 << 10) - 1))
    dev = D.device()
    lab = _labels_i8(tissue_id, H * W, k, dev)
    buf, band_rows = _band_buffer(H, W, C, r, band_rows)
    # the buffer may have come back lower than asked (alloc_rows halves on an
    # out-of-memory error) and stream.bands may lower the bands again: the
    # limb budget is checked on the bands actually summed (acc.add below)
    if -(-H // max(1, band_rows)) >= 1 << 10:
        raise MemoryError(f"the QC sums of this {H}-row slide need bands of >= {-(-H // 1023)} rows "
                          f"for exact limbs and HBM holds {band_rows}")

    def bands():
        for y0, y1, a, rb in read_bands(src, band_rows, r):
            out = buf[:rb.shape[0]]
            D.blur(rb, sigma, inv_mean=inv_mean, pseudoval=pseudoval, out=out, truncate=truncate)
            yield y0, y1, out[y0 - a:y1 - a]

    acc = None
    if colmax is None:
        cmax = torch.zeros(C, dtype=torch.float32, device=dev)
        pivot = None
        for y0, y1, core in bands():
            if pivot is None:
                pivot = _first_pixel_scaled(core, feat, mu, inv)
            _colmax(core, cmax, accumulate=True)
        acc = _DomainSSE(feat, F, mu, inv, centers, pivot, D.d2h(cmax), dev)
    for y0, y1, core in bands():
        if acc is None:  # the pivot is the slide's first pixel, as above
            acc = _DomainSSE(feat, F, mu, inv, centers, _first_pixel_scaled(core, feat, mu, inv),
                             colmax, dev)
        acc.add(core, lab[y0 * W:y1 * W])
    return acc.result()


class LabelPassQC:
    """The QC sums of ``domain_sse_image`` as extra outputs of the label pass
    (SURVEY 8f row 3): the banded label pass hands every fp32 band it has
    just labelled, with its labels, to ``band`` (no second blur of the
    slide); a resident slide is handed whole.  The fixed point comes from
    ``colmax`` (the slide's ``img._blur_bound``, known before the first band)
    and the pivot from the slide's first pixel, as the standalone
    ``domain_sse_image`` / ``domain_sse_deferred`` take them, so the sums are
    the same bits as those passes'."""

    def __init__(self, feat_idx, C, mu, inv, centers: np.ndarray, colmax):
        k, F = centers.shape
        self.feat = _check_feats(feat_idx, F, C)
        self.mu, self.inv = mu, inv
        self.centers = np.ascontiguousarray(centers, dtype=np.float64)
        self.colmax = colmax
        self.acc = None
        self.stats = None
        self.n_bands = 0

    def band(self, core: torch.Tensor, labels_i8: torch.Tensor):
        """Add an fp32 HWC band (the slide's rows from its first on) and its
        int8 labels (-1 = no domain), in slide order."""
        self.n_bands += 1
        if self.n_bands >= 1 << 10:  # past the exact-limb budget (domain_sse_deferred): no result
            self.acc = False
        if self.acc is False:
            return
        if self.acc is None:
            self.acc = _DomainSSE(self.feat, self.centers.shape[1], self.mu, self.inv, self.centers,
                                  _first_pixel_scaled(core, self.feat, self.mu, self.inv),
                                  self.colmax, core.device)
        self.acc.add(core, labels_i8.reshape(-1))

    def result(self):
        """The ``domain_sse_image`` dict, or None (nothing added, or too many
        bands: the estimators then run their own pass)."""
        self.stats = self.acc.result() if self.acc else None
        return self.stats


def domain_sse_rows(X: np.ndarray, centers: np.ndarray, labels) -> dict:
    """``domain_sse_image`` over host rows already in the centers' space (the
    ST estimators' cluster_data): the rows travel as a 1-pixel-wide fp64
    image (``mw_domain_sse_f64``: the reference's float64 rows, no fp32
    rounding), labels < 0 belong to no domain."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    S, F = X.shape
    dev = D.device()
    img = torch.from_numpy(X.reshape(S, 1, F)).to(dev)
    lab = torch.from_numpy(np.asarray(labels, dtype=np.int64).clip(-1, 127).astype(np.int8)).to(dev)
    return domain_sse_image(img, np.arange(F), np.zeros(F), np.ones(F), centers, lab.reshape(S, 1),
                            pivot=X[0].copy(), colmax=np.abs(X).max(axis=0) if S else np.zeros(F))


def dm_total(s: dict) -> np.float64:
    """sum over pixels and features of (x' - mean(x'))^2 from the shifted sums
    (np.float64, so a zero denominator gives inf / nan as the reference's
    numpy division does)."""
    n = np.float64(s["n"])
    return np.float64(np.sum(s["sumsq"] - s["sum"] * s["sum"] / n))


def assign_rows(X: np.ndarray, centers: np.ndarray, mu=None, inv=None):
    """Assign host rows (S x F, already in the centers' space unless an
    affine is given).  Returns (labels int64, conf fp64, dom fp64[3k]
    domain records, ``dom_sums``)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    S, F = X.shape
    dev = D.device()
    img = torch.from_numpy(X.reshape(S, 1, F)).to(dev)
    mask = torch.ones((S, 1), dtype=torch.uint8, device=dev)
    mu = np.zeros(F) if mu is None else mu
    inv = np.ones(F) if inv is None else inv
    lab, conf, dom = assign_image(img, np.arange(F), mu, inv, centers, mask)
    return (lab.reshape(-1).cpu().numpy().astype(np.int64),
            conf.reshape(-1).cpu().numpy().astype(np.float64), dom.cpu().numpy())


DOM_REC = 3  # label-pass domain records: [conf hi k | conf lo k | count k] (mw_assign_reduce)
_TWO32 = 4294967296.0


def dom_add_(dom: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    """dom += d for label-pass domain records (integer-valued fp64 limbs),
    with the lo limbs' carries moved into the hi limbs so that any number of
    bands stays exact (every entry below 2^53)."""
    dom += d
    return dom_carry_(dom)


def dom_carry_(dom: torch.Tensor) -> torch.Tensor:
    """Move the lo limbs' carries of domain records into their hi limbs (in
    place, exact): after adding records of several bands or ranks."""
    k = dom.shape[-1] // DOM_REC
    carry = torch.floor(dom[..., k:2 * k] / _TWO32)
    dom[..., :k] += carry
    dom[..., k:2 * k] -= carry * _TWO32
    return dom


def dom_sums(dom, k: int):
    """(per-domain sums of the confidences, pixel counts) as fp64 from the
    records: one rounding of the exact fixed-point total, so the same bits
    for any split of the pixels."""
    d = np.asarray(dom, dtype=np.float64)
    s = (d[..., :k] * _TWO32 + d[..., k:2 * k]) * 2.0 ** -32
    return s, d[..., 2 * k:3 * k]


def domain_means(dom: np.ndarray, k: int) -> dict:
    """Per-domain mean confidence ``np.mean(cID[tissue_ID == i])`` from the
    label pass's records: NaN for an empty domain (numpy's mean of an empty
    slice)."""
    s, cnt = dom_sums(dom, k)
    out = {}
    for i in range(k):
        n = cnt[i]
        out[i] = float(s[i] / n) if n > 0 else float("nan")
    return out
