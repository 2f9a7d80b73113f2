"""Label + confidence pass (KMeans.predict on every pixel fused with
``estimate_confidence_score_mxif``, MILWRM.py:237-277 and 389-450) on device."""
from __future__ import annotations

import numpy as np
import torch

from . import _native as N
from . import device as D
from . import profiling


def assign_image(img_f32: torch.Tensor, feat_idx, mu, inv, centers: np.ndarray,
                 mask_u8: torch.Tensor):
    """One streaming pass over an HWC fp32 image.

    Returns (labels int8 [H,W] with -1 outside the mask, conf fp32 [H,W] with
    NaN outside the mask, dom fp64 [2k] = per-label sum of confidences then
    per-label pixel counts, both over mask != 0)."""
    H, W, C = img_f32.shape
    k, F = centers.shape
    dev = img_f32.device
    feat = D.h2d(np.asarray(feat_idx, dtype=np.int32), dev)
    a = D.h2d(np.asarray(inv, dtype=np.float64).astype(np.float32), dev)
    b = D.h2d((-np.asarray(mu, dtype=np.float64) * np.asarray(inv, dtype=np.float64))
              .astype(np.float32), dev)
    c32 = D.h2d(np.asarray(centers, dtype=np.float32), dev)
    n = H * W
    lab = torch.empty((H, W), dtype=torch.int8, device=dev)
    conf = torch.empty((H, W), dtype=torch.float32, device=dev)
    dom = torch.empty(2 * k, dtype=torch.float64, device=dev)
    ws = D.WS.get("assign", N.query("mw_assign_ws_bytes", n, k))
    st = D.stream()
    with profiling.timed("assign_conf", n * (C * 4 + 1 + 5)):
        N.call("mw_assign_conf", D.P(img_f32), C, D.P(feat), F, D.P(a), D.P(b), D.P(c32), k,
               D.P(mask_u8), n, D.P(lab), D.P(conf), D.P(ws), st)
    N.call("mw_assign_reduce", D.P(ws), n, k, D.P(dom), st)
    return lab, conf, dom


def blur_assign_image(raw: torch.Tensor, sigma: float, inv_mean, pseudoval: float, mu, inv,
                      centers: np.ndarray, mask_u8: torch.Tensor, truncate: float = 4.0):
    """``assign_image(blur(lognorm(raw)), all channels, ...)`` in one pass over
    the raw slide (the fused blur assign epilogue; the blurred slide is never
    stored), then the same per-block domain records.  None when the fused
    kernel does not take this shape (the caller materialises the blur)."""
    H, W, C = raw.shape
    k, F = centers.shape
    if F != C or inv_mean is None:
        return None
    dev = raw.device
    a = D.h2d(np.asarray(inv, dtype=np.float64).astype(np.float32), dev)
    b = D.h2d((-np.asarray(mu, dtype=np.float64) * np.asarray(inv, dtype=np.float64))
              .astype(np.float32), dev)
    c32 = D.h2d(np.asarray(centers, dtype=np.float32), dev)
    w = D.gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    n = H * W
    lab = torch.empty((H, W), dtype=torch.int8, device=dev)
    conf = torch.empty((H, W), dtype=torch.float32, device=dev)
    mask_u8 = D.padded_mask(mask_u8)
    st = D.stream()
    with profiling.timed("blur_assign", n * (C * raw.element_size() + 5)):
        ok = N.try_call("mw_blur_assign_conf", D.P(raw), D.dtype_code(raw), H, W, C, D.P(inv_mean),
                        float(pseudoval), w.ctypes.data, r, D.P(a), D.P(b), D.P(c32), k,
                        D.P(mask_u8), D.P(lab), D.P(conf), st)
    if not ok:
        return None
    D.FUSED_USED["assign"] += 1
    dom = torch.empty(2 * k, dtype=torch.float64, device=dev)
    ws = D.WS.get("assign", N.query("mw_assign_ws_bytes", n, k))
    with profiling.timed("domain_records", n * 5):
        N.call("mw_domain_records", D.P(lab), D.P(conf), n, C, k, D.P(ws), st)
    N.call("mw_assign_reduce", D.P(ws), n, k, D.P(dom), st)
    return lab, conf, dom


def assign_rows(X: np.ndarray, centers: np.ndarray, mu=None, inv=None):
    """Assign host rows (S x F, already in the centers' space unless an
    affine is given).  Returns (labels int64, conf fp64, dom fp64[2k])."""
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


def domain_means(dom: np.ndarray, k: int) -> dict:
    """Per-domain mean confidence ``np.mean(cID[tissue_ID == i])``: NaN for an
    empty domain (numpy's mean of an empty slice)."""
    out = {}
    for i in range(k):
        n = dom[k + i]
        out[i] = float(dom[i] / n) if n > 0 else float("nan")
    return out
