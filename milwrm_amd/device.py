"""Device engine: thin typed wrappers over the C ABI that take torch tensors
(PyTorch supplies HBM allocations and the current HIP stream — plumbing only;
every computation is a hand-written HIP kernel in ``csrc/``)."""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native as N
from . import profiling

_DTYPE_CODE = {torch.uint8: N.MW_U8, torch.int16: N.MW_U16, torch.float32: N.MW_F32}


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("milwrm_amd runs on an AMD Instinct GPU (HIP); no device is visible "
                           "and there is no CPU fallback")
    N.load()


def device():
    require_gpu()
    return torch.device("cuda", torch.cuda.current_device())


def stream():
    return torch.cuda.current_stream().cuda_stream


def P(t):
    """Raw device pointer of a tensor (or None)."""
    return None if t is None else t.data_ptr()


class Workspace:
    """Grow-only scratch buffers per (device, tag); never freed inside a pass."""

    def __init__(self):
        self._bufs = {}

    def get(self, tag: str, nbytes: int) -> torch.Tensor:
        dev = torch.cuda.current_device()
        key = (dev, tag)
        b = self._bufs.get(key)
        nbytes = max(int(nbytes), 256)
        if b is None or b.numel() < nbytes:
            self._bufs.pop(key, None)
            b = None
            try:
                b = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", dev))
            except torch.OutOfMemoryError:  # the other passes' cached scratch goes first
                self.drop()
                torch.cuda.empty_cache()
                b = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", dev))
            self._bufs[key] = b
        return b

    def cached_bytes(self) -> int:
        return sum(b.numel() for b in self._bufs.values())

    def drop(self) -> int:
        """Hand every cached scratch buffer back to the allocator (they are
        made again on their next use; the kernels that used them were
        enqueued on the current stream, so stream-ordered reuse is safe).
        Returns the bytes dropped.  Config 5 at 4 slides per GPU: the fit's
        workspace (~21 B per row, 21 GiB) and the sample map (8 B per pixel,
        12 GiB) would otherwise stay cached through the label pass."""
        n = self.cached_bytes()
        self._bufs.clear()
        return n

    def clear(self):
        self._bufs.clear()


WS = Workspace()


class _PinnedPool:
    """Page-locked staging buffers allocated once per process and reused.

    torch's caching host allocator sometimes (per process, not per box) fails
    to reuse its blocks and then pays a page-locking allocation of several ms
    on every small transfer (measured: +50 ms per bench step).  Here a buffer
    is handed out again only when the event recorded after its last
    asynchronous copy has completed, so a non-blocking host-to-device copy is
    never overwritten before the DMA has read it."""

    def __init__(self):
        self._slots = {}  # bucket bytes -> list of [uint8 pinned tensor, event or None]

    def take(self, nbytes: int):
        bucket = 1 << max(12, (max(int(nbytes), 1) - 1).bit_length())
        lst = self._slots.setdefault(bucket, [])
        for slot in lst:
            ev = slot[1]
            if ev is None or ev.query():
                slot[1] = None
                return slot
        slot = [torch.empty(bucket, dtype=torch.uint8, pin_memory=True), None]
        lst.append(slot)
        return slot


_PINNED = _PinnedPool()


class _Busy:
    """Event stand-in for a slot held by a d2h call until it returns."""

    @staticmethod
    def query():
        return False


def _staged(slot, a: np.ndarray) -> torch.Tensor:
    """Flat typed view of a pinned slot holding a copy of ``a``."""
    v = slot[0][:a.nbytes].view(torch.from_numpy(a.reshape(-1)[:0]).dtype)
    v.numpy()[:] = a.reshape(-1)
    return v


def _mark(slot):
    ev = torch.cuda.Event()
    ev.record()
    slot[1] = ev


def h2d(a, device=None) -> torch.Tensor:
    """Small host array → device without a synchronous pageable copy: staged
    through a pooled pinned buffer, copied non-blocking on the current
    stream."""
    a = np.ascontiguousarray(a)
    dev = device if device is not None else torch.cuda.current_device()
    if a.nbytes == 0:
        return torch.from_numpy(a).to(dev)
    slot = _PINNED.take(a.nbytes)
    out = _staged(slot, a).to(dev, non_blocking=True).view(a.shape)
    _mark(slot)
    return out


def h2d_many(arrays, device=None):
    """Several small host arrays → device in ONE staged copy (16-byte aligned
    sections of one buffer); returns device views with the arrays' dtypes and
    shapes."""
    arrays = [np.ascontiguousarray(a) for a in arrays]
    offs, n = [], 0
    for a in arrays:
        offs.append(n)
        n += (a.nbytes + 15) & ~15
    buf = np.zeros(max(n, 16), dtype=np.uint8)
    for a, o in zip(arrays, offs):
        buf[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
    dev = h2d(buf, device)
    return [dev[o:o + a.nbytes].view(torch.from_numpy(a.reshape(-1)[:0]).dtype).view(a.shape)
            for a, o in zip(arrays, offs)]


def h2d_into(dst: torch.Tensor, a) -> None:
    """dst (contiguous device tensor) ← host array of the same size, staged
    like h2d."""
    a = np.ascontiguousarray(a, dtype=torch.empty(0, dtype=dst.dtype).numpy().dtype)
    assert a.size == dst.numel() and dst.is_contiguous()
    slot = _PINNED.take(a.nbytes)
    dst.view(-1).copy_(_staged(slot, a), non_blocking=True)
    _mark(slot)


class PendingD2H:
    """Device → host copies queued by ``d2h_async``; ``wait()`` returns the
    arrays (one or a tuple) after the copies, not after work queued later."""

    def __init__(self, staged, ev):
        self._staged, self._ev, self._out = staged, ev, None

    def wait(self):
        if self._out is None:
            self._ev.synchronize()
            arrs = tuple(v.numpy().copy().reshape(shape) for _, v, shape in self._staged)
            for slot, _, _ in self._staged:
                slot[1] = None
            self._staged = ()
            self._out = arrs[0] if len(arrs) == 1 else arrs
        return self._out


def d2h_async(*ts: torch.Tensor) -> PendingD2H:
    """Queue device tensors → host copies: each is copied non-blocking into a
    pooled pinned buffer (DMA straight into page-locked memory, no pageable
    staging by the runtime), followed by an event.  The host may queue more
    device work before it waits (``PendingD2H.wait``)."""
    staged = []
    for t in ts:
        t = t.contiguous()
        nbytes = t.numel() * t.element_size()
        slot = _PINNED.take(nbytes)
        slot[1] = _Busy
        v = slot[0][:nbytes].view(t.dtype)
        v.copy_(t.reshape(-1), non_blocking=True)
        staged.append((slot, v, tuple(t.shape)))
    ev = torch.cuda.Event()
    ev.record()
    return PendingD2H(staged, ev)


def d2h(*ts: torch.Tensor):
    """Device tensors → host numpy arrays (fresh copies) with ONE
    synchronisation (on the copies).  Returns one array or a tuple."""
    return d2h_async(*ts).wait()


def dtype_code(t: torch.Tensor) -> int:
    try:
        return _DTYPE_CODE[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported device image dtype {t.dtype}") from None


def to_device_image(arr: np.ndarray) -> torch.Tensor:
    """Upload an HWC host image keeping a compact element type: uint8/uint16
    stay integral (uint16 travels as int16 bits), everything else → fp32."""
    require_gpu()
    a = np.ascontiguousarray(arr)
    if a.dtype == np.uint8:
        h = torch.from_numpy(a)
    elif a.dtype == np.uint16:
        h = torch.from_numpy(a.view(np.int16))
    elif a.dtype == np.bool_:
        h = torch.from_numpy(a.astype(np.uint8))
    else:
        if np.issubdtype(a.dtype, np.integer) and a.size and (a.min() >= 0 and a.max() <= 65535):
            h = torch.from_numpy(a.astype(np.uint16).view(np.int16))
        else:
            h = torch.from_numpy(a.astype(np.float32))
    return h.to(device(), non_blocking=False)


def as_float32(t: torch.Tensor) -> torch.Tensor:
    """Element-type cast of a raw device image (uint16 travels as int16)."""
    if t.dtype == torch.float32:
        return t
    if t.dtype == torch.int16:
        return (t.to(torch.int32) & 0xFFFF).to(torch.float32)
    return t.to(torch.float32)


def to_host_float64(t: torch.Tensor) -> np.ndarray:
    if t.dtype == torch.int16:
        return t.cpu().numpy().view(np.uint16).astype(np.float64)
    return t.cpu().numpy().astype(np.float64)


# ------------------------------------------------------------------ kernels

def nz_stats(img: torch.Tensor):
    """Per-channel (sum, count) of non-zero elements of an HWC image."""
    H, W, C = img.shape
    n_pix = H * W
    s = torch.empty(C, dtype=torch.float64, device=img.device)
    c = torch.empty(C, dtype=torch.int64, device=img.device)
    ws = WS.get("nz", N.query("mw_nz_stats_ws_bytes", n_pix, C))
    with profiling.timed("nz_stats", n_pix * C * img.element_size()):
        N.call("mw_nz_stats", P(img), dtype_code(img), n_pix, C, P(s), P(c), P(ws), stream())
    return s, c


def lognorm(img: torch.Tensor, inv_mean: torch.Tensor, pseudoval: float, out=None):
    H, W, C = img.shape
    if out is None:
        out = torch.empty((H, W, C), dtype=torch.float32, device=img.device)
    N.call("mw_lognorm", P(img), dtype_code(img), H * W, C, P(inv_mean), float(pseudoval),
           P(out), stream())
    return out


def gaussian_taps(sigma: float, truncate: float = 4.0) -> np.ndarray:
    """scipy ``_gaussian_kernel1d`` order 0 (radius int(truncate*sigma+0.5)),
    computed in fp64 then rounded to fp32 for the kernel."""
    r = int(truncate * float(sigma) + 0.5)
    x = np.arange(-r, r + 1, dtype=np.float64)
    phi = np.exp(-0.5 / (float(sigma) * float(sigma)) * x * x)
    return (phi / phi.sum())[::-1].astype(np.float32).copy()  # correlate1d(weights[::-1])


def blur(img: torch.Tensor, sigma: float, inv_mean=None, pseudoval: float = 1.0, out=None,
         truncate: float = 4.0):
    H, W, C = img.shape
    w = gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    if out is None:
        out = torch.empty((H, W, C), dtype=torch.float32, device=img.device)
    wsb = N.query("mw_blur_ws_bytes", H, W, C, r)
    ws = WS.get("blur", wsb) if wsb else None
    with profiling.timed("blur", H * W * C * (img.element_size() + 4)):
        N.call("mw_blur", P(img), dtype_code(img), H, W, C, P(inv_mean), float(pseudoval),
               w.ctypes.data, r, P(out), P(ws), stream())
    return out


def block_mean(img: torch.Tensor, fact: int):
    H, W, C = img.shape
    Ho, Wo = -(-H // fact), -(-W // fact)
    out = torch.empty((Ho, Wo, C), dtype=torch.float32, device=img.device)
    N.call("mw_block_mean", P(img), dtype_code(img), H, W, C, int(fact), P(out), stream())
    return out


class RankIndex:
    """The mask rank of a slide as the compact index of mw_mask_rank_index
    (per 64-pixel word: mask bits and the tissue pixels before it; ~n/6
    bytes): the kernels map a tissue rank to its pixel through it (+
    ``pix_off``, the pixel offset of a band inside a larger array)."""

    def __init__(self, buf: torch.Tensor, n_pix: int, pix_off: int = 0):
        self.buf, self.n_pix, self.pix_off = buf, int(n_pix), int(pix_off)

    def offset(self, k: int) -> "RankIndex":
        return RankIndex(self.buf, self.n_pix, self.pix_off + int(k))

    def __getitem__(self, sl):  # r2p[:M] of the table form: the index covers every rank
        return self


# The rank -> pixel table (mw_mask_rank, 4 bytes per tissue pixel: one lookup
# per draw, the faster gather -- config 2: 1.67 vs 1.81 ms) for slides up to
# RANK_TABLE_MAX_PIX pixels (1 GiB of table); the compact index above (config
# 5's 40k x 40k slide: 0.27 GB instead of 6.4 GB).  MW_RANK_TABLE=1 / 0 forces
# the table / the index.  (Round 5, MW_GATHER_PX=1 with the index: the draws
# turned into pixels beside the blur, then a lookup-free gather: gather 1.59
# -> 1.22 ms, but the 17M index lookups take 1.2 ms on the side stream and
# slow the blur by 0.65 ms: the step is unchanged, 17.65 vs 17.68 ms.)
_RT = os.environ.get("MW_RANK_TABLE")
RANK_TABLE_MAX_PIX = (1 << 62) if _RT == "1" else 0 if _RT == "0" else (1 << 28)


def mask_rank_async(mask_u8: torch.Tensor):
    """Launch the mask rank (no host sync): (the rank→pixel int32 table of
    length n -- a RankIndex above RANK_TABLE_MAX_PIX pixels --, device count
    of mask != 0)."""
    n = mask_u8.numel()
    cnt = torch.empty(1, dtype=torch.int64, device=mask_u8.device)
    ws = WS.get("mrank", N.query("mw_mask_rank_ws_bytes", n))
    if n <= RANK_TABLE_MAX_PIX:
        r2p = torch.empty(n, dtype=torch.int32, device=mask_u8.device)
        with profiling.timed("mask_rank", n):
            N.call("mw_mask_rank", P(mask_u8), n, P(r2p), P(cnt), P(ws), stream())
    else:
        buf = torch.empty(N.query("mw_rank_index_bytes", n), dtype=torch.uint8, device=mask_u8.device)
        with profiling.timed("mask_rank", n):
            N.call("mw_mask_rank_index", P(mask_u8), n, P(buf), P(cnt), P(ws), stream())
        r2p = RankIndex(buf, n)
    # the count comes back by its own copy and event, so reading it later
    # does not wait for work queued after the rank (e.g. the blur)
    slot = _PINNED.take(8)
    slot[1] = _Busy
    hv = slot[0][:8].view(torch.int64)
    hv.copy_(cnt, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return r2p, cnt, (slot, hv, ev)


def mask_rank(mask_u8: torch.Tensor, pending=None):
    """(RankIndex or rank→pixel int32 tensor of length M, M) for mask != 0
    (row-major); ``pending`` = an earlier mask_rank_async result for the same
    mask."""
    r2p, cnt, (slot, hv, ev) = mask_rank_async(mask_u8) if pending is None else pending
    ev.synchronize()
    M = int(hv[0])
    slot[1] = None
    return r2p[:M], M


def gather_rows(img_f32: torch.Tensor, feat: torch.Tensor, idx: torch.Tensor, r2p: torch.Tensor,
                X_out: torch.Tensor, stats: torch.Tensor, accumulate: bool, absmax=None):
    """X_out[j] = img[r2p[idx[j]], feat] (``r2p`` None: idx holds the pixels,
    rank_to_pixel); Chan-merge column stats into ``stats`` = [n, mean[F],
    M2[F]] (fp64); max |x| per column maxed into ``absmax`` (fp32 [F],
    optional)."""
    H, W, C = img_f32.shape
    S, F = X_out.shape
    if S == 0:
        return
    ws = WS.get("gather", N.query("mw_gather_ws_bytes", S, F))
    with profiling.timed("gather", S * (F * 4 * 2 + 8)):
        if r2p is None:
            N.call("mw_gather_rows_px", P(img_f32), C, P(feat), F, P(idx), S, P(X_out), P(ws), stream())
        elif isinstance(r2p, RankIndex):
            N.call("mw_gather_rows_ri", P(img_f32), C, P(feat), F, P(idx), P(r2p.buf), r2p.n_pix, r2p.pix_off,
                   S, P(X_out), P(ws), stream())
        else:
            N.call("mw_gather_rows", P(img_f32), C, P(feat), F, P(idx), P(r2p), S, P(X_out), P(ws),
                   stream())
    N.call("mw_col_stats_finalize", P(ws), S, F, P(stats), 1 if accumulate else 0, stream())
    if absmax is not None:
        N.call("mw_col_stats_absmax", P(ws), S, F, P(absmax), 1, stream())


def rank_to_pixel(idx: torch.Tensor, index: "RankIndex"):
    """idx[j] (tissue ranks, int32) -> their pixels (+ index.pix_off), in place."""
    S = idx.numel()
    if S:
        with profiling.timed("rank_to_pixel", S * 8):
            N.call("mw_rank_to_pixel_ri", P(idx), S, P(index.buf), index.n_pix, index.pix_off, stream())
    return idx


def col_stats_rows(X: torch.Tensor, stats: torch.Tensor, accumulate: bool, absmax=None):
    """Column statistics of rows already in ``X`` (the records mw_gather_rows
    would produce for the same rows), Chan-merged into ``stats``."""
    S, F = X.shape
    if S == 0:
        return
    ws = WS.get("gather", N.query("mw_gather_ws_bytes", S, F))
    with profiling.timed("col_stats", S * F * 4):
        N.call("mw_col_stats_rows", P(X), S, F, P(ws), stream())
    N.call("mw_col_stats_finalize", P(ws), S, F, P(stats), 1 if accumulate else 0, stream())
    if absmax is not None:
        N.call("mw_col_stats_absmax", P(ws), S, F, P(absmax), 1, stream())


# deferred-blur paths taken (tests read it); *_streamed: over a slide read band by band (stream.py)
FUSED_USED = {"sample": 0, "assign": 0, "assign_banded": 0, "sample_streamed": 0, "assign_streamed": 0,
              "nz_streamed": 0}


def defer_blur(H: int, W: int, C: int) -> bool:
    """Whether ``img.blurring`` defers the Gaussian into the fused epilogues
    (subsample gather and label pass recompute it from the raw slide, the
    fp32 blurred slide is never stored).  ``MW_FUSED_BLUR`` = 1 / 0 forces
    it; by default ("auto") only when the fp32 slide would take more than
    half of the free HBM -- at config 2 materialising is faster (the label
    pass then reads 4 bytes per element instead of recomputing 17x17 taps)."""
    mode = os.environ.get("MW_FUSED_BLUR", "auto")
    if mode in ("0", "1"):
        return mode == "1"
    free, _ = torch.cuda.mem_get_info()
    return H * W * C * 4 > free // 2


def padded_mask(mask_u8: torch.Tensor, pad: int = 256) -> torch.Tensor:
    """``mask_u8`` in a buffer readable ``pad`` bytes past its end (the fused
    assign epilogue DMAs whole 1-KB pieces of mask rows)."""
    n = mask_u8.numel()
    st = mask_u8.untyped_storage()
    if mask_u8.is_contiguous() and st.nbytes() - mask_u8.storage_offset() >= n + pad:
        return mask_u8
    buf = torch.zeros(n + pad, dtype=torch.uint8, device=mask_u8.device)
    buf[:n].copy_(mask_u8.reshape(-1))
    return buf[:n].view(mask_u8.shape)


def blur_gather_fused(img: torch.Tensor, sigma: float, inv_mean, pseudoval: float,
                      feat: torch.Tensor, idx: torch.Tensor, r2p: torch.Tensor, X_out: torch.Tensor,
                      truncate: float = 4.0) -> bool:
    """X_out[j] = blur(lognorm(img))[r2p[idx[j]], feat] without storing the
    blurred slide (stream.blur_gather over the resident slide as one band):
    sample map (per pixel its first two sample slots, later draws on an
    overflow list) → blur with the sample epilogue, which writes both table
    slots → overflow copies.  False (nothing done) when nothing is sampled."""
    from .stream import blur_gather

    return blur_gather(img, sigma, inv_mean, pseudoval, feat, idx, r2p, X_out, truncate)


def synth_slide(H, W, C, seed, mode="hard"):
    """Benchmark input generated on device (SURVEY §8d shape): uint16 HWC
    (int16 storage) + uint8 mask."""
    from .stream import _synth_params

    syx, prof, shape, bg_rows, n_seeds, n_domains = _synth_params(H, W, C, seed, mode)
    dev = device()
    d_syx = torch.from_numpy(syx.ravel()).to(dev)
    d_prof = torch.from_numpy(prof.ravel()).to(dev)
    img = torch.empty((H, W, C), dtype=torch.int16, device=dev)
    mask = torch.empty((H, W), dtype=torch.uint8, device=dev)
    N.call("mw_synth_slide", H, W, C, P(d_syx), n_seeds, P(d_prof), n_domains, shape,
           bg_rows, int(seed) & 0xFFFFFFFFFFFFFFFF, P(img), P(mask), stream())
    return img, mask
