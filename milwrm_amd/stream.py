"""Slide residency in HBM and row-band streaming of slides that are not resident.

SURVEY §7 step 8 / BASELINE config 5: a cohort of 16 slides of 40k x 40k x 50
uint16 is 160 GB of raw pixels per slide.  One MI355X (288 GB of HBM) holds
one such slide, not the two per GPU of an 8-GPU node beside the ~55 GB of
clustering rows each slide contributes.  The reference keeps every image as a
float64 host array (MxIF.py:147) and walks the images one at a time, for the
preparation (MILWRM.py:1718-1733) and again for the labels (:1789-1794).
Here:

* the raw pixels of an image a host array backs are uploaded whole while
  they fit the HBM budget (``MW_HBM_BUDGET`` bytes, e.g. ``64G``; default
  half of the device memory), least recently used first out: an upload that
  does not fit evicts older such copies (their host arrays stay), and so
  does a pass that needs HBM for its own buffers (``Residency.release``);
* an image that is not resident is STREAMED: every pass that needs its
  pixels (non-zero statistics, blur + subsample, blur + label/confidence,
  the QC sums) reads it as row bands (``band_rows`` rows plus the blur's
  halo rows above and below), double-buffered: band b+1 is read on a side
  stream (host-to-device copy, or the synthetic generator standing in for a
  slide reader) while band b is processed;
* the kernels compute every output value from the same input rows in the
  same order whichever band holds it (the fused blur epilogues take an output
  row window: mw_blur_sample_rows / mw_blur_assign_rows; the non-zero sums of
  integer slides are exact integers), so a streamed slide gives bit for bit
  the resident slide's results (tests/test_gpu_stream.py).

Sources (``RowSource``): ``DeviceSource`` (a resident tensor; its bands are
views, no copy), ``HostSource`` (a host array: pinned memory -- e.g.
``pinned_empty`` -- is copied asynchronously, pageable memory through the
runtime's staging), ``SynthSource`` (the benchmark's synthetic slide
generated band by band on the device, bit for bit ``device.synth_slide``).
"""
from __future__ import annotations

import os
import weakref
from collections import OrderedDict

import numpy as np
import torch

from . import _native as N
from . import device as D
from . import profiling


# ------------------------------------------------------------------ budget

def _parse_bytes(s: str) -> int:
    s = s.strip().upper()
    mult = 1
    for suf, m in (("T", 1 << 40), ("G", 1 << 30), ("M", 1 << 20), ("K", 1 << 10)):
        if s.endswith(suf):
            s, mult = s[:-1], m
            break
    return int(float(s) * mult)


def hbm_budget(dev=None) -> int:
    """Bytes of HBM that host-backed raw slides may occupy together."""
    env = os.environ.get("MW_HBM_BUDGET")
    if env:
        return _parse_bytes(env)
    dev = torch.cuda.current_device() if dev is None else dev
    return int(torch.cuda.get_device_properties(dev).total_memory // 2)


def free_bytes(dev=None) -> int:
    """Free HBM including what torch's caching allocator holds unused.  (The
    allocator's two counters are read from its raw statistics: the public
    memory_reserved / memory_allocated flatten ~300 statistics into a dict
    each call, ~0.1 ms apiece, on the host path between the prep and the fit.)"""
    dev = torch.cuda.current_device() if dev is None else dev
    free, _ = torch.cuda.mem_get_info(dev)
    st = torch.cuda.memory.memory_stats_as_nested_dict(dev)
    return int(free + st["reserved_bytes"]["all"]["current"] - st["allocated_bytes"]["all"]["current"])


def alloc_bytes(dev=None) -> int:
    """Bytes ONE new allocation can get: the device's free memory plus the
    cached segments the allocator can hand back whole.  ``free_bytes`` also
    counts the unused remainders of split segments (a segment partly in use
    cannot be released), which no single large block can use: a 28.7 GiB band
    buffer sized against 24.9 GiB free + 25.1 GiB of such cache failed."""
    dev = torch.cuda.current_device() if dev is None else dev
    free, _ = torch.cuda.mem_get_info(dev)
    st = torch.cuda.memory.memory_stats_as_nested_dict(dev)
    cached = st["reserved_bytes"]["all"]["current"] - st["allocated_bytes"]["all"]["current"]
    split = st.get("inactive_split_bytes", {}).get("all", {}).get("current", 0)
    return int(free + max(0, cached - split))


def alloc_rows(rows: int, row_shape, dtype, min_rows: int = 1, dev=None) -> torch.Tensor:
    """``torch.empty((rows, *row_shape))`` for a band buffer whose height is a
    choice, not a requirement: on an allocation failure the cache is emptied
    and the height halved (down to ``min_rows``, then the error propagates).
    The caller reads the height it got from the tensor."""
    dev = D.device() if dev is None else dev
    rows = max(int(rows), int(min_rows), 1)
    while True:
        try:
            return torch.empty((rows, *row_shape), dtype=dtype, device=dev)
        except torch.OutOfMemoryError:
            if D.WS.drop():  # the passes' cached scratch first, at the same height
                torch.cuda.empty_cache()
                continue
            if rows <= min_rows:
                raise
            torch.cuda.empty_cache()
            rows = max(int(min_rows), rows // 2)


class Residency:
    """LRU of images whose raw pixels were uploaded whole from a host array
    (the only device copies that can be dropped and read again)."""

    def __init__(self):
        self._lru = OrderedDict()  # id(img) -> [weakref, nbytes]
        self.evictions = 0

    def _live(self):
        for key in [k for k, (r, _) in self._lru.items() if r() is None]:
            del self._lru[key]
        return self._lru

    def used(self) -> int:
        return sum(n for _, n in self._live().values())

    def register(self, im, nbytes: int):
        self._lru[id(im)] = [weakref.ref(im), int(nbytes)]
        self._lru.move_to_end(id(im))

    def touch(self, im):
        if id(im) in self._lru:
            self._lru.move_to_end(id(im))

    def forget(self, im):
        self._lru.pop(id(im), None)

    def _evict_oldest(self, keep=None) -> bool:
        for key, (ref, _) in list(self._live().items()):
            im = ref()
            if im is None or im is keep:
                continue
            del self._lru[key]
            im._evict()
            self.evictions += 1
            return True
        return False

    def admit(self, im, nbytes: int) -> bool:
        """Whether ``im``'s raw pixels (``nbytes``) may be uploaded whole now;
        evicts least recently used copies to make room.  False: stream it."""
        if nbytes > hbm_budget():
            return False
        while self.used() + nbytes > hbm_budget():
            if not self._evict_oldest(keep=im):
                return False
        while nbytes + (256 << 20) > alloc_bytes():
            if not self._evict_oldest(keep=im):
                return False
        return True

    def release(self, need: int) -> int:
        """Drop the passes' cached scratch (``device.WS``), then evict resident
        slides, until ``need`` bytes can be allocated (``alloc_bytes``: free
        memory plus the allocator's whole cached segments) or nothing is left
        to free; returns those bytes."""
        if alloc_bytes() < need and D.WS.drop():
            torch.cuda.empty_cache()
        while alloc_bytes() < need and self._evict_oldest():
            pass
        return alloc_bytes()


RESIDENCY = Residency()


# ----------------------------------------------------------------- sources

def device_dtype_of(a: np.ndarray) -> torch.dtype:
    """The element type ``device.to_device_image`` would give ``a``."""
    if a.dtype in (np.uint8, np.bool_):
        return torch.uint8
    if a.dtype == np.uint16:
        return torch.int16
    if np.issubdtype(a.dtype, np.integer) and a.size and a.min() >= 0 and a.max() <= 65535:
        return torch.int16
    return torch.float32


class RowSource:
    """An H x W x C raw slide whose rows are read on demand (device element
    type ``dtype``: uint8, int16 holding uint16 bits, or float32)."""

    H = W = C = 0
    dtype = torch.int16
    zero_copy = False  # bands are views of resident memory (no buffers, no copies)
    kind = "rows"

    @property
    def shape(self):
        return (self.H, self.W, self.C)

    @property
    def row_bytes(self) -> int:
        return self.W * self.C * torch.empty(0, dtype=self.dtype).element_size()

    def read(self, y0: int, y1: int, out: torch.Tensor) -> torch.Tensor:
        """Rows [y0, y1) into ``out`` (a device tensor of >= y1 - y0 rows),
        enqueued on the current stream; returns the filled rows."""
        raise NotImplementedError

    def mask_device(self):
        """The slide's mask as a device uint8 tensor, if the source has one."""
        return None

    def materialize(self) -> torch.Tensor:
        out = torch.empty(self.shape, dtype=self.dtype, device=D.device())
        return self.read(0, self.H, out)


class DeviceSource(RowSource):
    """A slide resident in HBM (HWC tensor)."""

    zero_copy = True
    kind = "device"

    def __init__(self, t: torch.Tensor):
        self.t = t
        self.H, self.W, self.C = (int(x) for x in t.shape)
        self.dtype = t.dtype

    def read(self, y0, y1, out=None):
        return self.t[y0:y1]


class HostSource(RowSource):
    """A slide in host memory: a numpy array or CPU tensor (HWC or HW), or a
    list of CPU tensors holding consecutive row ranges (e.g. page-locked
    chunks, ``pinned_rows``)."""

    kind = "host"

    def __init__(self, arr):
        self._chunks = None
        if isinstance(arr, (list, tuple)):
            self._chunks = [t if t.dim() == 3 else t[:, :, None] for t in arr]
            self.H = sum(int(t.shape[0]) for t in self._chunks)
            _, self.W, self.C = (int(x) for x in self._chunks[0].shape)
            self.dtype = self._chunks[0].dtype
            self._starts = np.cumsum([0] + [int(t.shape[0]) for t in self._chunks])
            self._t = self._a = None
        elif isinstance(arr, torch.Tensor):
            t = arr if arr.dim() == 3 else arr[:, :, None]
            self.H, self.W, self.C = (int(x) for x in t.shape)
            self.dtype = t.dtype
            self._t, self._a = t, None
        else:
            a = np.asarray(arr)
            a = a if a.ndim == 3 else a[:, :, None]
            self.H, self.W, self.C = a.shape
            self.dtype = device_dtype_of(a)
            self._t, self._a = None, a
        self._keep = []

    def _host_rows(self, y0, y1) -> torch.Tensor:
        if self._t is not None:
            return self._t[y0:y1]
        a = self._a[y0:y1]
        if self.dtype == torch.uint8:
            a = a if a.dtype == np.uint8 else a.astype(np.uint8)
        elif self.dtype == torch.int16:
            a = (a if a.dtype == np.uint16 else a.astype(np.uint16)).view(np.int16)
        else:
            a = a if a.dtype == np.float32 else a.astype(np.float32)
        return torch.from_numpy(np.ascontiguousarray(a))

    def read(self, y0, y1, out):
        dst = out[:y1 - y0]
        if self._chunks is not None:
            for i, t in enumerate(self._chunks):
                a, b = max(y0, int(self._starts[i])), min(y1, int(self._starts[i + 1]))
                if a < b:
                    dst[a - y0:b - y0].copy_(t[a - self._starts[i]:b - self._starts[i]], non_blocking=True)
            return dst
        h = self._host_rows(y0, y1)
        dst.copy_(h, non_blocking=True)
        if not h.is_pinned():
            self._keep = [h]  # (a pageable copy is staged by the runtime before it returns)
        return dst


def pinned_empty(shape, dtype=torch.int16) -> torch.Tensor:
    """Page-locked host tensor: bands of a HostSource over it are copied by
    DMA without a staging copy."""
    return torch.empty(shape, dtype=dtype, pin_memory=True)


def pinned_rows(src: RowSource, chunk_bytes: int = 1 << 30, progress=None) -> list:
    """The rows of ``src`` copied into page-locked host chunks of about
    ``chunk_bytes`` (a ``HostSource`` over the list reads them back by DMA)."""
    rows = max(1, chunk_bytes // src.row_bytes)
    buf = torch.empty((min(rows, src.H), src.W, src.C), dtype=src.dtype, device=D.device())
    out = []
    for y0 in range(0, src.H, rows):
        y1 = min(src.H, y0 + rows)
        h = torch.empty((y1 - y0, src.W, src.C), dtype=src.dtype, pin_memory=True)
        h.copy_(src.read(y0, y1, buf))
        out.append(h)
        if progress:
            progress(y1)
    return out


# generator modes: (lognormal spread of the domain profiles, gamma shape of
# the noise); "design" overlaps the domains so that the k = 8 fit runs near
# SURVEY 8d's I = 17 Lloyd iterations (MW_SYNTH_SPREAD overrides its spread)
SYNTH_MODES = {"hard": (0.15, 1), "easy": (0.8, 4), "design": (0.07, 1)}


def synth_mode(mode):
    sp_, shape = SYNTH_MODES[mode]
    if mode == "design" and os.environ.get("MW_SYNTH_SPREAD"):
        sp_ = float(os.environ["MW_SYNTH_SPREAD"])
    return sp_, shape


def _synth_params(H, W, C, seed, mode="hard", n_seeds=32, n_domains=8, bg_frac=0.15):
    rng = np.random.default_rng(seed)
    sp_, shape = synth_mode(mode)
    syx = np.stack([rng.uniform(0, H, n_seeds), rng.uniform(0, W, n_seeds)], 1).astype(np.float32)
    prof = rng.lognormal(4.0, sp_, size=(n_domains, C)).astype(np.float32)
    return syx, prof, shape, int(round(bg_frac * H)), n_seeds, n_domains


class SynthSource(RowSource):
    """The benchmark's synthetic slide (``device.synth_slide``)
    generated band by band on the device: the stand-in for a slide reader
    (every value is a hash of its slide pixel index, so any band is bit for
    bit those rows of the whole slide)."""

    kind = "synth"

    def __init__(self, H, W, C, seed, mode="hard"):
        self.H, self.W, self.C = int(H), int(W), int(C)
        self.dtype = torch.int16
        self.seed = int(seed)
        syx, prof, self.shape_k, self.bg_rows, self.n_seeds, self.n_domains = _synth_params(H, W, C, seed, mode)
        dev = D.device()
        self._syx = torch.from_numpy(syx.ravel()).to(dev)
        self._prof = torch.from_numpy(prof.ravel()).to(dev)

    def read(self, y0, y1, out, mask_out=None):
        dst = out[:y1 - y0]
        N.call("mw_synth_rows", self.H, self.W, self.C, int(y0), int(y1), D.P(self._syx), self.n_seeds,
               D.P(self._prof), self.n_domains, self.shape_k, self.bg_rows,
               self.seed & 0xFFFFFFFFFFFFFFFF, D.P(dst), D.P(mask_out), D.stream())
        return dst

    def mask_device(self):
        m = torch.ones((self.H, self.W), dtype=torch.uint8, device=D.device())
        m[:self.bg_rows] = 0
        return m


# ------------------------------------------------------------------- bands

def band_rows_for(src: RowSource, extra_per_row: int = 0) -> int:
    """Rows per streamed band: ``MW_STREAM_BAND_ROWS``, else about
    ``MW_STREAM_BAND_BYTES`` (default 4 GiB) of raw rows plus ``extra_per_row``
    bytes of the pass's own per-row buffers."""
    env = os.environ.get("MW_STREAM_BAND_ROWS")
    if env:
        return max(1, min(int(env), src.H))
    target = _parse_bytes(os.environ.get("MW_STREAM_BAND_BYTES", "4G"))
    return max(1, min(src.H, target // max(1, src.row_bytes + extra_per_row)))


_SIDE = {}


def _side_stream(dev) -> torch.cuda.Stream:
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


def _plan(H, band_rows, halo, r0, r1):
    plan = []
    for y0 in range(r0, r1, max(1, band_rows)):
        y1 = min(r1, y0 + band_rows)
        plan.append((y0, y1, max(0, y0 - halo), min(H, y1 + halo)))
    return plan


def bands(src: RowSource, band_rows: int, halo: int, r0: int = 0, r1=None):
    """Yield (y0, y1, a, raw): output rows [y0, y1) of [r0, r1) in bands of
    ``band_rows``, ``raw`` = the device rows [a, a + len(raw)) = [y0 - halo,
    y1 + halo) clipped to the slide.  A resident source yields views; any
    other is read into two buffers, band b+1 on a side stream while the
    caller's work on band b runs on the current stream.  When HBM cannot hold
    two buffers of ``band_rows`` + 2 halo rows, the bands get lower
    (``alloc_rows``); every output row is computed the same way whatever
    band holds it.  The side stream's reads are ordered before the main
    stream's later work also when the consumer stops early (an exception, or
    a caller that abandons the generator), so the buffers are never handed
    back to the allocator while a read into them is in flight."""
    H = src.H
    r1 = H if r1 is None else r1
    plan = _plan(H, band_rows, halo, r0, r1)
    if src.zero_copy:
        for y0, y1, a, b in plan:
            yield y0, y1, a, src.read(a, b, None)
        return
    if not plan:
        return
    dev = torch.device("cuda", torch.cuda.current_device())
    rows = max(b - a for _, _, a, b in plan)
    nbuf = min(2, len(plan))
    RESIDENCY.release(nbuf * rows * src.row_bytes + (256 << 20))
    lo = min(rows, 2 * halo + 1)
    bufs = [alloc_rows(rows, (src.W, src.C), src.dtype, min_rows=lo, dev=dev)]
    if nbuf > 1:
        bufs.append(alloc_rows(int(bufs[0].shape[0]), (src.W, src.C), src.dtype, min_rows=lo, dev=dev))
    got = min(int(b.shape[0]) for b in bufs)
    while got < rows:  # HBM was short: lower bands into the buffers that could be had
        rows = got
        plan = _plan(H, max(1, got - 2 * halo), halo, r0, r1)
        if len(plan) > 1 and len(bufs) < 2:  # a one-band plan became several: try for a second buffer
            try:
                bufs.append(alloc_rows(got, (src.W, src.C), src.dtype, min_rows=min(got, lo), dev=dev))
            except torch.OutOfMemoryError:
                pass  # one buffer: each read waits until the band before it is consumed
        bufs = bufs[:max(1, min(2, len(plan)))]
        got = min(int(b.shape[0]) for b in bufs)
    nbuf = len(bufs)
    side = _side_stream(dev)
    main = torch.cuda.current_stream()
    ready = [None] * nbuf
    free = [None] * nbuf
    side.wait_stream(main)  # the source's own inputs (e.g. generator tables) queued on main

    def issue(i):
        _, _, a, b = plan[i]
        s = i % nbuf
        if free[s] is not None:
            side.wait_event(free[s])
        with torch.cuda.stream(side):
            with profiling.timed(f"read_{src.kind}", (b - a) * src.row_bytes):
                src.read(a, b, bufs[s])
            ev = torch.cuda.Event()
            ev.record(side)
        ready[s] = ev

    try:
        issue(0)
        for i, (y0, y1, a, b) in enumerate(plan):
            if nbuf > 1 and i + 1 < len(plan):  # the next band into the other buffer, now
                issue(i + 1)
            s = i % nbuf
            main.wait_event(ready[s])
            yield y0, y1, a, bufs[s][:b - a]
            ev = torch.cuda.Event()
            ev.record(main)
            free[s] = ev
            if nbuf == 1 and i + 1 < len(plan):  # one buffer: after this band's consumers
                issue(i + 1)
    finally:
        main.wait_stream(side)


def as_source(x) -> RowSource:
    return x if isinstance(x, RowSource) else DeviceSource(x)


# ------------------------------------------------------------ band passes

def nz_stats(src: RowSource):
    """``device.nz_stats`` of a slide band after band: per-channel sums (fp64)
    and counts (int64) added on the device.  For uint8 / uint16 slides every
    band's sums are exact integers, so the totals are the whole slide's bits."""
    src = as_source(src)
    if src.zero_copy:
        return D.nz_stats(src.read(0, src.H, None))
    dev = D.device()
    s = torch.zeros(src.C, dtype=torch.float64, device=dev)
    c = torch.zeros(src.C, dtype=torch.int64, device=dev)
    for _, _, _, raw in bands(src, band_rows_for(src), 0):
        sb, cb = D.nz_stats(raw)
        s += sb
        c += cb
    return s, c


def blur_gather(src, sigma: float, inv_mean, pseudoval: float, feat: torch.Tensor, idx: torch.Tensor,
                r2p, X_out: torch.Tensor, truncate: float = 4.0, band_rows=None) -> bool:
    """X_out[j] = blur(lognorm(slide))[pixel of rank idx[j], feat] (``r2p``: a
    device.RankIndex or a rank -> pixel table) without storing the
    blurred slide (``img.subsample_pixels`` after a deferred blur,
    MxIF.py:457-492): the sample map (per pixel its first two sample slots,
    later draws on an overflow list), then per band the blur with its sample
    epilogue over the band's output rows (mw_blur_sample_rows) -- or, for a
    shape the fused kernel does not take, the band blurred into fp32 and its
    sampled pixels copied out (mw_slot_gather) -- then the overflow copies.
    A resident slide is one band.  False when nothing was sampled."""
    src = as_source(src)
    H, W, C = src.shape
    S, F = X_out.shape
    if S == 0:
        return False
    w = D.gaussian_taps(sigma, truncate)
    r = (len(w) - 1) // 2
    n = H * W
    slots = D.WS.get("sample_slots", 4 * N.query("mw_sample_slot_elems", n))
    ovf = D.WS.get("sample_ovf", 4 * (S + 1))
    st = D.stream()
    ri = isinstance(r2p, D.RankIndex)
    with profiling.timed("sample_map", S * 16):
        if ri:
            N.call("mw_sample_map_ri", D.P(idx), D.P(r2p.buf), r2p.n_pix, r2p.pix_off, S, n, D.P(slots),
                   D.P(ovf), st)
        else:
            N.call("mw_sample_map", D.P(idx), D.P(r2p), S, n, D.P(slots), D.P(ovf), st)
    elem = torch.empty(0, dtype=src.dtype).element_size()
    if band_rows is None:
        band_rows = H if src.zero_copy else band_rows_for(src)
    fused = True
    fbuf = None
    for y0, y1, a, raw in bands(src, band_rows, r):
        hb = int(raw.shape[0])
        if fused:
            # algorithmic bytes: the band's raw rows + its share of the sampled rows written
            with profiling.timed("blur_sample", (y1 - y0) * W * C * elem + S * F * 4 * (y1 - y0) / H):
                fused = N.try_call("mw_blur_sample_rows", D.P(raw), D.dtype_code(raw), hb, W, C, a, y0 - a,
                                   y1 - a, D.P(inv_mean), float(pseudoval), w.ctypes.data, r, D.P(slots), S,
                                   D.P(feat), F, D.P(X_out), D.stream())
            if fused:
                continue
        # the fused kernel does not take this shape: blur the band into fp32
        if fbuf is None:  # (bands no higher than the raw band just read)
            fbuf = torch.empty((min(H, max(band_rows + 2 * r, hb)), W, C), dtype=torch.float32,
                               device=raw.device)
        out = fbuf[:hb]
        D.blur(raw, sigma, inv_mean=inv_mean, pseudoval=pseudoval, out=out, truncate=truncate)
        core = out[y0 - a:y1 - a]
        with profiling.timed("slot_gather", (y1 - y0) * W * 8):
            N.call("mw_slot_gather", D.P(core), C, (y1 - y0) * W, y0 * W, D.P(slots), S, D.P(feat), F,
                   D.P(X_out), D.stream())
    with profiling.timed("sample_overflow", 0):
        if ri:
            N.call("mw_sample_overflow_ri", D.P(idx), D.P(r2p.buf), r2p.n_pix, r2p.pix_off, D.P(slots), D.P(ovf),
                   S, F, D.P(X_out), D.stream())
        else:
            N.call("mw_sample_overflow", D.P(idx), D.P(r2p), D.P(slots), D.P(ovf), S, F, D.P(X_out), D.stream())
    D.FUSED_USED["sample"] += 1
    if not src.zero_copy:
        D.FUSED_USED["sample_streamed"] += 1
    return True
