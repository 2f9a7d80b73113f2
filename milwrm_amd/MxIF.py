"""``img``: the MxIF image container of MILWRM (MxIF.py:125-589), re-designed
around HBM residency.

The pixels live on the GPU in HWC layout with a compact element type (the raw
uint8/uint16 planes as read from TIFFs, or fp32 once transformed); ``.img``
materialises the reference's float64 host array only when someone reads it.
``log_normalize`` is deferred and fused into the Gaussian blur kernel (one
HBM pass: raw → log10(x/mean+1) → 17-tap separable blur → fp32).  All
arithmetic runs in the HIP kernels of ``csrc/``; there is no CPU fallback.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import device as D
from .rng import check_total, set_global_state_after_draws, subsample_indices_device


def checktype(obj):
    """True for a non-empty iterable of str (MxIF.py:25-26)."""
    return bool(obj) and all(isinstance(elem, str) for elem in obj)


def _out_of_scope(name):
    def f(*a, **k):
        raise NotImplementedError(f"{name} is outside the MI355X hot path (plotting / intensity "
                                  "utilities); use the reference implementation")
    f.__name__ = name
    return f


clip_values = _out_of_scope("clip_values")
scale_rgb = _out_of_scope("scale_rgb")
CLAHE = _out_of_scope("CLAHE")


class _DeviceMask:
    """Host-side stand-in for a mask that lives in HBM (materialised on use)."""

    def __init__(self, t):
        self._t = t
        self.shape = tuple(t.shape)
        self.dtype = np.dtype(np.uint8)

    def __array__(self, dtype=None, copy=None):
        a = self._t.cpu().numpy()
        return a if dtype is None else a.astype(dtype)

    def copy(self):
        return _DeviceMask(self._t.clone())


class img:
    def __init__(self, img_arr, channels=None, mask=None):
        """Same validation and attributes as MxIF.py:126-167 (``img``, ``n_ch``,
        ``ch``, ``mask``); the pixels are uploaded lazily."""
        assert img_arr.ndim > 1, "Image does not have enough dimensions: {} given".format(img_arr.ndim)
        self._ndim = img_arr.ndim
        self._host = np.asarray(img_arr)
        self._host64 = None
        self._dev = None            # HWC device tensor (authoritative when set)
        self._pending = None        # (inv_mean fp32 device tensor, pseudoval) deferred log_normalize
        self._pending_blur = None   # (sigma, truncate) deferred gaussian (fused-epilogue mode)
        self._lognorm_host = None   # (inv_mean fp32 host array, pseudoval) of the pending log_normalize
        self._xbound = None         # per-channel bound on |pixel| of blur(lognorm(raw)), see _blur_bound
        self.n_ch = img_arr.shape[2] if img_arr.ndim > 2 else 1
        if channels is None:
            self.ch = ["ch_{}".format(x) for x in range(self.n_ch)]
        else:
            if not isinstance(channels, list):
                raise Exception("Channels must be given in a list")
            assert len(channels) == self.n_ch, "Number of channels must match img_arr.shape[2]"
            self.ch = channels
        if mask is not None:
            assert mask.shape == img_arr.shape[:2], \
                "Shape of mask must match the first two dimensions of img_arr"
        self.mask = mask
        self._mask_dev = None
        self._band = None  # bands.BandInfo when this img is one row band of a slide
        self._src = None   # stream.RowSource of a slide that is read band by band
        self._hsrc = None  # cached stream.HostSource over _host
        self._revert = None  # how to redo a transformed copy (_transformed / _evict)

    # ----------------------------------------------------------- residency
    # The raw pixels of a host-backed image are uploaded whole while they fit
    # the HBM budget (stream.RESIDENCY, least recently used out); otherwise
    # every pass that needs them streams them in row bands (milwrm_amd.stream)
    @property
    def shape(self):
        if self._dev is not None:
            return tuple(self._dev.shape) if self._ndim > 2 else tuple(self._dev.shape[:2])
        if self._host is None and self._src is not None:
            return self._src.shape if self._ndim > 2 else self._src.shape[:2]
        return self._host.shape

    def _raw_nbytes(self) -> int:
        from .stream import device_dtype_of

        a = self._host
        memo = getattr(self, "_rawb", None)
        if memo is None or memo[0] is not a:
            elem = torch.empty(0, dtype=device_dtype_of(a)).element_size()
            memo = self._rawb = (a, int(a.size) * elem)
        return memo[1]

    def _device(self) -> torch.Tensor:
        """HWC device tensor (uploads on first use; a host-backed upload may
        first evict older resident copies, stream.RESIDENCY)."""
        from .stream import RESIDENCY

        if self._dev is None:
            if self._host is None and self._src is not None:
                src = self._src
                self._fits_whole(src.H * src.row_bytes)
                self._dev = src.materialize()  # an explicit whole-slide read
            else:
                a = self._host if self._host.ndim > 2 else self._host[:, :, None]
                if not RESIDENCY.admit(self, self._raw_nbytes()):
                    self._fits_whole(self._raw_nbytes())  # over the budget: only if HBM holds it
                self._dev = D.to_device_image(a)
            RESIDENCY.register(self, self._dev.numel() * self._dev.element_size())
        else:
            RESIDENCY.touch(self)
        return self._dev

    def _fits_whole(self, nbytes: int):
        """Raise a MemoryError naming the streamed alternative when a
        whole-slide device copy of ``nbytes`` cannot be had even after evicting
        every other resident slide (instead of an allocator failure deep in a
        pass)."""
        from .stream import RESIDENCY, alloc_bytes

        RESIDENCY.release(nbytes + (256 << 20))
        have = alloc_bytes()
        if nbytes + (256 << 20) > have:
            raise MemoryError(
                f"this operation needs the whole raw slide in HBM ({nbytes / 2**30:.1f} GiB) and "
                f"{have / 2**30:.1f} GiB can be allocated: the slide is streamed in row bands instead by "
                f"the passes that take bands (calculate_non_zero_mean, log_normalize + blurring with the "
                f"default batch mean, subsample_pixels, label_tissue_regions, confidence_score_images)")

    def _source(self):
        """None when the raw pixels are resident (or are admitted now: the
        caller then takes ``_device()``); else the ``stream.RowSource`` to read
        them from band by band."""
        from .stream import RESIDENCY, HostSource

        if self._dev is not None:
            RESIDENCY.touch(self)
            return None
        if self._band is not None:  # a slide band (milwrm_amd.bands) stays resident
            return None
        if self._host is None:
            return self._src
        if RESIDENCY.admit(self, self._raw_nbytes()):
            return None
        if self._hsrc is None:
            self._hsrc = HostSource(self._host)
        return self._hsrc

    def _may_hold(self, nbytes: int) -> bool:
        """Whether a device copy of ``nbytes`` may be kept for this image: any
        for an image born on the device; within the HBM budget (evicting older
        copies) for one a host array or a source backs."""
        from .stream import RESIDENCY

        if self._host is None and self._src is None:
            return True
        return RESIDENCY.admit(self, nbytes)

    @classmethod
    def from_source(cls, src, mask=None, channels=None) -> "img":
        """An image whose raw pixels come from a ``stream.RowSource`` band by
        band (never resident whole): a slide reader, a host array, or the
        benchmark's synthetic generator.  ``mask``: host or device H x W
        (default: the source's own mask)."""
        obj = cls.__new__(cls)
        obj._ndim = 3
        obj._host = None
        obj._host64 = None
        obj._dev = None
        obj._pending = None
        obj._pending_blur = None
        obj._lognorm_host = None
        obj._xbound = None
        obj._src = src
        obj._hsrc = None
        obj._revert = None
        obj.n_ch = int(src.C)
        obj.ch = channels if channels is not None else ["ch_{}".format(x) for x in range(obj.n_ch)]
        obj._mask = None
        obj._mask_dev = None
        obj._mrank = None
        obj._band = None
        if mask is None:
            mask = src.mask_device()
        if isinstance(mask, torch.Tensor):
            obj._mask = _DeviceMask(mask)
            obj._mask_dev = D.padded_mask((mask != 0).to(torch.uint8) if mask.dtype != torch.uint8 else mask)
        elif mask is not None:
            assert tuple(mask.shape) == (src.H, src.W), \
                "Shape of mask must match the first two dimensions of img_arr"
            obj._mask = mask
        return obj

    def _materialize(self) -> torch.Tensor:
        """Apply a deferred blur (with its log_normalize fused) or a deferred
        log_normalize (standalone kernel)."""
        if self._pending_blur is not None:
            sigma, truncate = self._pending_blur
            inv, p = self._pending
            self._transformed(lambda: D.blur(self._device(), sigma, inv_mean=inv, pseudoval=p,
                                             truncate=truncate))
        if self._pending is not None:
            inv, p = self._pending
            if inv is None:
                self._pending = None
            else:
                self._transformed(lambda: D.lognorm(self._device(), inv, p))
        return self._device()

    def _transformed(self, make):
        """Replace the pixels by ``make()`` (the pending transforms applied).
        An image backed by a host array or a source keeps how to redo it: its
        transformed copy stays evictable (``_evict`` returns it to the
        deferred state, which gives the same bits, stream.py)."""
        from .stream import RESIDENCY

        backed = self._host is not None or self._src is not None
        state = (self._host, self._src, self._pending, self._pending_blur) if backed else None
        out = make()
        self._pending = None
        self._pending_blur = None
        self._set_device(out)
        if state is not None:
            self._revert = state
            RESIDENCY.register(self, out.numel() * out.element_size())

    def _set_device(self, t: torch.Tensor):
        """The image's pixels are now ``t`` (not a raw copy that could be read
        again: not evictable unless ``_transformed`` records how to redo it)."""
        from .stream import RESIDENCY

        RESIDENCY.forget(self)
        self._dev = t
        self._host64 = None
        self._host = None
        self._src = None
        self._hsrc = None
        self._revert = None

    def _evict(self):
        """Drop the device copy: the raw copy of a host array / source, or a
        transformed copy back to its deferred state."""
        rv = getattr(self, "_revert", None)
        if rv is not None:
            self._host, self._src, self._pending, self._pending_blur = rv
            self._revert = None
            self._host64 = None
        self._dev = None

    @property
    def img(self) -> np.ndarray:
        """The reference's float64 HWC array (materialised from HBM on read)."""
        if self._host64 is None:
            if (self._dev is None and self._host is not None and self._pending is None
                    and self._pending_blur is None):
                self._host64 = self._host.astype("float64")
            else:
                t = self._materialize()
                a = D.to_host_float64(t)
                self._host64 = a if self._ndim > 2 else a[:, :, 0]
        return self._host64

    @img.setter
    def img(self, value):
        from .stream import RESIDENCY

        value = np.asarray(value)
        RESIDENCY.forget(self)
        self._ndim = value.ndim
        self._host = value
        self._host64 = None
        self._dev = None
        self._src = None
        self._hsrc = None
        self._pending = None
        self._pending_blur = None
        self._lognorm_host = None
        self._xbound = None

    @property
    def mask(self):
        return self._mask

    @mask.setter
    def mask(self, m):
        self._mask = m
        self._mask_dev = None
        self._mrank = None

    def _mask_device(self) -> torch.Tensor:
        if self._mask_dev is None:
            if self._mask is None:
                raise AssertionError("No tissue mask available")
            m = np.ascontiguousarray(np.asarray(self._mask) != 0, dtype=np.uint8)
            self._mask_dev = D.padded_mask(torch.from_numpy(m).to(D.device()))
        return self._mask_dev

    def _prefetch_mask_rank(self):
        """Queue the mask rank on the stream without waiting for it (it only
        depends on the mask): it then overlaps the host work between
        calculate_non_zero_mean and subsample_pixels."""
        if getattr(self, "_mrank", None) is None and self._mask is not None:
            self._mrank = D.mask_rank_async(self._mask_device().reshape(-1))

    def _mask_rank(self):
        """(rank→pixel, M) of the current mask, from the prefetched launch if any."""
        pending = getattr(self, "_mrank", None)
        self._mrank = None
        return D.mask_rank(self._mask_device().reshape(-1), pending)

    # -------------------------------------------------------------- basics
    def __repr__(self) -> str:
        descr = "img object with {} of {} and shape {}px x {}px\n".format(
            np.ndarray, np.dtype("float64"), self.shape[0], self.shape[1]
        ) + "{} image channels:\n\t{}".format(self.n_ch, self.ch)
        if self.mask is not None:
            descr += "\n\ntissue mask {} of {} and shape {}px x {}px".format(
                type(self.mask), self.mask.dtype, self.mask.shape[0], self.mask.shape[1])
        return descr

    def copy(self) -> "img":
        new = img.__new__(img)
        new.__dict__.update(self.__dict__)
        new.ch = list(self.ch)
        new._host = None if self._host is None else self._host.copy()
        new._host64 = None if self._host64 is None else self._host64.copy()
        new._dev = None if self._dev is None else self._dev.clone()
        new._hsrc = None
        new._mask = None if self._mask is None else self._mask.copy()
        new._mask_dev = None
        new._mrank = None
        return new

    def _features(self, features):
        if isinstance(features, int):
            features = [features]
        if isinstance(features, str):
            features = [self.ch.index(features)]
        if checktype(features):
            features = [self.ch.index(x) for x in features]
        if features is None:
            features = [x for x in range(self.n_ch)]
        features = [int(f) for f in features]
        for f in features:  # checked on the host: the kernels index channels with them
            if not -self.n_ch <= f < self.n_ch:
                raise IndexError(f"index {f} is out of bounds for axis 2 with size {self.n_ch}")
        return [f % self.n_ch for f in features]

    def __getitem__(self, channels):
        return self.img[:, :, self._features(channels)]

    @classmethod
    def from_device(cls, tensor, mask=None, channels=None) -> "img":
        """Wrap an HWC image already resident in HBM (uint8 / uint16-as-int16 /
        fp32) and an optional device mask (nonzero = tissue)."""
        assert tensor.dim() == 3, "device image must be H x W x C"
        obj = cls.__new__(cls)
        obj._ndim = 3
        obj._host = None
        obj._host64 = None
        obj._dev = tensor
        obj._pending = None
        obj._pending_blur = None
        obj._lognorm_host = None
        obj._xbound = None
        obj.n_ch = int(tensor.shape[2])
        obj.ch = channels if channels is not None else ["ch_{}".format(x) for x in range(obj.n_ch)]
        obj._mask = None
        obj._mask_dev = None
        obj._mrank = None
        obj._band = None
        obj._src = None
        obj._hsrc = None
        obj._revert = None
        if mask is not None:
            obj._mask = _DeviceMask(mask)
            obj._mask_dev = (mask != 0).to(torch.uint8) if mask.dtype != torch.uint8 else mask
        return obj

    # ----------------------------------------------------------------- I/O
    @classmethod
    def from_tiffs(cls, tiffdir, channels, common_strings=None, mask=None):
        """MxIF.py:211-283 (needs an installed TIFF reader: skimage.io)."""
        try:
            from skimage.io import imread
        except ImportError as e:  # pragma: no cover - image has no skimage
            raise ImportError("img.from_tiffs needs scikit-image (skimage.io.imread)") from e
        if common_strings is not None and isinstance(common_strings, str):
            common_strings = [common_strings]
        A = []
        for channel in channels:
            if common_strings is None:
                f = [f for f in os.listdir(tiffdir) if channel in f]
            else:
                f = [f for f in os.listdir(tiffdir) if all(x in f for x in common_strings + [channel])]
            assert len(f) != 0, "No file found with channel {}".format(channel)
            assert len(f) == 1, "More than one match found for file with channel {}".format(channel)
            A.append(imread(os.path.join(tiffdir, f[0])))
        A_arr = np.dstack(A)
        A_mask = None
        if mask is not None:
            f = [f for f in os.listdir(tiffdir) if mask in f]
            assert len(f) != 0, "No tissue mask file found"
            assert len(f) == 1, "More than one match found for tissue mask file"
            A_mask = imread(os.path.join(tiffdir, f[0]))
            assert A_mask.shape == A_arr.shape[:2], \
                "Mask (shape: {}) is not the same shape as marker images (shape: {})".format(
                    A_mask.shape, A_arr.shape[:2])
        return cls(img_arr=A_arr, channels=channels, mask=A_mask)

    @classmethod
    def from_npz(cls, file):
        """MxIF.py:285-309 (no pickles: allow_pickle stays False)."""
        print("Loading img object from {}...".format(file))
        tmp = np.load(file)
        assert "img" in tmp.files, \
            "Unexpected files in .npz: {}, expected ['img','mask','ch'].".format(tmp.files)
        A_mask = tmp["mask"] if "mask" in tmp.files else None
        A_ch = list(tmp["ch"]) if "ch" in tmp.files else None
        return cls(img_arr=tmp["img"], channels=A_ch, mask=A_mask)

    def to_npz(self, file):
        """MxIF.py:311-328."""
        print("Saving img object to {}...".format(file))
        if self.mask is None:
            np.savez_compressed(file, img=self.img, ch=self.ch)
        else:
            np.savez_compressed(file, img=self.img, ch=self.ch, mask=self.mask)

    clip = _out_of_scope("img.clip")
    scale = _out_of_scope("img.scale")
    equalize_hist = _out_of_scope("img.equalize_hist")
    show = _out_of_scope("img.show")
    plot_image_histogram = _out_of_scope("img.plot_image_histogram")

    # ------------------------------------------------------- preprocessing
    def blurring(self, filter_name="gaussian", sigma=2, **kwargs):
        """MxIF.py:375-414.  'gaussian' runs the fused lognorm+blur kernel."""
        if filter_name == "gaussian":
            print("Applying gaussian filter")
            truncate = float(kwargs.pop("truncate", 4.0))
            mode = kwargs.pop("mode", "nearest")
            kwargs.pop("preserve_range", None)
            if mode != "nearest" or kwargs:
                raise NotImplementedError(f"gaussian options {dict(mode=mode, **kwargs)} "
                                          "(only mode='nearest' is implemented)")
            bound = self._blur_bound()
            self._blur_(float(sigma), truncate)
            self._xbound = bound
        elif filter_name == "median":
            # The reference's median branch calls np.ones(sigma, sigma), which
            # raises for any integer sigma (MxIF.py:403); keep that behaviour.
            print("Applying median filter")
            if isinstance(sigma, float):
                sigma = int(sigma)
            np.ones(sigma, sigma)
            raise NotImplementedError("median filter")
        elif filter_name == "bilateral":
            raise NotImplementedError("bilateral filter is outside the MI355X hot path")
        else:
            raise Exception("filter name should be either gaussian, median or bilateral")

    def _raw_int_max(self):
        """The largest value the current pixels' element type holds when they
        are a raw uint8 / uint16 slide (device, host or streamed), else None."""
        if self._pending_blur is not None:
            return None
        if self._dev is not None:
            t = self._dev.dtype
        elif self._host is not None:
            t = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint16): torch.int16}.get(self._host.dtype)
        elif self._src is not None:
            t = self._src.dtype
        else:
            return None
        return {torch.uint8: 255.0, torch.int16: 65535.0}.get(t)  # int16 storage = uint16 bits

    def _blur_bound(self):
        """Per-channel bound on |x| of blur(lognorm(raw)) for a raw integer
        slide, known before any pixel is blurred: log10(x inv + p) is monotone
        in x in [0, dtype max], and the gaussian is a convex combination, so
        |x| <= max(|log10 p|, |log10(max inv + p)|) (max itself without a
        log_normalize), with slack for the fp32 arithmetic.  The exact QC sums
        take their fixed point from it (milwrm_amd.assign._DomainSSE): the
        label pass can then add each band's sums as it labels it, and the
        standalone estimators give the same bits without a first pass for the
        column maxima.  None when the pixels are not such a slide."""
        mx = self._raw_int_max()
        if mx is None:
            return None
        if self._pending is None:
            return np.full(self.n_ch, mx * (1 + 1e-3))
        if self._lognorm_host is None:
            return None
        inv, p = self._lognorm_host
        if not (np.isfinite(p) and p > 0):
            return None
        with np.errstate(invalid="ignore", over="ignore"):
            hi = np.log10(mx * inv.astype(np.float64) + p)
        return np.maximum(abs(np.log10(p)), np.abs(hi)) * (1 + 1e-3) + 1e-30

    def _blur_(self, sigma: float, truncate: float):
        """The gaussian branch of ``blurring``: deferred (streamed slide, or the
        fp32 copy would not fit) or materialised."""
        if self._pending_blur is None and self._source() is not None:
            # not resident: the blur runs inside every pass over the
            # streamed bands (stream.blur_gather, the banded label pass)
            self._pending_blur = (sigma, truncate)
            if self._pending is None:
                self._pending = (None, 1.0)  # no log-normalise before this blur
            self._host64 = None
            return
        src = self._materialize() if self._pending_blur is not None else self._device()
        if self._pending is not None and src.dim() == 3 and (
                D.defer_blur(*src.shape) or not self._may_hold(src.numel() * 4)):
            # fused-epilogue mode: the subsample gather and the label pass
            # recompute the blur from the raw slide (D.defer_blur, or the
            # fp32 copy of a host-backed slide would exceed the HBM budget)
            self._pending_blur = (sigma, truncate)
            self._host64 = None
            return
        self._pending_blur = (sigma, truncate)
        if self._pending is None:
            self._pending = (None, 1.0)
        inv, p = self._pending
        self._transformed(lambda: D.blur(src, sigma, inv_mean=inv, pseudoval=p,
                                         truncate=truncate))

    def log_normalize(self, pseudoval=1, mean=None, mask=True):
        """MxIF.py:416-455: log10(x/mean_c + pseudoval) on every pixel.  The
        transform is deferred and fused into the next blur (or materialised
        when ``.img`` is read)."""
        if mask:
            assert self.mask is not None, "No tissue mask available"
        else:
            print("WARNING: Performing normalization without a tissue mask.")
        if mean is None:
            print("mean calculated to perform log normalization")
            s, _ = self._nz_stats()  # zeros add nothing: channel sum over all pixels
            n = self.shape[0] * self.shape[1]
            mean = s.cpu().numpy() / n
        elif self._pending is not None or self._pending_blur is not None:
            self._materialize()  # a transform already pending applies first
        mean = np.asarray(mean, dtype=np.float64)
        with np.errstate(divide="ignore"):
            inv = (1.0 / mean).astype(np.float32)
        # a raw integer slide's bound survives a pending log_normalize (_blur_bound)
        raw = self._raw_int_max() is not None and self._pending is None and self._pending_blur is None
        self._pending = (D.h2d(inv, D.device()), float(pseudoval))
        self._lognorm_host = (inv, float(pseudoval)) if raw else None
        self._xbound = None
        self._host64 = None

    def _subsample_device(self, features, fract=0.2, random_state=16, X_out=None, stats=None,
                          accumulate=False):
        """Device subsample: mask rank → legacy-RNG indices → row gather into
        ``X_out`` (fp32) with column statistics folded into ``stats``."""
        from .stream import blur_gather

        features = self._features(features)
        np.random.seed(random_state)  # the reference's global-RNG side effect (MxIF.py:484)
        deferred = self._pending_blur is not None
        src = None if deferred else D.as_float32(self._materialize())
        r2p, M = self._mask_rank()
        dev = D.device()
        d_idx, total = subsample_indices_device(M, fract, random_state, dev)
        S = d_idx.shape[0]
        if X_out is None:
            X_out = torch.empty((S, len(features)), dtype=torch.float32, device=dev)
        if stats is None:
            stats = torch.zeros(1 + 2 * len(features), dtype=torch.float64, device=dev)
        if S:
            feat = D.h2d(np.asarray(features, dtype=np.int32), dev)
            if deferred:  # rows straight from the blur (resident or streamed slide)
                sigma, truncate = self._pending_blur
                inv, p = self._pending
                blur_gather(self._source() or self._device(), sigma, inv, p, feat, d_idx, r2p, X_out,
                            truncate)
                D.col_stats_rows(X_out, stats, accumulate)
            else:
                D.gather_rows(src, feat, d_idx, r2p, X_out, stats, accumulate)
            check_total(total, S)
            set_global_state_after_draws()
        return X_out, stats

    def subsample_pixels(self, features, fract=0.2, random_state=16):
        """MxIF.py:457-492 — returns the float64 (S x F) host array."""
        X, _ = self._subsample_device(features, fract, random_state)
        return X.double().cpu().numpy()

    def downsample(self, fact, func=np.mean):
        """MxIF.py:494-517 with func=np.mean (block_reduce, zero padded, pad
        zeros counted); the mask becomes fractional exactly as the reference."""
        if func is not np.mean:
            raise NotImplementedError("downsample supports func=np.mean on the device")
        if self.mask is not None:
            m = torch.from_numpy(np.ascontiguousarray(self.mask, dtype=np.float32)[:, :, None]).to(D.device())
            self.mask = D.block_mean(m, int(fact))[:, :, 0].double().cpu().numpy()
        out = D.block_mean(self._materialize(), int(fact))
        self._set_device(out)
        self._xbound = None

    def _nz_stats(self):
        """Per-channel non-zero (sum, count) of the current pixels: band by
        band when the raw slide is not resident (stream.nz_stats: exact
        integer sums for uint8 / uint16, the whole-slide bits)."""
        from . import stream

        src = self._source() if self._pending is None and self._pending_blur is None else None
        if src is not None:
            D.FUSED_USED["nz_streamed"] += 1
            return stream.nz_stats(src)
        return D.nz_stats(self._materialize())

    def calculate_non_zero_mean(self, comm=None):
        """MxIF.py:519-541: ([mean_c * pixels], pixels) with pixels = non-zero
        elements over all channels.  A row band of a slide (milwrm_amd.bands)
        sums its band rows and all-reduces the exact integer-valued sums over
        ``comm``: every band returns the whole slide's values."""
        if getattr(self, "_band", None) is not None:
            s, c = D.nz_stats(self._materialize()[self._band.rows].contiguous())
            if comm is not None and comm.sharded():
                comm.all_reduce_(s)
                comm.all_reduce_(c)
            s, c = D.d2h(s, c)
            pixels = int(c.sum())
            with np.errstate(invalid="ignore", divide="ignore"):
                means = s / c
            return [float(m) * pixels for m in means], pixels
        s, c = self._nz_stats()
        pending = D.d2h_async(s, c)
        # the mask rank queued behind the copies: it runs while the host waits
        # for them and does the work that follows (the blur needs its result
        # only later), instead of before them
        self._prefetch_mask_rank()
        s, c = pending.wait()
        pixels = int(c.sum())
        with np.errstate(invalid="ignore", divide="ignore"):
            means = s / c
        return [float(m) * pixels for m in means], pixels

    def create_tissue_mask(self, features=None, fract=0.2):
        """MxIF.py:543-589 on the device kernels: log-normalise (global channel
        means), Gaussian sigma=2, subsample ``features``, KMeans(2,
        random_state=18) on the UNscaled samples, predict every pixel on ALL
        channels (as the reference's ``kmeans.predict(image_ar_reshape)``, so a
        feature subset raises sklearn's feature-count error), background flip."""
        from .assign import assign_image
        from .kmeans import DeviceRows, KMeans

        cp = self.copy()
        H, W = cp.shape[0], cp.shape[1]
        cp.mask = np.ones((H, W))
        cp.log_normalize()
        cp.blurring("gaussian", sigma=2)
        X, st = cp._subsample_device(features, fract)
        stats = st.cpu().numpy()
        F = X.shape[1]
        var = stats[1 + F:] / stats[0]
        km = KMeans(n_clusters=2, random_state=18).fit(DeviceRows(X, feature_var=var))
        d = cp.n_ch
        if d != F:
            raise ValueError(f"X has {d} features, but KMeans is expecting {F} features as input.")
        lab, _, _ = assign_image(D.as_float32(cp._materialize()), list(range(d)), np.zeros(F),
                                 np.ones(F), km.cluster_centers_, cp._mask_device())
        tID = lab.cpu().numpy().astype(float)
        scores = km.cluster_centers_
        z = (scores - scores.mean()) / scores.std()
        if z[0].mean() > 0:
            tID = np.where(tID == 0.0, 0.5, tID)
            tID = np.where(tID == 1.0, 0.0, tID)
            tID = np.where(tID == 0.5, 1.0, tID)
        self.mask = tID
