"""Tissue-domain labelers of MILWRM (MILWRM.py:29-2264) on the MI355X engine.

Same classes, methods, arguments, attributes and error messages as the
reference for the pixel-clustering path; the numerics behind them are the HIP
kernels (fused lognorm+blur, subsample gather + column statistics, k-means++,
fused Lloyd E+M, label+confidence pass).  Plotting / UMAP methods are outside
the hot path and raise ``NotImplementedError``.

Data placement: per-image pixels and the clustering rows stay in HBM; the
reference's host attributes (``cluster_data``, ``tissue_IDs``,
``confidence_IDs``) are materialised as float64 numpy arrays on first access.
``n_jobs`` is accepted for signature compatibility and ignored (one process
drives the device; multi-GPU runs go through ``milwrm_amd.dist``).
"""
from __future__ import annotations

import itertools
import os

import numpy as np
import pandas as pd
import torch

from . import _native as N
from . import device as D
from .assign import (DOM_REC, assign_image, assign_rows, banded_assign_image, blur_assign_image,
                     dm_total, dom_carry_, dom_sums, domain_means, domain_sse_deferred, domain_sse_image,
                     domain_sse_rows, LabelPassQC)
from .kmeans import DeviceRows, KMeans, StandardScaler, fit_many
from .MxIF import checktype, img
from .ST import blur_features_st
from .dist import LOCAL_COMM
from .rng import _release_last_draw, check_total, set_global_state_after_draws, subsample_indices_device


# ------------------------------------------------------------ k selection

def kMeansRes(scaled_data, k, alpha_k=0.02, random_state=18, comm=None):
    """MILWRM.py:29-54: inertia / inertia_o + alpha_k * k."""
    comm = LOCAL_COMM if comm is None else comm
    rows = scaled_data if isinstance(scaled_data, DeviceRows) else DeviceRows.from_host(scaled_data)
    inertia_o = _inertia_o(rows, comm)
    kmeans = KMeans(n_clusters=k, random_state=random_state).fit(rows, comm=comm)
    return kmeans.inertia_ / inertia_o + alpha_k * k


def _inertia_o(rows: DeviceRows, comm=LOCAL_COMM) -> float:
    """sum((X - X.mean)^2) of the scaled rows = S_total * sum_f var_f."""
    S = rows.S
    if comm.sharded():
        S = int(comm.all_gather_np(np.array([S], dtype=np.int64))[:, 0].sum())
    return float(S * np.sum(rows.feature_var()))


def chooseBestKforKMeansParallel(scaled_data, k_range, n_jobs=-1, comm=None, **kwargs):
    """MILWRM.py:57-90 (fits run one after another on the device)."""
    rows = scaled_data if isinstance(scaled_data, DeviceRows) else DeviceRows.from_host(scaled_data)
    if os.environ.get("MW_SWEEP_BATCH", "1") == "0":  # one fit after another (A/B timing)
        ans = [kMeansRes(rows, k, comm=comm, **kwargs) for k in k_range]
    else:
        # all k fitted together: one pass over the rows per Lloyd iteration
        # for every fit still running (kmeans.fit_many); same values as kMeansRes
        alpha_k = kwargs.get("alpha_k", 0.02)
        inertia_o = _inertia_o(rows, LOCAL_COMM if comm is None else comm)
        fits = fit_many(rows, list(k_range), random_state=kwargs.get("random_state", 18),
                        comm=comm)
        ans = [km.inertia_ / inertia_o + alpha_k * k for km, k in zip(fits, k_range)]
        n_iter = {int(k): int(km.n_iter_) for km, k in zip(fits, k_range)}
    ans = list(zip(k_range, ans))
    results = pd.DataFrame(ans, columns=["k", "Scaled Inertia"]).set_index("k")
    if os.environ.get("MW_SWEEP_BATCH", "1") != "0":
        results.attrs["n_iter"] = n_iter  # Lloyd iterations per k (bench.py --sweep)
    best_k = results.idxmin().iloc[0]
    return best_k, results


# --------------------------------------------------------- MxIF workers

def prep_data_single_sample_mxif(image, use_path, mean, filter_name, sigma, features, fract,
                                 path_save):
    """MILWRM.py:172-234 (host-returning form)."""
    if use_path:
        if path_save is None:
            raise Exception("Path to save final preprocessed npz files is requird when given path "
                            "to image files")
        image_path = image
        image = img.from_npz(image_path + ".npz")
    image.log_normalize(mean=mean)
    image.blurring(filter_name=filter_name, sigma=sigma)
    subsampled = image.subsample_pixels(features, fract)
    if use_path:
        file_save = _save_preprocessed(image, image_path, path_save)
        return subsampled, file_save
    return subsampled


def _save_preprocessed(image, image_path, path_save):
    new_image_path = os.path.join(path_save, "_final_preprocessed_images")
    if not os.path.exists(new_image_path):
        os.mkdir(new_image_path)
    file_save = os.path.join(new_image_path, image_path.split("/")[-1] + "_final_preprocessed")
    image.to_npz(file_save)
    return file_save


def add_tissue_ID_single_sample_mxif(image, use_path, features, kmeans, scaler):
    """MILWRM.py:237-277: H x W float labels, NaN outside the mask."""
    if use_path:
        image = img.from_npz(image + ".npz")
    lab, _, _ = _assign_img(image, features, kmeans.cluster_centers_, scaler)
    return _labels_to_host(lab)


def estimate_confidence_score_mxif(image, use_path, scaler, centroids, features, tissue_ID):
    """MILWRM.py:389-450: (cID H x W float, NaN outside the mask; per-domain
    mean over the given tissue_ID)."""
    if use_path:
        image = img.from_npz(image + ".npz")
    lab, conf, dom = _assign_img(image, features, centroids, scaler)
    cid = _conf_to_host(conf)
    tid = np.asarray(tissue_ID)
    own = _labels_to_host(lab)
    if tid.shape == own.shape and np.array_equal(np.nan_to_num(tid, nan=-1), np.nan_to_num(own, nan=-1)):
        means = domain_means(dom.cpu().numpy(), len(centroids))
    else:
        means = {}
        with np.errstate(invalid="ignore"):
            import warnings

            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                for i in range(len(centroids)):
                    means[i] = np.mean(cid[tid == i])
    return cid, means


def estimate_confidence_score_st(sub_cluster_data, adata, centroids):
    """MILWRM.py:557-598."""
    _, cid, _ = assign_rows(sub_cluster_data, np.asarray(centroids, dtype=np.float64))
    adata.obs["confidence_score"] = cid
    score_df = pd.DataFrame(cid, columns=["score"])
    score_df["tissue_ID"] = adata.obs["tissue_ID"].values
    mean_conf_score = {}
    for i in range(len(centroids)):
        if (adata.obs["tissue_ID"] == i).any():
            mean_conf_score[i] = score_df[score_df["tissue_ID"] == i]["score"].mean()
        else:
            mean_conf_score[i] = np.nan
    return mean_conf_score


def _domain_stats(image, use_path, scaler, centroids, features, tissue_ID):
    if use_path:
        image = img.from_npz(image + ".npz")
    feats = image._features(features)
    mu, inv = scaler.affine()
    centroids = np.asarray(centroids, dtype=np.float64)
    if image._pending_blur is not None:
        # deferred blur (the fp32 blurred slide does not fit HBM): blurred band
        # by band into a reused buffer; the exact sums make it bitwise the
        # materialised slide's result
        sigma, truncate = image._pending_blur
        inv_mean, p = image._pending
        return domain_sse_deferred(image._source() or image._device(), sigma, inv_mean, p, feats, mu,
                                   inv, centroids, tissue_ID, truncate=truncate,
                                   colmax=getattr(image, "_xbound", None))
    return domain_sse_image(D.as_float32(image._materialize()), feats, mu, inv, centroids, tissue_ID,
                            colmax=getattr(image, "_xbound", None))


def estimate_percentage_variance_mxif(image, use_path, scaler, centroids, features, tissue_ID):
    """MILWRM.py:280-333: 100 * sum over domains of (x' - c)^2 / sum over the
    whole slide of (x' - mean(x'))^2, from ``mw_domain_sse`` passes."""
    s = _domain_stats(image, use_path, scaler, centroids, features, tissue_ID)
    return np.float64(np.sum(s["sse"])) / dm_total(s) * 100


def estimate_mse_mxif(images, use_path, tissue_IDs, scaler, centroids, features, k):
    """MILWRM.py:453-515: {domain: [per-feature MSE for each image]} (zeros for
    a domain an image does not hold)."""
    centroids = np.asarray(centroids, dtype=np.float64)[:k]
    mse_temp = []
    for image, tid in zip(images, tissue_IDs):
        s = _domain_stats(image, use_path, scaler, centroids, features, tid)
        cnt = s["count"][:, None]
        mse_temp.append(np.where(cnt > 0, s["sse"] / np.maximum(cnt, 1), 0.0))
    return {i: [m[i] for m in mse_temp] for i in range(k)} if len(images) else {}


def _st_labels(adata) -> np.ndarray:
    t = adata.obs["tissue_ID"]
    v = np.asarray(t.astype(float) if hasattr(t, "astype") else t, dtype=np.float64)
    return np.where(np.isfinite(v), v, -1).astype(np.int64)


def estimate_percentage_variance_st(sub_cluster_data, adata, centroids):
    """MILWRM.py:518-554: the spots of one section, their tissue_IDs and the
    centroids -> 100 * sum of (x - c_id)^2 / sum of (x - mean(x))^2 (one
    ``mw_domain_sse`` pass over the section's rows)."""
    X = np.asarray(sub_cluster_data, dtype=np.float64)
    s = domain_sse_rows(X, np.asarray(centroids, dtype=np.float64), _st_labels(adata))
    return np.float64(np.sum(s["sse"])) / dm_total(s) * 100


def estimate_mse_st(cluster_data, adatas, centroids, k):
    """MILWRM.py:601-644: {domain: [per-feature MSE for each section]}.  The
    reference slices section m's rows as cluster_data[n_obs(m-1):...] (its
    ``i_slice = adata.n_obs``), so section m >= 1 reads rows from offset
    n_obs of the previous section; kept as is."""
    cluster_data = np.asarray(cluster_data, dtype=np.float64)
    centroids = np.asarray(centroids, dtype=np.float64)
    per = []
    off = 0
    for adata in adatas:
        lab = _st_labels(adata)
        rows = cluster_data[off:off + adata.n_obs]
        s = domain_sse_rows(rows, centroids[:k], lab)
        cnt = s["count"][:, None]
        per.append(np.where(cnt > 0, s["sse"] / np.maximum(cnt, 1), 0.0))
        off = adata.n_obs
    return {i: [m[i] for m in per] for i in range(k)}


def _check_rows_fit(S: int, F: int, dev) -> None:
    """The clustering rows of this rank stay in HBM for the whole fit (fp32
    rows + ~17 bytes of per-row fit state: k-means++ potential, distance
    bounds, labels).  A cohort whose sampled rows exceed what is free (config
    5 at 1-2 GPUs: 870 GB of rows) raises here, before any allocation, with the
    remedy, instead of failing inside a kernel launch."""
    from .stream import RESIDENCY

    need = S * (F * 4 + 17)
    free = RESIDENCY.release(need)  # resident copies of host-backed slides go first (stream.py)
    if need > free:
        raise MemoryError(
            f"the {S} clustering rows of this rank ({F} features) need {need / 2**30:.1f} GiB of HBM "
            f"for the fit and {free / 2**30:.1f} GiB are free: shard the images over more GPUs "
            f"(comm=milwrm_amd.dist.make_comm() under torchrun; rows are split by image, or one "
            f"slide by row bands, milwrm_amd.bands) or lower fract")


def _assign_img(image: img, features, centers, scaler, qc=False):
    """(labels, confidences, per-domain records[, QC sums]) of one image: the
    QC sums of ``_domain_stats`` as extra outputs of the same pass when
    ``qc`` (a whole slide with a known pixel bound, ``img._blur_bound``;
    else None: the estimators run their own pass later)."""
    res = _assign_img_(image, features, centers, scaler, qc)
    if not qc:
        return res
    lab, conf, dom, q = res
    return lab, conf, dom, (q.result() if q is not None else None)


def _assign_img_(image: img, features, centers, scaler, qc):
    feats = image._features(features)
    mu, inv = scaler.affine()
    centers = np.asarray(centers, dtype=np.float64)
    band = getattr(image, "_band", None)
    bound = getattr(image, "_xbound", None)
    q = LabelPassQC(feats, image.n_ch, mu, inv, centers, bound) if (
        qc and band is None and bound is not None) else None

    def out(r):
        return r if not qc else (*r, q)

    if image._pending_blur is not None:
        # deferred blur (D.defer_blur: the fp32 blurred slide does not fit
        # HBM): blur band by band into a reused buffer and label each band
        # (MW_DEFERRED_ASSIGN=band, the default), or recompute the blur
        # inside the fused assign epilogue (=fused, or when no band fits)
        sigma, truncate = image._pending_blur
        inv_mean, p = image._pending
        how = os.environ.get("MW_DEFERRED_ASSIGN", "band")
        res = None
        band = getattr(image, "_band", None)  # a slide band: label its own rows only
        out_rows = None if band is None else (band.rows.start, band.rows.stop)
        # resident raw slide, or (not resident) its stream.RowSource read band by band
        raw = image._source() or image._device()
        fusable = band is None and feats == list(range(image.n_ch))
        if how == "fused" and fusable:  # no fp32 band: the QC sums are left to the estimators
            res = blur_assign_image(raw, sigma, inv_mean, p, mu, inv, centers, image._mask_device(),
                                    truncate=truncate)
            q = None
        if res is None:
            res = banded_assign_image(raw, sigma, inv_mean, p, feats, mu, inv, centers,
                                      image._mask_device(), truncate=truncate, out_rows=out_rows, qc=q)
        if res is None and how != "fused" and fusable:  # not even a 16-row fp32 band fits
            res = blur_assign_image(raw, sigma, inv_mean, p, mu, inv, centers, image._mask_device(),
                                    truncate=truncate)
            q = None
        if res is not None:
            return out(res)
    src = D.as_float32(image._materialize())
    if band is not None:  # label the band rows only (milwrm_amd.bands)
        return out(assign_image(src[band.rows], feats, mu, inv, centers,
                                D.padded_mask(image._mask_device()[band.rows].contiguous())))
    res = assign_image(src, feats, mu, inv, centers, image._mask_device())
    if q is not None:  # the slide is resident: its QC sums from the same fp32 pixels
        q.band(src, res[0])
    return out(res)


_SIDE = {}
# 1: with the rank index, the draws become pixels before the gather (A/B;
# device.py RANK_TABLE_MAX_PIX: no faster at config 2)
GATHER_BY_PIXEL = os.environ.get("MW_GATHER_PX", "0") == "1"
DRAWS_BESIDE = os.environ.get("MW_DRAWS_BESIDE", "1") != "0"  # 0: in line after the blur (A/B)


def _draws_beside(M: int, fract: float, dev, after: torch.cuda.Event, index=None):
    """``subsample_indices_device(M, fract, 16)`` issued on a side stream the
    current stream then waits for: the MT19937 segments (compute) overlap
    the blur (HBM) queued before them.  Same draws, same global-state replay.
    ``index`` (a D.RankIndex): the draws are turned into pixels there too
    (mw_rank_to_pixel_ri, lookups in the on-die caches), so the gather reads
    rows with no dependent lookup."""
    main = torch.cuda.current_stream(dev)
    side = _SIDE.get(str(dev))
    if side is None:
        side = _SIDE[str(dev)] = torch.cuda.Stream(device=dev)
    side.wait_event(after)  # the work queued before the blur (not the blur)
    with torch.cuda.stream(side):
        idx, tot = subsample_indices_device(M, fract, 16, dev)
        if index is not None:
            D.rank_to_pixel(idx, index)
    main.wait_stream(side)
    idx.record_stream(main)
    tot.record_stream(main)
    return idx, tot


def _gather_deferred(image: img, feat, idx, r2p, X_out) -> bool:
    """Subsample rows written by the blur itself for an image whose blur is
    deferred (D.defer_blur); False when it is not, or the fused kernel does
    not take the shape (the caller materialises and gathers)."""
    from .stream import blur_gather

    if image._pending_blur is None:
        return False
    sigma, truncate = image._pending_blur
    inv_mean, p = image._pending
    # resident raw slide (one band), or its stream.RowSource read band by band
    return blur_gather(image._source() or image._device(), sigma, inv_mean, p, feat, idx, r2p, X_out,
                       truncate=truncate)


def _host_threads() -> int:
    """Threads of the host conversion loops (the box's CPU share is 16)."""
    return max(1, min(16, os.cpu_count() or 1))


def _d2h_pinned(t: torch.Tensor) -> torch.Tensor:
    """One asynchronous copy of a device tensor into page-locked host memory
    (torch's caching host allocator: the staging buffer is reused), then a
    wait for it."""
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    return h


def _labels_to_host(lab: torch.Tensor) -> np.ndarray:
    """tissue_IDs[i] as the reference holds it (MILWRM.py:275-276): float64,
    NaN outside the mask, from the device's int8 labels (-1 = no domain)."""
    h = _d2h_pinned(lab)
    out = np.empty(tuple(lab.shape), dtype=np.float64)
    N.call("mw_host_labels_f64", h.data_ptr(), h.numel(), out.ctypes.data, _host_threads())
    return out


class _LazyHostList(list):
    """List of device tensors that reads as the reference's list of float64
    host arrays (converted on first access, then cached)."""

    def __init__(self, items, convert):
        super().__init__(items)
        self._convert = convert
        self._done = [False] * len(items)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if not self._done[i]:
            super().__setitem__(i, self._convert(super().__getitem__(i)))
            self._done[i] = True
        return super().__getitem__(i)

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


def _conf_to_host(conf: torch.Tensor) -> np.ndarray:
    """confidence_IDs[i] (MILWRM.py:444-445): float64 from the device's fp32
    confidences (NaN outside the mask stays NaN)."""
    h = _d2h_pinned(conf)
    out = np.empty(tuple(conf.shape), dtype=np.float64)
    N.call("mw_host_f32_to_f64", h.data_ptr(), h.numel(), out.ctypes.data, _host_threads())
    return out


# ---------------------------------------------------------------- classes

def _stacked_bar(df, cmap, figsize, xlabel, save_to):
    """The reference's proportion bar chart (matplotlib)."""
    import matplotlib.pyplot as plt

    ax = df.plot.bar(stacked=True, cmap=cmap, figsize=figsize)
    ax.legend(loc="best", bbox_to_anchor=(1, 1))
    ax.set_xlabel(xlabel)
    ax.set_ylabel("tissue domain proportion")
    ax.set_ylim((0, 1))
    plt.tight_layout()
    if save_to is not None:
        ax.figure.savefig(save_to)
        return None
    return ax


class tissue_labeler:
    """MILWRM.py:647-922 (plots out of scope)."""

    def __init__(self):
        self._rows = None
        self._cluster_host = None
        self.k = None
        self._comm = LOCAL_COMM

    # cluster_data: device rows, host float64 on read (MILWRM.py:1745)
    @property
    def cluster_data(self):
        if self._cluster_host is None and self._rows is not None:
            self._cluster_host = self._rows.to_host_scaled()
        return self._cluster_host

    @cluster_data.setter
    def cluster_data(self, value):
        self._rows = None
        self._cluster_host = None if value is None else np.asarray(value, dtype=np.float64)

    def _device_rows(self) -> DeviceRows:
        if self._rows is None:
            if self._cluster_host is None:
                raise Exception("No cluster data found. Run prep_cluster_data() first.")
            self._rows = DeviceRows.from_host(self._cluster_host)
        return self._rows

    def find_optimal_k(self, plot_out=False, alpha=0.05, random_state=18, n_jobs=-1):
        """MILWRM.py:659-704: k in 2..20, best = first argmin of scaled inertia."""
        if self._rows is None and self._cluster_host is None:
            raise Exception("No cluster data found. Run prep_cluster_data() first.")
        self.random_state = random_state
        k_range = range(2, 21)
        best_k, results = chooseBestKforKMeansParallel(self._device_rows(), k_range, n_jobs=n_jobs,
                                                       comm=self._comm, random_state=random_state,
                                                       alpha_k=alpha)
        self.inertia_curve_ = results
        print("The optimal number of clusters is {}".format(best_k))
        self.k = int(best_k)

    def find_tissue_regions(self, k=None, random_state=18):
        """MILWRM.py:706-737."""
        if self._rows is None and self._cluster_host is None:
            raise Exception("No cluster data found. Run prep_cluster_data() first.")
        if k is None and self.k is None:
            raise Exception("No k found or provided. Run find_optimal_k() first or pass a k value.")
        if k is not None:
            print("Overriding optimal k value with k={}.".format(k))
            self.k = k
        self.random_state = random_state
        self._qc_stats = None  # QC sums a label pass took belong to the previous centers
        print("Performing k-means clustering with {} target clusters".format(self.k))
        self.kmeans = KMeans(n_clusters=self.k, random_state=random_state).fit(
            self._device_rows(), comm=self._comm)

    def _plot(self, *a, **k):
        raise NotImplementedError("plotting is outside the MI355X hot path")

    plot_feature_proportions = _plot
    plot_feature_loadings = _plot
    plot_percentage_variance_explained = _plot
    plot_mse_mxif = _plot
    plot_mse_st = _plot
    make_umap = _plot
    show_marker_overlay = _plot
    plot_gene_loadings = _plot


class mxif_labeler(tissue_labeler):
    """MILWRM.py:1632-2264 (hot path)."""

    def __init__(self, image_df):
        tissue_labeler.__init__(self)
        if np.all(image_df.columns == ["Img", "batch_names", "mean estimators", "pixels"]):
            self.image_df = image_df
        else:
            raise Exception("Image_df must be given with these columns in this format ['Img', "
                            "'batch_names', 'mean estimators', 'pixels']")
        imgs = list(self.image_df["Img"])  # (the reference's Series.apply(isinstance).all())
        if all(isinstance(x, img) for x in imgs):
            self.use_paths = False
        elif all(isinstance(x, str) for x in imgs):
            self.use_paths = True
        else:
            raise Exception("Img column in the dataframe should be either str for paths to the "
                            "files or mxif.img object")

    @property
    def merged_batch_labels(self):
        """MILWRM.py:1734-1737: image index of every clustering row (a plain
        list, built lazily — it has S entries and only the UMAP plots read it)."""
        if getattr(self, "_mbl", None) is None:
            counts = getattr(self, "_batch_counts", None)
            if counts is None:
                raise AttributeError("merged_batch_labels")
            self._mbl = list(itertools.chain(*[[x] * c for x, c in enumerate(counts)]))
        return self._mbl

    @merged_batch_labels.setter
    def merged_batch_labels(self, value):
        self._mbl = value

    def _batch_means(self, comm=LOCAL_COMM):
        """MILWRM.py:1706-1714 (summed over ranks when sharded)."""
        # per batch, in order of first appearance: sum of the images' estimator
        # arrays and pixel counts, accumulated in row order from 0 exactly as
        # the reference's sum(map(np.array, ...)) / sum(Series) over its
        # boolean selection (one pass instead of a selection per batch)
        per = {}
        df = self.image_df
        for im, batch, est, px in zip(df["Img"], df["batch_names"], df["mean estimators"],
                                      df["pixels"]):
            band = getattr(im, "_band", None)
            if band is not None and band.band != 0:
                # a slide split into row bands (milwrm_amd.bands): every band
                # reports the whole slide's estimators; count them once
                est, px = np.zeros(len(est)), 0
            acc = per.setdefault(batch, [0, 0])
            acc[0] = acc[0] + np.array(est)
            acc[1] = acc[1] + px
        per = {b: (e, p) for b, (e, p) in per.items()}
        if comm.sharded():
            per = comm.sum_batches(per)
        return {b: est / pixels for b, (est, pixels) in per.items()}

    def prep_cluster_data(self, features, filter_name="gaussian", sigma=2, fract=0.2,
                          path_save=None, comm=None):
        """MILWRM.py:1672-1745: batch means, per-image lognorm + blur (one
        fused kernel) + subsample gather straight into one HBM row block,
        StandardScaler from device column statistics.  With a sharded
        ``comm`` (milwrm_amd.dist) each rank holds its own slides and the
        statistics are merged across ranks."""
        comm = LOCAL_COMM if comm is None else comm
        self._comm = comm
        self._mbl = None
        if self._rows is not None or self._cluster_host is not None:
            print("WARNING: overwriting existing cluster data")
            self.cluster_data = None
        self.model_features = features
        use_path = self.use_paths
        means = self._batch_means(comm)
        images = []
        for image in self.image_df["Img"]:
            if use_path:
                if path_save is None:
                    raise Exception("Path to save final preprocessed npz files is requird when "
                                    "given path to image files")
                images.append(img.from_npz(image + ".npz"))
            else:
                images.append(image)
        if getattr(images[0], "_band", None) is not None:
            # one slide in row bands over the ranks (milwrm_amd.bands)
            from .bands import prep_banded

            X, img_stats, xmax = prep_banded(images[0], self.image_df["batch_names"].iloc[0],
                                             means, features, filter_name, sigma, fract, comm)
            self._batch_counts = [int(X.shape[0])]
            self._images = images
            st = comm.merge_image_stats(D.d2h(img_stats), X.shape[1])
            self.scaler = StandardScaler.from_stats(st)
            mu, inv = self.scaler.affine()
            self._rows = DeviceRows(X, mu, inv, feature_var=self.scaler.var_ * inv * inv,
                                    xmax_local=D.d2h(xmax))
            self._cluster_host = None
            return
        # the first image's log-normalise + blur is queued before the host
        # work below (mask-rank counts, allocations), which then overlaps it
        batches = list(self.image_df["batch_names"])
        ev0 = torch.cuda.Event()  # the work queued before this pass (see _draws_beside)
        ev0.record()
        if images:
            images[0].log_normalize(mean=means[batches[0]])
            images[0].blurring(filter_name=filter_name, sigma=sigma)
        # phase 1: mask ranks → sample counts → one preallocated row block.
        # Only the first image keeps its rank→pixel table (4 bytes per tissue
        # pixel: 5.4 GB per 40k^2 slide); the others are ranked again when
        # their rows are gathered, so a cohort holds one table at a time
        dev = D.device()
        ranks = []
        for i, im in enumerate(images):
            r2p, M = im._mask_rank()
            ranks.append((r2p if i == 0 else None, M))
        counts = [int(M * fract) for _, M in ranks]
        F = len(images[0]._features(features))
        _check_rows_fit(sum(counts), F, dev)
        X = torch.empty((sum(counts), F), dtype=torch.float32, device=dev)
        # per-image column statistics [n, mean, M2], merged on the host in
        # image order (comm.merge_image_stats): the same merge sequence for any
        # sharding of the images over ranks, so the scaler is bitwise the same
        img_stats = torch.zeros((len(images), 1 + 2 * F), dtype=torch.float64, device=dev)
        xmax = torch.zeros(F, dtype=torch.float32, device=dev)  # column max |x| (Lloyd fixed point)
        # the first image's draws do not depend on its pixels: issued now on a
        # side stream, the generator runs beside the blur instead of after it
        # materialised images gather by pixel: the draws become pixels through
        # the rank index first (mw_rank_to_pixel_ri), not per row in the gather
        def by_pixel(im, r2p):
            return isinstance(r2p, D.RankIndex) and im._pending_blur is None and GATHER_BY_PIXEL

        pre = None
        # (only beside a materialised blur: a deferred slide has no blur running
        # yet, and its streamed passes want the allocator on one stream --
        # config-5 share 7.29 s in line vs 7.70 s beside)
        if images and counts[0] and DRAWS_BESIDE and images[0]._pending_blur is None:
            px0 = by_pixel(images[0], ranks[0][0])
            pre = _draws_beside(ranks[0][1], fract, dev, ev0, ranks[0][0] if px0 else None) + (px0,)
        # phase 2: fused lognorm+blur, gather rows into X (image_df order)
        off = 0
        paths = []
        totals = []
        draws = []  # (row offset, rows, rank draws, rank base): the rows' slide order, for a spatial row sort
        rank_base = 0
        for n_img, (im, batch, (r2p, M), S) in enumerate(
                zip(images, self.image_df["batch_names"], ranks, counts)):
            if n_img > 0:
                im.log_normalize(mean=means[batch])
                im.blurring(filter_name=filter_name, sigma=sigma)
            np.random.seed(16)
            if S:
                if r2p is None:
                    r2p, _ = im._mask_rank()
                if n_img == 0 and pre is not None:
                    idx, tot, px = pre
                    pre = None
                else:
                    idx, tot = subsample_indices_device(M, fract, 16, dev)
                    px = by_pixel(im, r2p)
                    if px:
                        D.rank_to_pixel(idx, r2p)
                totals.append((tot, S))
                feat = D.h2d(np.asarray(im._features(features), dtype=np.int32), dev)
                if _gather_deferred(im, feat, idx, r2p, X[off:off + S]):
                    D.col_stats_rows(X[off:off + S], img_stats[n_img], accumulate=False,
                                     absmax=xmax)
                else:
                    D.gather_rows(D.as_float32(im._materialize()), feat, idx, None if px else r2p,
                                  X[off:off + S], img_stats[n_img], accumulate=False, absmax=xmax)
                # slide-order keys: pixels or ranks (both monotone in the pixel)
                # past the previous images' pixel counts
                draws.append((off, S, idx, rank_base))
                del idx
            else:
                # seed(16) then choice(M, 0) draws nothing: the global state
                # is the fresh seed's, not past an earlier image's draws
                _release_last_draw()
            r2p = None
            ranks[n_img] = (None, M)
            off += S
            rank_base += int(im.shape[0]) * int(im.shape[1])
            if use_path:
                paths.append(_save_preprocessed(im, self.image_df["Img"].iloc[n_img], path_save))
        self._batch_counts = counts  # merged_batch_labels is built on first access
        if use_path:
            self.image_df["Img"] = paths
        else:
            self._images = images
        # np.random as the reference leaves it (MxIF.py:484-490): waits for the
        # last draw's counts only, so the host replay overlaps the gather
        set_global_state_after_draws()
        host = D.d2h(img_stats, xmax, *[t for t, _ in totals])  # one synchronisation
        for (_, S), tot in zip(totals, host[2:]):
            check_total(int(tot[0]), S)
        st = comm.merge_image_stats(host[0], F)
        self.scaler = StandardScaler.from_stats(st)
        mu, inv = self.scaler.affine()
        self._rows = DeviceRows(X, mu, inv, feature_var=self.scaler.var_ * inv * inv,
                                xmax_local=host[1])
        self._rows.draws = draws
        self._cluster_host = None

    def _image_list(self):
        if self.use_paths:
            return [img.from_npz(p + ".npz") for p in self.image_df["Img"]]
        return list(self.image_df["Img"])

    def label_tissue_regions(self, k=None, alpha=0.05, plot_out=True, random_state=18, n_jobs=-1,
                             comm=None, qc=False):
        """MILWRM.py:1747-1794 plus the fused confidence pass (MILWRM.py:389-450
        is computed in the same sweep over each image).  ``qc``: also take the
        QC sums behind ``plot_percentage_variance_explained`` /
        ``plot_mse_mxif`` (MILWRM.py:280-333, 453-515) from the same pass --
        band by band on a deferred-blur slide, so the slide is not blurred
        again for them; the same bits as the estimators' own passes."""
        if comm is not None:
            self._comm = comm
        if k is None:
            print("Determining optimal cluster number k via scaled inertia")
            self.find_optimal_k(alpha=alpha, plot_out=plot_out, random_state=random_state,
                                n_jobs=n_jobs)
        self.find_tissue_regions(k=k, random_state=random_state)
        print("Creating tissue_ID images for image objects...")
        labs, confs, doms, qcs = [], [], [], []
        for image in self._image_list():
            res = _assign_img(image, self.model_features, self.kmeans.cluster_centers_, self.scaler,
                              qc=qc)
            labs.append(res[0])
            confs.append(res[1])
            doms.append(res[2])
            qcs.append(res[3] if qc else None)
        self._labels_dev, self._conf_dev, self._dom_dev = labs, confs, doms
        self._qc_stats = qcs
        self.tissue_IDs = _LazyHostList(labs, _labels_to_host)

    def _image_qc_stats(self) -> list:
        """Per image, the QC sums (``_domain_stats``) of the current labelling:
        those the label pass took (``label_tissue_regions(qc=True)``), else an
        estimator pass over the image."""
        cached = getattr(self, "_qc_stats", None) or []
        out = []
        for i, (image, tid) in enumerate(zip(self.image_df["Img"], self.tissue_IDs)):
            s = cached[i] if i < len(cached) else None
            if s is None:
                s = _domain_stats(image, self.use_paths, self.scaler, self.kmeans.cluster_centers_,
                                  self.model_features, tid)
            out.append(s)
        return out

    def percentage_variance_images(self) -> list:
        """S^2 per image: estimate_percentage_variance_mxif (MILWRM.py:280-333)
        of each image under the current labelling, as
        ``plot_percentage_variance_explained`` (:1796-1866) computes them."""
        return [np.float64(np.sum(s["sse"])) / dm_total(s) * 100 for s in self._image_qc_stats()]

    def mse_images(self) -> dict:
        """{domain: [per-feature MSE for each image]}: estimate_mse_mxif
        (MILWRM.py:453-515) as ``plot_mse_mxif`` (:1902-2011) computes it."""
        k = int(self.k)
        per = []
        for s in self._image_qc_stats():
            cnt = s["count"][:k, None]
            per.append(np.where(cnt > 0, s["sse"][:k] / np.maximum(cnt, 1), 0.0))
        return {i: [m[i] for m in per] for i in range(k)} if per else {}

    def plot_percentage_variance_explained(self, fig_size=(5, 5), R_square=False, save_to=None):
        """MILWRM.py:1796-1866: per image, the percentage of variance the
        clustering explains (R^2 = 100 - S^2) or leaves (S^2), as a scatter
        with the mean as a dashed line."""
        import matplotlib.pyplot as plt

        S = self.percentage_variance_images()
        vals = [100 - v for v in S] if R_square else S
        fig = plt.figure(figsize=fig_size)
        plt.scatter(range(len(vals)), vals, color="black")
        plt.xlabel("images")
        plt.ylabel("percentage variance explained by Kmeans")
        plt.ylim((0, 100))
        plt.axhline(y=np.mean(vals), linestyle="dashed", linewidth=1, color="black")
        fig.tight_layout()
        if save_to:
            plt.savefig(fname=save_to, transparent=True, bbox_inches="tight", dpi=300)
        return fig

    def plot_mse_mxif(self, figsize=(5, 5), ncols=None, labels=None, legend_cols=2, titles=None,
                      loc="lower right", bbox_coordinates=(0, 0, 1.5, 1.5), save_to=None):
        """MILWRM.py:1902-2011: per tissue domain, a box plot over features of
        the per-image MSE, the images as jittered dots (np.random.uniform, the
        reference's global-RNG draws)."""
        import matplotlib.pyplot as plt
        from matplotlib import gridspec

        assert self.kmeans is not None, "No cluster results found. Run \
        label_tissue_regions() first."
        mse_id = self.mse_images()
        n_img = len(self.image_df["Img"])
        features = self.model_features
        if labels is None:
            labels = range(n_img)
        if titles is None:
            titles = ["tissue_ID " + str(x) for x in range(self.k)]
        n_panels = len(mse_id)
        if ncols is None:
            ncols = len(titles)
        n_rows, n_cols = (1, n_panels) if n_panels <= ncols else (-(-n_panels // ncols), ncols)
        colors = plt.cm.tab20(np.linspace(0, 1, n_img))
        fig = plt.figure(figsize=(n_cols * figsize[0], n_rows * figsize[1]))
        left, bottom = 0.1 / n_cols, 0.1 / n_rows
        gs = gridspec.GridSpec(nrows=n_rows, ncols=n_cols, left=left, bottom=bottom,
                               right=1 - (n_cols - 1) * left - 0.01 / n_cols,
                               top=1 - (n_rows - 1) * bottom - 0.1 / n_rows)
        for i in mse_id:
            plt.subplot(gs[i])
            df = pd.DataFrame.from_dict(mse_id[i])
            plt.boxplot(df, positions=range(len(features)), showfliers=False)
            plt.xticks(ticks=range(len(features)), labels=self.model_features, rotation=60, fontsize=8)
            for col in df:
                for j in range(n_img):
                    dots = plt.scatter(col, df[col][j], s=j + 1, color=colors[j],
                                       label=labels[j] if col == 0 else "")
                    off = dots.get_offsets()
                    off[:, 0] += np.random.uniform(-0.3, 0.3, off.shape[0])  # x jitter only
                    dots.set_offsets(off)
            plt.xlabel("marker")
            plt.ylabel("mean square error")
            plt.title(titles[i])
        plt.legend(loc=loc, bbox_to_anchor=bbox_coordinates, ncol=legend_cols)
        gs.tight_layout(fig)
        if save_to:
            plt.savefig(fname=save_to, transparent=True, dpi=300)
        return fig

    def plot_tissue_ID_proportions_mxif(self, tID_labels=None, slide_labels=None, figsize=(5, 5),
                                        cmap="tab20", save_to=None):
        """MILWRM.py:2013-2073: per image, the share of the masked pixels in each
        tissue domain (``self.tissue_ID_proportion``, domains x images), from
        the label pass's per-domain pixel counts; then the stacked bar plot."""
        k = int(self.k)
        if getattr(self, "_dom_dev", None):
            doms = self._slide_doms()
            counts = dom_sums(doms, k)[1].T  # domains x images
        else:
            counts = np.array([[np.sum(np.asarray(t) == j) for t in self.tissue_IDs]
                               for j in range(k)], dtype=np.float64)
        df_count = pd.DataFrame(counts.astype(np.int64), index=range(k),
                                columns=range(counts.shape[1]))
        df_count = df_count / df_count.sum()
        if tID_labels:
            assert len(tID_labels) == df_count.shape[1], \
                "Length of given tissue domain labels does not match number of tissue domains!"
            df_count.columns = tID_labels
        if slide_labels:
            assert len(slide_labels) == df_count.shape[0], \
                "Length of given slide labels does not match number of slides!"
            df_count.index = slide_labels
        self.tissue_ID_proportion = df_count
        return _stacked_bar(df_count.T, cmap, figsize, "images", save_to)

    def _slide_doms_dev(self) -> torch.Tensor:
        """images x domain records (exact limbs of the per-domain confidence
        sums | pixel counts, ``dom_sums``) from the label pass, on the device;
        a slide split into row bands (milwrm_amd.bands) sums its bands'
        records exactly (one all-reduce over the ranks)."""
        t = torch.stack(self._dom_dev)
        ims = getattr(self, "_images", None) or []
        if ims and getattr(ims[0], "_band", None) is not None and self._comm.sharded():
            t = dom_carry_(self._comm.all_reduce_(t.clone()))
        return t

    def _slide_doms(self) -> np.ndarray:
        return D.d2h(self._slide_doms_dev())

    def confidence_score_images(self):
        """MILWRM.py:1868-1900 from the fused pass: confidence_IDs and the
        images x domains DataFrame of mean confidences.  The frame is built on
        first access of ``confidence_score_df`` from the domain records queued
        here (no host round trip until it is read: the next slide's work can
        be queued behind this one's label pass)."""
        k = self.kmeans.cluster_centers_.shape[0]
        t = self._slide_doms_dev() if self._dom_dev else None  # (its collective, if any, now)

        def frame():
            # images x domains, the frame the reference concatenates row by row
            # (index 0..n-1, columns 0..k-1), built in one constructor call
            doms = D.d2h(t) if t is not None else np.zeros((0, DOM_REC * k))
            rows = [list(domain_means(dom, k).values()) for dom in doms]
            return pd.DataFrame(np.asarray(rows, dtype=np.float64).reshape(-1, k))

        self.confidence_IDs = _LazyHostList(list(self._conf_dev), _conf_to_host)
        self._conf_df_pending = frame

    @property
    def confidence_score_df(self):
        """MILWRM.py:1868-1900's images x domains frame of mean confidences."""
        pending = self.__dict__.pop("_conf_df_pending", None)
        if pending is not None:
            self._confidence_score_df = pending()
        return self._confidence_score_df

    @confidence_score_df.setter
    def confidence_score_df(self, value):
        self.__dict__.pop("_conf_df_pending", None)
        self._confidence_score_df = value


class st_labeler(tissue_labeler):
    """MILWRM.py:925-1629 (ST plumbing; fit / confidence on the device)."""

    def __init__(self, adatas):
        tissue_labeler.__init__(self)
        if not isinstance(adatas, list):
            adatas = [adatas]
        print("Initiating ST labeler with {} anndata objects".format(len(adatas)))
        self.adatas = adatas
        self.raw = adatas.copy()

    def prep_cluster_data(self, use_rep, features=None, n_rings=1, histo=False,
                          fluor_channels=None, spatial_graph_key=None, n_jobs=-1):
        """MILWRM.py:951-1041."""
        if self._rows is not None or self._cluster_host is not None:
            print("WARNING: overwriting existing cluster data")
            self.cluster_data = None
        if features is None:
            self.features = [x for x in range(self.adatas[0].obsm[use_rep].shape[1])]
        else:
            self.features = features
        self.rep, self.histo, self.fluor_channels, self.n_rings = use_rep, histo, fluor_channels, n_rings
        print("Collecting and blurring {} features from .obsm[{}]...".format(len(self.features), use_rep))
        cluster_data = [prep_data_single_sample_st(a, i, use_rep, self.features, histo,
                                                   fluor_channels, spatial_graph_key, n_rings)
                        for i, a in enumerate(self.adatas)]
        batch_labels = [[x] * len(cluster_data[x]) for x in range(len(cluster_data))]
        self.merged_batch_labels = list(itertools.chain(*batch_labels))
        subsampled_data = pd.concat(cluster_data)
        self.scaler = StandardScaler().fit(subsampled_data.values)
        self.cluster_data = self.scaler.transform(subsampled_data.values)
        print("Collected clustering data of shape: {}".format(self.cluster_data.shape))

    def label_tissue_regions(self, k=None, alpha=0.05, plot_out=True, random_state=18, n_jobs=-1):
        """MILWRM.py:1043-1089 (labels are the fit labels, sliced per adata)."""
        if k is None:
            print("Determining optimal cluster number k via scaled inertia")
            self.find_optimal_k(plot_out=plot_out, alpha=alpha, random_state=random_state,
                                n_jobs=n_jobs)
        self.find_tissue_regions(k=k, random_state=random_state)
        start = 0
        print("Adding tissue_ID label to anndata objects")
        IDs = self.kmeans.labels_
        for i in range(len(self.adatas)):
            self.adatas[i].obs["tissue_ID"] = IDs[start:start + self.adatas[i].n_obs]
            self.adatas[i].obs["tissue_ID"] = self.adatas[i].obs["tissue_ID"].astype("category")
            self.adatas[i].obs["tissue_ID"] = self.adatas[i].obs["tissue_ID"].cat.set_categories(
                np.unique(IDs))
            start += self.adatas[i].n_obs

    def plot_tissue_ID_proportions_st(self, tID_labels=None, slide_labels=None, figsize=(5, 5),
                                      cmap="tab20", save_to=None):
        """MILWRM.py:1400-1452: per section, the share of spots in each tissue
        domain (value counts of the fit labels), as a stacked bar plot."""
        df_count = pd.DataFrame()
        for adata in self.adatas:
            df = adata.obs["tissue_ID"].value_counts(normalize=True, sort=False)
            df_count = pd.concat([df_count, df], axis=1)
        df_count = df_count.T.reset_index(drop=True)
        if tID_labels:
            assert len(tID_labels) == df_count.shape[1], \
                "Length of given tissue domain labels does not match number of tissue domains!"
            df_count.columns = tID_labels
        if slide_labels:
            assert len(slide_labels) == df_count.shape[0], \
                "Length of given slide labels does not match number of slides!"
            df_count.index = slide_labels
        self.tissue_ID_proportion = df_count
        return _stacked_bar(df_count, cmap, figsize, "slides", save_to)

    def confidence_score(self):
        """MILWRM.py:1091-1121."""
        assert self.kmeans is not None, "No cluster results found. Run label_tissue_regions() first."
        i_slice = j_slice = 0
        df_all = pd.DataFrame()
        centroids = self.kmeans.cluster_centers_
        for i, adata in enumerate(self.adatas):
            j_slice += adata.n_obs
            data = self.cluster_data[i_slice:j_slice]
            scores = estimate_confidence_score_st(data, adata, centroids)
            df = pd.DataFrame(scores.values(), columns=[i])
            df_all = pd.concat([df_all, df], axis=1)
            i_slice += adata.n_obs
        self.confidence_score_df = df_all


def prep_data_single_sample_st(adata, adata_i, use_rep, features, histo, fluor_channels,
                               spatial_graph_key=None, n_rings=1):
    """MILWRM.py:93-169."""
    tmp = pd.DataFrame()
    tmp[[use_rep + "_{}".format(x) for x in features]] = adata.obsm[use_rep][:, features]
    if histo:
        assert fluor_channels is None, "If histo is True, fluor_channels must be None. \
            Histology specifies brightfield H&E with three (3) features."
        print("Adding mean RGB histology features for adata #{}".format(adata_i))
        tmp[["R_mean", "G_mean", "B_mean"]] = adata.obsm["image_means"]
    if fluor_channels:
        assert histo is False, "If fluorescence channels are given, histo must be False. \
            Histology specifies brightfield H&E with three (3) features."
        print("Adding mean fluorescent channels {} for adata #{}".format(fluor_channels, adata_i))
        tmp[["ch_{}_mean".format(x) for x in fluor_channels]] = adata.obsm["image_means"][:, fluor_channels]
    if n_rings > 0:
        tmp = blur_features_st(adata, tmp, spatial_graph_key=spatial_graph_key, n_rings=n_rings)
    return tmp
