"""Generate golden vectors by running the REFERENCE's own code (build container only).

Runs /root/reference/MILWRM (read-only) with no-op stubs for its absent
plotting/IO imports (tkinter, umap, seaborn, scanpy, squidpy) and an
``skimage`` stub whose ``filters.gaussian`` / ``measure.block_reduce`` restate
scikit-image's published float semantics (scikit-image is not installed in
this image; documented assumption).  All arithmetic other
than those two functions is the reference's own code calling the pinned
sklearn 1.7.2 / SciPy 1.15.3 / NumPy 2.2.6 numerics.

Outputs small compressed ``.npz`` fixtures next to this script.  Nothing from
the reference is copied: the fixtures are inputs and outputs only.

Usage:  python tests/golden/make_golden.py [mxif_small mxif_hard256 preproc_edges st_hex qc st_hex_k8]
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


# ----------------------------------------------------------------- stubs ---
def _install_stubs():
    import scipy.ndimage as ndi

    def _mod(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    _mod("tkinter", E="e")
    _mod("umap", UMAP=object)
    _mod("seaborn", set_style=lambda *a, **k: None)
    _mod("scanpy", set_figure_params=lambda *a, **k: None)
    sq = _mod("squidpy")
    sq.gr = types.SimpleNamespace(spatial_neighbors=None)

    def gaussian(image, sigma=1, output=None, mode="nearest", cval=0,
                 preserve_range=False, truncate=4.0, *, channel_axis=None):
        # skimage >= 0.19: sigma 0 on the channel axis, float64 input kept.
        image = np.asarray(image)
        if channel_axis is not None:
            if np.isscalar(sigma):
                sigma = [sigma] * (image.ndim - 1)
            sigma = list(sigma)
            if len(sigma) == image.ndim - 1:
                sigma.insert(channel_axis % image.ndim, 0)
        assert image.dtype == np.float64
        return ndi.gaussian_filter(image, sigma, output=output, mode=mode,
                                   cval=cval, truncate=truncate)

    def block_reduce(image, block_size=2, func=np.sum, cval=0, func_kwargs=None):
        image = np.asarray(image)
        bs = tuple(block_size)
        pad = [(0, (-s) % b) for s, b in zip(image.shape, bs)]
        p = np.pad(image, pad, mode="constant", constant_values=cval)
        shp = []
        for s, b in zip(p.shape, bs):
            shp += [s // b, b]
        r = p.reshape(shp)
        return func(r, axis=tuple(range(1, 2 * len(bs), 2)))

    sk = _mod("skimage")
    sk.filters = _mod("skimage.filters", gaussian=gaussian)
    sk.measure = _mod("skimage.measure", block_reduce=block_reduce)
    sk.exposure = _mod("skimage.exposure")
    sk.io = _mod("skimage.io", imread=None)
    sk.restoration = _mod("skimage.restoration", denoise_bilateral=None)


def _import_reference():
    _install_stubs()
    import matplotlib

    matplotlib.use("Agg")
    sys.path.insert(0, REF)
    import MILWRM  # noqa: F401  (the reference package)
    from MILWRM import MILWRM as MW
    from MILWRM import MxIF

    return MW, MxIF


def _synth(h, w, c, seed, mode):
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle.milwrm_oracle import synth_slide

    return synth_slide(h, w, c, seed, mode)


def _nan_to_i8(a):
    out = np.where(np.isnan(a), -1, a).astype(np.int8)
    return out


def make_mxif_small(MW, MxIF):
    """3 slides 96x128x8 (2 batches), full mxif_labeler run with the sweep."""
    import pandas as pd
    from sklearn.cluster import kmeans_plusplus

    shapes = (96, 128, 8)
    raw, masks = [], []
    for s in range(3):
        im, m = _synth(*shapes, seed=20251015 + s, mode="hard")
        raw.append(im)
        masks.append(m)
    imgs = [MxIF.img(r.copy(), mask=m.copy()) for r, m in zip(raw, masks)]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b1", "b1", "b2"],
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = MW.mxif_labeler(df)
    features = list(range(8))
    lab.prep_cluster_data(features=features, filter_name="gaussian", sigma=2, fract=0.2)
    X = lab.cluster_data
    best_k, results = MW.chooseBestKforKMeansParallel(
        X, range(2, 21), n_jobs=1, random_state=18, alpha_k=0.05)
    lab.label_tissue_regions(k=None, alpha=0.05, plot_out=False, random_state=18, n_jobs=1)
    lab.confidence_score_images()
    kpp = np.full((21, 20), -1, dtype=np.int64)
    Xc = X - X.mean(axis=0)
    for k in range(2, 21):
        _, idx = kmeans_plusplus(Xc, k, random_state=18)
        kpp[k, :k] = idx
    # single Lloyd step from the k=8 k-means++ init (sklearn's own cython)
    from sklearn.cluster._k_means_lloyd import lloyd_iter_chunked_dense

    c0 = Xc[kpp[8, :8]].copy()
    cn = np.zeros_like(c0)
    w = np.zeros(8)
    labels = np.full(X.shape[0], -1, dtype=np.int32)
    shift = np.zeros(8)
    lloyd_iter_chunked_dense(Xc, np.ones(X.shape[0]), c0, cn, w, labels, shift, 1)
    # subsample indices as the reference draws them (MxIF.py:484,490)
    sub_idx = []
    for m in masks:
        M = int((m != 0).sum())
        np.random.seed(16)
        sub_idx.append(np.random.choice(M, int(M * 0.2)))
    out = dict(
        raw=np.stack(raw), masks=np.stack(masks),
        batch_names=np.array(["b1", "b1", "b2"]),
        mean_estimators=np.array(ests), pixels=np.array(pix),
        batch_mean_b1=np.asarray(sum(map(np.array, [ests[0], ests[1]])) / (pix[0] + pix[1])),
        batch_mean_b2=np.asarray(np.array(ests[2]) / pix[2]),
        preprocessed0=lab.image_df["Img"][0].img,
        preprocessed2=lab.image_df["Img"][2].img,
        sub_idx0=sub_idx[0], sub_idx2=sub_idx[2],
        cluster_data=X, scaler_mean=lab.scaler.mean_, scaler_scale=lab.scaler.scale_,
        merged_batch_labels=np.array(lab.merged_batch_labels),
        sweep_k=np.array(list(results.index)), sweep_scaled_inertia=results["Scaled Inertia"].values,
        best_k=np.array(best_k), k=np.array(lab.k),
        centers=lab.kmeans.cluster_centers_, labels=lab.kmeans.labels_,
        inertia=np.array(lab.kmeans.inertia_), n_iter=np.array(lab.kmeans.n_iter_),
        tissue_IDs=np.stack([_nan_to_i8(t) for t in lab.tissue_IDs]),
        confidence_IDs=np.stack(lab.confidence_IDs),
        confidence_score_df=lab.confidence_score_df.values.astype(np.float64),
        kpp_indices=kpp,
        lloyd1_centers_in=c0, lloyd1_labels=labels, lloyd1_centers_out=cn,
        lloyd1_weights=w, lloyd1_shift=shift,
    )
    np.savez_compressed(os.path.join(HERE, "mxif_small.npz"), **out)
    print("mxif_small: best_k", best_k, "k", lab.k, "n_iter", lab.kmeans.n_iter_, "S", X.shape)


def make_mxif_hard256(MW, MxIF):
    """One 256x256x30 hard-mode slide, k=8 end to end (no sweep)."""
    import pandas as pd

    raw, mask = _synth(256, 256, 30, seed=20251015, mode="hard")
    im = MxIF.img(raw.copy(), mask=mask.copy())
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"],
                       "mean estimators": [est], "pixels": [pix]})
    lab = MW.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(30)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=8, plot_out=False, random_state=18, n_jobs=1)
    lab.confidence_score_images()
    out = dict(raw=raw, mask=mask, centers=lab.kmeans.cluster_centers_,
               inertia=np.array(lab.kmeans.inertia_), n_iter=np.array(lab.kmeans.n_iter_),
               scaler_mean=lab.scaler.mean_, scaler_scale=lab.scaler.scale_,
               n_samples=np.array(lab.cluster_data.shape[0]),
               labels=lab.kmeans.labels_.astype(np.int8),
               tissue_IDs=_nan_to_i8(lab.tissue_IDs[0]),
               confidence_IDs=lab.confidence_IDs[0].astype(np.float32),
               confidence_score_df=lab.confidence_score_df.values.astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "mxif_hard256.npz"), **out)
    print("mxif_hard256: n_iter", lab.kmeans.n_iter_, "inertia", lab.kmeans.inertia_)


def make_preproc_edges(MW, MxIF):
    """Gaussian edge cases (sigma, H or W < radius) and downsample shapes,
    through the reference's own img.blurring / img.downsample."""
    rng = np.random.default_rng(7)
    out = {}
    cases = [((5, 7, 3), 0.5), ((40, 33, 2), 1.0), ((23, 61, 4), 2.0),
             ((3, 60, 1), 3.7), ((64, 9, 2), 2.0)]
    for i, (shp, sig) in enumerate(cases):
        a = rng.uniform(0, 3, size=shp)
        im = MxIF.img(a.copy(), mask=np.ones(shp[:2]))
        im.blurring("gaussian", sigma=sig)
        out[f"gauss{i}_in"] = a
        out[f"gauss{i}_sigma"] = np.array(sig)
        out[f"gauss{i}_out"] = im.img
    for i, (shp, f) in enumerate([((10, 13, 3), 4), ((16, 16, 2), 2), ((7, 5, 1), 3)]):
        a = rng.integers(0, 1000, size=shp).astype(np.uint16)
        m = (rng.uniform(size=shp[:2]) > 0.3).astype(np.uint8)
        im = MxIF.img(a.copy(), mask=m.copy())
        im.downsample(f)
        out[f"down{i}_in"] = a
        out[f"down{i}_mask"] = m
        out[f"down{i}_fact"] = np.array(f)
        out[f"down{i}_out"] = im.img
        out[f"down{i}_mask_out"] = im.mask
    # log_normalize with mean=None (per-image channel mean) and with a mean
    a = rng.integers(0, 500, size=(12, 17, 3)).astype(np.float64)
    im = MxIF.img(a.copy(), mask=np.ones((12, 17)))
    im.log_normalize()
    out["lognorm_none_in"] = a
    out["lognorm_none_out"] = im.img
    np.savez_compressed(os.path.join(HERE, "preproc_edges.npz"), **out)
    print("preproc_edges done")


class _DuckAnnData:
    """Minimal AnnData stand-in (obsm/obsp/obs/n_obs) for st_labeler."""

    def __init__(self, pcs, adj):
        import pandas as pd

        self.obsm = {"X_pca": pcs}
        self.obsp = {"spatial_connectivities": adj}
        self.obs = pd.DataFrame(index=[str(i) for i in range(pcs.shape[0])])
        self.n_obs = pcs.shape[0]


def _hex_grid(rows, cols):
    import scipy.sparse as sp

    n = rows * cols
    coords = []
    for r in range(rows):
        for c in range(cols):
            coords.append((r, c))
    idx = {rc: i for i, rc in enumerate(coords)}
    I, J = [], []
    for (r, c), i in idx.items():
        off = [(0, -1), (0, 1), (-1, 0), (1, 0)]
        off += [(-1, -1), (1, -1)] if r % 2 == 0 else [(-1, 1), (1, 1)]
        for dr, dc in off:
            j = idx.get((r + dr, c + dc))
            if j is not None:
                I.append(i)
                J.append(j)
    A = sp.csr_matrix((np.ones(len(I)), (I, J)), shape=(n, n))
    return A, np.array(coords)


def make_st_hex(MW):
    """st_labeler plumbing (config 1 stand-in): 2 hex-grid sections, 10 PCs."""
    rng = np.random.default_rng(11)
    adatas, pcs_all, adjs = [], [], []
    for s, (rows, cols) in enumerate([(50, 55), (48, 52)]):
        A, coords = _hex_grid(rows, cols)
        dom = ((coords[:, 0] // 12) * 3 + coords[:, 1] // 14) % 6
        prof = rng.normal(0, 3, size=(6, 10))
        pcs = prof[dom] + rng.normal(0, 1.0, size=(coords.shape[0], 10))
        adatas.append(_DuckAnnData(pcs, A))
        pcs_all.append(pcs)
        adjs.append(A)
    lab = MW.st_labeler(adatas)
    lab.prep_cluster_data(use_rep="X_pca", features=None, n_rings=1,
                          spatial_graph_key="spatial_connectivities", n_jobs=1)
    lab.label_tissue_regions(k=None, alpha=0.05, plot_out=False, random_state=18, n_jobs=1)
    lab.confidence_score()
    out = dict(
        pcs0=pcs_all[0], pcs1=pcs_all[1],
        adj0_indptr=adjs[0].indptr, adj0_indices=adjs[0].indices,
        adj1_indptr=adjs[1].indptr, adj1_indices=adjs[1].indices,
        cluster_data=lab.cluster_data, scaler_mean=lab.scaler.mean_,
        scaler_scale=lab.scaler.scale_, k=np.array(lab.k),
        centers=lab.kmeans.cluster_centers_, labels=lab.kmeans.labels_,
        inertia=np.array(lab.kmeans.inertia_), n_iter=np.array(lab.kmeans.n_iter_),
        conf0=adatas[0].obs["confidence_score"].values,
        conf1=adatas[1].obs["confidence_score"].values,
        confidence_score_df=lab.confidence_score_df.values.astype(np.float64),
    )
    np.savez_compressed(os.path.join(HERE, "st_hex.npz"), **out)
    print("st_hex: k", lab.k, "n_iter", lab.kmeans.n_iter_)


def make_st_hex_k8(MW):
    """Config 1's k (BASELINE.json: "st_labeler ... k=8"): the st_hex sections
    (same inputs, rebuilt from the same seed) labelled at k = 8 instead of the
    sweep's k."""
    rng = np.random.default_rng(11)
    adatas = []
    for s, (rows, cols) in enumerate([(50, 55), (48, 52)]):
        A, coords = _hex_grid(rows, cols)
        dom = ((coords[:, 0] // 12) * 3 + coords[:, 1] // 14) % 6
        prof = rng.normal(0, 3, size=(6, 10))
        pcs = prof[dom] + rng.normal(0, 1.0, size=(coords.shape[0], 10))
        adatas.append(_DuckAnnData(pcs, A))
    lab = MW.st_labeler(adatas)
    lab.prep_cluster_data(use_rep="X_pca", features=None, n_rings=1,
                          spatial_graph_key="spatial_connectivities", n_jobs=1)
    lab.label_tissue_regions(k=8, alpha=0.05, plot_out=False, random_state=18, n_jobs=1)
    lab.confidence_score()
    out = dict(pcs0=adatas[0].obsm["X_pca"], k=np.array(lab.k),
               centers=lab.kmeans.cluster_centers_, labels=lab.kmeans.labels_,
               inertia=np.array(lab.kmeans.inertia_), n_iter=np.array(lab.kmeans.n_iter_),
               conf0=adatas[0].obs["confidence_score"].values,
               conf1=adatas[1].obs["confidence_score"].values,
               tissue_ID1=np.asarray(adatas[1].obs["tissue_ID"].astype(int)),
               confidence_score_df=lab.confidence_score_df.values.astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "st_hex_k8.npz"), **out)
    print("st_hex_k8: n_iter", lab.kmeans.n_iter_)


def make_qc(MW, MxIF):
    """Clustering QC and tissue masks through the reference's own functions:
    estimate_percentage_variance_mxif / estimate_mse_mxif (MILWRM.py:280-333,
    453-515) on a k=4 and a k=24 labelling of the mxif_small slides,
    tissue-ID proportions (plot_tissue_ID_proportions_mxif, MILWRM.py:2013-2073,
    drawn to an Agg canvas), img.create_tissue_mask (MxIF.py:543-589), and the
    ST estimators estimate_percentage_variance_st / estimate_mse_st
    (MILWRM.py:518-554, 601-644) on the st_hex sections."""
    import pandas as pd

    shapes = (96, 128, 8)
    raw, masks = [], []
    for s in range(3):
        im, m = _synth(*shapes, seed=20251015 + s, mode="hard")
        raw.append(im)
        masks.append(m)
    out = {"raw": np.stack(raw), "masks": np.stack(masks)}
    for k in (4, 24):
        imgs = [MxIF.img(r.copy(), mask=m.copy()) for r, m in zip(raw, masks)]
        ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
        df = pd.DataFrame({"Img": imgs, "batch_names": ["b1", "b1", "b2"],
                           "mean estimators": list(ests), "pixels": list(pix)})
        lab = MW.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(8)), filter_name="gaussian", sigma=2, fract=0.2)
        lab.label_tissue_regions(k=k, plot_out=False, random_state=18, n_jobs=1)
        cents = lab.kmeans.cluster_centers_
        pv = [MW.estimate_percentage_variance_mxif(lab.image_df["Img"][i], False, lab.scaler, cents,
                                                   list(range(8)), lab.tissue_IDs[i])
              for i in range(3)]
        mse = MW.estimate_mse_mxif(list(lab.image_df["Img"]), False, lab.tissue_IDs, lab.scaler,
                                   cents, list(range(8)), k)
        lab.plot_tissue_ID_proportions_mxif()
        out[f"k{k}_centers"] = cents
        out[f"k{k}_scaler_mean"] = lab.scaler.mean_
        out[f"k{k}_scaler_scale"] = lab.scaler.scale_
        out[f"k{k}_tissue_IDs"] = np.stack([_nan_to_i8(t) for t in lab.tissue_IDs])
        out[f"k{k}_pct_variance"] = np.array(pv)
        out[f"k{k}_mse"] = np.array([[mse[i][j] for j in range(3)] for i in range(k)])  # k x images x F
        out[f"k{k}_proportions"] = lab.tissue_ID_proportion.values.astype(np.float64)
    # create_tissue_mask on the raw slides (features=None: all channels)
    tm = []
    for r in raw[:2]:
        im = MxIF.img(r.copy())
        im.create_tissue_mask()
        tm.append(np.asarray(im.mask, dtype=np.float64))
    out["tissue_mask"] = np.stack(tm)
    # ST estimators on the st_hex sections (3 copies: estimate_mse_st's slice offsets)
    rng = np.random.default_rng(11)
    adatas = []
    for s, (rows, cols) in enumerate([(50, 55), (48, 52), (20, 30)]):
        A, coords = _hex_grid(rows, cols)
        dom = ((coords[:, 0] // 12) * 3 + coords[:, 1] // 14) % 6
        prof = rng.normal(0, 3, size=(6, 10))
        pcs = prof[dom] + rng.normal(0, 1.0, size=(coords.shape[0], 10))
        adatas.append(_DuckAnnData(pcs, A))
        out[f"st_pcs{s}"] = pcs
        out[f"st_adj{s}_indptr"] = A.indptr
        out[f"st_adj{s}_indices"] = A.indices
    st = MW.st_labeler(adatas)
    st.prep_cluster_data(use_rep="X_pca", features=None, n_rings=1,
                         spatial_graph_key="spatial_connectivities", n_jobs=1)
    st.label_tissue_regions(k=5, alpha=0.05, plot_out=False, random_state=18, n_jobs=1)
    cd, cents = st.cluster_data, st.kmeans.cluster_centers_
    pv, i0 = [], 0
    for a in adatas:
        pv.append(MW.estimate_percentage_variance_st(cd[i0:i0 + a.n_obs], a, cents))
        i0 += a.n_obs
    mse = MW.estimate_mse_st(cd, adatas, cents, 5)
    out["st_cluster_data"] = cd
    out["st_centers"] = cents
    out["st_labels"] = st.kmeans.labels_
    out["st_pct_variance"] = np.array(pv)
    out["st_mse"] = np.array([[mse[i][j] for j in range(3)] for i in range(5)])
    out["st_proportions"] = np.stack(
        [a.obs["tissue_ID"].value_counts(normalize=True, sort=False).reindex(range(5)).values
         for a in adatas]).astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "qc_small.npz"), **out)
    print("qc_small: pct_variance k4", out["k4_pct_variance"], "k24", out["k24_pct_variance"])


if __name__ == "__main__":
    MW, MxIF = _import_reference()
    which = set(sys.argv[1:]) or {"mxif_small", "mxif_hard256", "preproc_edges", "st_hex", "qc",
                                   "st_hex_k8"}
    if "mxif_small" in which:
        make_mxif_small(MW, MxIF)
    if "mxif_hard256" in which:
        make_mxif_hard256(MW, MxIF)
    if "preproc_edges" in which:
        make_preproc_edges(MW, MxIF)
    if "st_hex" in which:
        make_st_hex(MW)
    if "qc" in which:
        make_qc(MW, MxIF)
    if "st_hex_k8" in which:
        make_st_hex_k8(MW)
