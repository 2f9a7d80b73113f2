"""CPU oracle for the MILWRM pixel-clustering hot path.

TEST INFRASTRUCTURE ONLY.  This module is a plain-numpy restatement of the
reference algorithm (codyheiser/MILWRM + the third-party numerics it calls).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it, and only as the *checker* / CPU baseline.
The product (``milwrm_amd``) never imports, links or executes anything here.

Parity pinning: every function below is checked against golden vectors that
were produced by running the reference's own code in the build container
(``tests/golden/make_golden.py``, skimage stubbed by its documented
scipy-equivalent semantics).

Third-party algorithms restated here (versions pinned in the build image):
  * scikit-learn 1.7.2  ``sklearn/cluster/_kmeans.py``, ``_k_means_lloyd.pyx``,
    ``_k_means_common.pyx``; ``sklearn/preprocessing/_data.py`` (StandardScaler)
  * SciPy 1.15.3        ``scipy/ndimage/_filters.py`` (gaussian_filter)
  * scikit-image (absent; >= 0.19 implied by ``channel_axis``) ``filters.gaussian``
    and ``measure.block_reduce`` — restated from their published semantics.
  * NumPy 2.2.6         legacy ``RandomState`` (MT19937), used directly.

Citations ``MILWRM.py:L`` / ``MxIF.py:L`` refer to /root/reference/MILWRM/.
"""
from __future__ import annotations

import math

import numpy as np

# ---------------------------------------------------------------------------
# L1 preprocessing (MILWRM/MxIF.py)
# ---------------------------------------------------------------------------


def non_zero_mean(img_hwc: np.ndarray):
    """``img.calculate_non_zero_mean`` (MxIF.py:519-541).

    ``pixels`` counts non-zero elements over ALL H*W*C entries (MxIF.py:535);
    the per-channel mean is over that channel's non-zero entries (:539) and
    the estimator is ``mean * pixels`` (:540).
    """
    image = np.asarray(img_hwc, dtype=np.float64)
    pixels = np.count_nonzero(image != 0)
    est = []
    for i in range(image.shape[2]):
        ar = image[:, :, i]
        est.append(ar[ar != 0].mean() * pixels)
    return est, pixels


def batch_means(mean_estimators, pixels, batch_names):
    """Batch-wise channel means (MILWRM.py:1706-1714)."""
    out = {}
    names = list(batch_names)
    for b in dict.fromkeys(names):
        sel = [i for i, n in enumerate(names) if n == b]
        est = sum(map(np.array, [mean_estimators[i] for i in sel]))
        pix = sum(pixels[i] for i in sel)
        out[b] = est / pix
    return out


def log_normalize(img_hwc: np.ndarray, mean=None, pseudoval=1.0) -> np.ndarray:
    """``img.log_normalize`` (MxIF.py:416-455): log10(x/mean_c + pseudoval)
    on every pixel of every channel (the mask is only asserted)."""
    x = np.asarray(img_hwc, dtype=np.float64).copy()
    for i in range(x.shape[2]):
        fact = mean[i] if mean is not None else x[:, :, i].mean()
        x[:, :, i] = np.log10(x[:, :, i] / fact + pseudoval)
    return x


def gaussian_kernel1d(sigma: float, truncate: float = 4.0) -> np.ndarray:
    """scipy ``_gaussian_kernel1d`` (order 0) with radius int(truncate*sigma+0.5)
    (scipy/ndimage/_filters.py:226-236, :316)."""
    radius = int(truncate * float(sigma) + 0.5)
    x = np.arange(-radius, radius + 1)
    phi = np.exp(-0.5 / (float(sigma) * float(sigma)) * x**2)
    return phi / phi.sum()


def _correlate1d_nearest(a: np.ndarray, w: np.ndarray, axis: int) -> np.ndarray:
    r = (len(w) - 1) // 2
    pad = [(0, 0)] * a.ndim
    pad[axis] = (r, r)
    p = np.pad(a, pad, mode="edge")
    out = np.zeros_like(a)
    n = a.shape[axis]
    for t in range(len(w)):
        sl = [slice(None)] * a.ndim
        sl[axis] = slice(t, t + n)
        out += w[t] * p[tuple(sl)]
    return out


def gaussian_blur(img_hwc: np.ndarray, sigma=2.0, truncate=4.0) -> np.ndarray:
    """``img.blurring('gaussian', sigma)`` (MxIF.py:387-394) →
    ``skimage.filters.gaussian(img, sigma, channel_axis=2)`` → float64 input is
    passed unchanged to ``scipy.ndimage.gaussian_filter(img, [s, s, 0],
    mode='nearest', truncate=4.0)``: axis 0 then axis 1, edge-replicate,
    float64 intermediate; sigma <= 1e-15 axes skipped (_filters.py:421-427)."""
    x = np.asarray(img_hwc, dtype=np.float64)
    sig = [float(sigma), float(sigma)] if np.isscalar(sigma) else [float(s) for s in sigma]
    for ax, s in enumerate(sig):
        if s > 1e-15:
            w = gaussian_kernel1d(s, truncate)
            x = _correlate1d_nearest(x, w[::-1], ax)
    return x


def block_reduce_mean(arr: np.ndarray, fact: int) -> np.ndarray:
    """``img.downsample(fact, np.mean)`` (MxIF.py:494-517) → skimage
    ``block_reduce(x, (f, f[, 1]), np.mean, cval=0)``: zero-pad each spatial
    axis to a multiple of ``fact`` (pad at the end), then the block mean
    INCLUDING the pad zeros."""
    a = np.asarray(arr, dtype=np.float64)
    h, w = a.shape[:2]
    ph = (-h) % fact
    pw = (-w) % fact
    pad = [(0, ph), (0, pw)] + [(0, 0)] * (a.ndim - 2)
    p = np.pad(a, pad, mode="constant", constant_values=0)
    H2, W2 = p.shape[0] // fact, p.shape[1] // fact
    r = p.reshape((H2, fact, W2, fact) + p.shape[2:])
    return r.mean(axis=(1, 3))


def subsample_indices(M: int, fract: float, random_state: int = 16) -> np.ndarray:
    """Index draw of ``img.subsample_pixels`` (MxIF.py:484,490):
    ``np.random.seed(16); np.random.choice(M, int(M*fract))`` — with
    replacement; uses NumPy's own legacy generator."""
    rs = np.random.RandomState(random_state)
    return rs.choice(M, int(M * fract))


def subsample_pixels(img_hwc, mask, features, fract=0.2, random_state=16):
    """``img.subsample_pixels`` (MxIF.py:457-492): all channels at mask!=0 in
    row-major order, then rows ``idx`` and columns ``features``."""
    x = np.asarray(img_hwc, dtype=np.float64)
    tmp = np.column_stack([x[:, :, i][mask != 0] for i in range(x.shape[2])])
    idx = subsample_indices(tmp.shape[0], fract, random_state)
    return tmp[np.ix_(idx, features)], idx


# --- MT19937 legacy randint restatement (pins the product's own generator) ---

_MT_N, _MT_M = 624, 397


def mt19937_init(seed: int) -> np.ndarray:
    """``init_genrand`` (numpy legacy seeding for an int seed)."""
    mt = np.zeros(_MT_N, dtype=np.uint64)
    mt[0] = seed & 0xFFFFFFFF
    for i in range(1, _MT_N):
        mt[i] = (1812433253 * (int(mt[i - 1]) ^ (int(mt[i - 1]) >> 30)) + i) & 0xFFFFFFFF
    return mt.astype(np.uint32)


def mt19937_stream(seed: int, nwords: int) -> np.ndarray:
    """First ``nwords`` tempered 32-bit outputs after legacy seeding."""
    mt = mt19937_init(seed).astype(np.uint64)
    out = np.empty(nwords, dtype=np.uint32)
    pos = 0
    while pos < nwords:
        for i in range(_MT_N):
            y = (int(mt[i]) & 0x80000000) | (int(mt[(i + 1) % _MT_N]) & 0x7FFFFFFF)
            v = int(mt[(i + _MT_M) % _MT_N]) ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            mt[i] = v
        take = min(_MT_N, nwords - pos)
        y = mt[:take].copy()
        y ^= y >> np.uint64(11)
        y ^= (y << np.uint64(7)) & np.uint64(0x9D2C5680)
        y ^= (y << np.uint64(15)) & np.uint64(0xEFC60000)
        y ^= y >> np.uint64(18)
        out[pos:pos + take] = (y & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        pos += take
    return out


def legacy_randint_masked(seed: int, high: int, size: int) -> np.ndarray:
    """``RandomState(seed).randint(0, high, size)`` for 0 < high-1 < 2**32-1:
    masked rejection on the raw 32-bit stream (numpy
    ``random_bounded_uint64_fill`` → ``buffered_bounded_masked_uint32``)."""
    rng = high - 1
    mask = (1 << max(rng.bit_length(), 1)) - 1
    out = np.empty(size, dtype=np.int64)
    got, nwords = 0, max(64, int(size * 2.2) + 64)
    stream = mt19937_stream(seed, nwords)
    vals = stream.astype(np.int64) & mask
    acc = vals[vals <= rng]
    while acc.size < size:  # pragma: no cover - only for tiny accept rates
        nwords *= 2
        stream = mt19937_stream(seed, nwords)
        vals = stream.astype(np.int64) & mask
        acc = vals[vals <= rng]
    out[:] = acc[:size]
    return out


# ---------------------------------------------------------------------------
# L0: StandardScaler (sklearn/preprocessing/_data.py:1049-1050,1096,1098)
# ---------------------------------------------------------------------------


def scaler_fit(X: np.ndarray):
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[0]
    mean = X.mean(axis=0)
    var = X.var(axis=0)  # ddof=0
    eps = np.finfo(np.float64).eps
    constant = var <= n * eps * var + (n * mean * eps) ** 2  # _data.py:76-89
    scale = np.sqrt(var)
    scale[constant] = 1.0
    return mean, scale, var


def scaler_transform(X, mean, scale):
    return (np.asarray(X, dtype=np.float64) - mean) / scale


# ---------------------------------------------------------------------------
# L0: sklearn KMeans (lloyd) restated
# ---------------------------------------------------------------------------


def _sq_dist_gemm(X, C, x_sq=None):
    """``_euclidean_distances(..., squared=True)`` : ||x||^2 - 2 x.c + ||c||^2,
    clipped at 0 (sklearn/metrics/pairwise.py)."""
    if x_sq is None:
        x_sq = np.einsum("ij,ij->i", X, X)
    c_sq = np.einsum("ij,ij->i", C, C)
    d = x_sq[:, None] - 2.0 * (X @ C.T) + c_sq[None, :]
    np.maximum(d, 0, out=d)
    return d


def first_center_index(n: int, u: float) -> int:
    """``random_state.choice(n, p=ones/n)`` given the drawn double ``u``:
    cdf = cumsum(p) (sequential); cdf /= cdf[-1]; searchsorted(u, 'right')."""
    p = np.full(n, 1.0 / float(n))
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return int(cdf.searchsorted(u, side="right"))


def kmeans_plusplus(X, n_clusters, random_state, n_local_trials=None):
    """sklearn ``_kmeans_plusplus`` (_kmeans.py:174-272), unit sample weights.
    ``X`` must already be centered (as KMeans.fit does, :1477-1481)."""
    rs = random_state if isinstance(random_state, np.random.RandomState) else np.random.RandomState(random_state)
    X = np.asarray(X, dtype=np.float64)
    n, f = X.shape
    w = np.ones(n)
    if n_local_trials is None:
        n_local_trials = 2 + int(np.log(n_clusters))
    x_sq = np.einsum("ij,ij->i", X, X)
    centers = np.empty((n_clusters, f))
    idx = np.full(n_clusters, -1, dtype=int)
    cid = rs.choice(n, p=w / w.sum())
    centers[0] = X[cid]
    idx[0] = cid
    closest = _sq_dist_gemm(X, centers[0:1], x_sq)[:, 0]
    pot = closest @ w
    for c in range(1, n_clusters):
        rv = rs.uniform(size=n_local_trials) * pot
        cum = np.cumsum(w * closest, dtype=np.float64)
        cand = np.searchsorted(cum, rv)
        np.clip(cand, None, closest.size - 1, out=cand)
        d = _sq_dist_gemm(X, X[cand], x_sq).T  # (T, n)
        np.minimum(closest, d, out=d)
        pots = d @ w
        b = int(np.argmin(pots))
        pot = pots[b]
        closest = d[b]
        centers[c] = X[cand[b]]
        idx[c] = cand[b]
    return centers, idx


def lloyd_iter(X, centers_old, update_centers=True):
    """``lloyd_iter_chunked_dense`` + ``_update_chunk_dense``
    (_k_means_lloyd.pyx:23-218): labels = argmin(||c||^2 - 2 x.c) with strict
    '<' (lowest index wins ties); weighted sums; then
    ``_relocate_empty_clusters_dense``, ``_average_centers``,
    ``_center_shift`` (_k_means_common.pyx:181-311)."""
    k, f = centers_old.shape
    c_sq = np.einsum("ij,ij->i", centers_old, centers_old)
    d = c_sq[None, :] - 2.0 * (X @ centers_old.T)
    labels = np.argmin(d, axis=1).astype(np.int32)  # first minimum
    if not update_centers:
        return labels, None, None, None
    centers_new = np.zeros((k, f))
    np.add.at(centers_new, labels, X)
    weight = np.bincount(labels, minlength=k).astype(np.float64)
    # relocate empty clusters
    empty = np.where(weight == 0)[0]
    if empty.size:
        dist = ((X - centers_old[labels]) ** 2).sum(axis=1)
        if np.max(dist) != 0:
            far = np.argpartition(dist, -empty.size)[: -empty.size - 1: -1]
            for e_i, far_idx in zip(empty, far):
                old = labels[far_idx]
                centers_new[old] -= X[far_idx]
                centers_new[e_i] = X[far_idx]
                weight[e_i] = 1.0
                weight[old] -= 1.0
    # average
    amax = int(np.argmax(weight))
    for j in range(k):
        if weight[j] > 0:
            centers_new[j] *= 1.0 / weight[j]
        else:
            centers_new[j] = centers_new[amax]
    shift = np.sqrt(((centers_new - centers_old) ** 2).sum(axis=1))
    return labels, centers_new, weight, shift


def inertia_dense(X, centers, labels):
    """``_inertia_dense`` (_k_means_common.pyx:94-124)."""
    return float(((X - centers[labels]) ** 2).sum())


def lloyd(X, centers_init, max_iter=300, tol=0.0):
    """``_kmeans_single_lloyd`` (_kmeans.py:624-752)."""
    centers = np.array(centers_init, dtype=np.float64)
    labels_old = np.full(X.shape[0], -1, dtype=np.int32)
    strict = False
    labels = labels_old
    for i in range(max_iter):
        labels, centers_new, _, shift = lloyd_iter(X, centers)
        centers = centers_new
        if np.array_equal(labels, labels_old):
            strict = True
            break
        if (shift ** 2).sum() <= tol:
            break
        labels_old = labels.copy()
    if not strict:
        labels, _, _, _ = lloyd_iter(X, centers, update_centers=False)
    return labels, inertia_dense(X, centers, labels), centers, i + 1


def kmeans_fit(X, n_clusters, random_state=18, init=None, max_iter=300, tol=1e-4):
    """``KMeans(n_clusters, random_state).fit(X)`` (_kmeans.py:1427-1554) with
    n_init='auto' → 1 for k-means++ (:879-881), lloyd algorithm.
    Returns dict(cluster_centers_, labels_, inertia_, n_iter_, init_indices)."""
    X = np.array(X, dtype=np.float64)
    _tol = float(np.mean(np.var(X, axis=0)) * tol) if tol else 0.0
    X_mean = X.mean(axis=0)
    X -= X_mean
    idx = None
    if init is None:
        centers_init, idx = kmeans_plusplus(X, n_clusters, np.random.RandomState(random_state))
    else:
        centers_init = np.array(init, dtype=np.float64) - X_mean
    labels, inertia, centers, n_iter = lloyd(X, centers_init, max_iter, _tol)
    centers = centers + X_mean
    return dict(cluster_centers_=centers, labels_=labels, inertia_=inertia,
                n_iter_=n_iter, init_indices=idx)


def predict(X, centers):
    """``KMeans.predict`` (_kmeans.py:1066-1098 → _labels_inertia): GEMM-trick
    argmin on the un-centered data, strict '<'."""
    X = np.asarray(X, dtype=np.float64)
    c_sq = np.einsum("ij,ij->i", centers, centers)
    return np.argmin(c_sq[None, :] - 2.0 * (X @ centers.T), axis=1).astype(np.int32)


# ---------------------------------------------------------------------------
# L2 / L3 (MILWRM/MILWRM.py)
# ---------------------------------------------------------------------------


def k_means_res(X, k, alpha_k=0.02, random_state=18):
    """``kMeansRes`` (MILWRM.py:29-54)."""
    inertia_o = np.square(X - X.mean(axis=0)).sum()
    r = kmeans_fit(X, k, random_state=random_state)
    return r["inertia_"] / inertia_o + alpha_k * k


def choose_best_k(X, k_range=range(2, 21), alpha_k=0.05, random_state=18):
    """``chooseBestKforKMeansParallel`` (MILWRM.py:57-90) + ``find_optimal_k``
    (:659-704): best_k = first argmin of the scaled inertia."""
    ks = list(k_range)
    vals = [k_means_res(X, k, alpha_k, random_state) for k in ks]
    return ks[int(np.argmin(vals))], dict(zip(ks, vals))


def tissue_ids(img_hwc, mask, features, centers, mean, scale):
    """``add_tissue_ID_single_sample_mxif`` (MILWRM.py:237-277)."""
    x = np.asarray(img_hwc, dtype=np.float64)[:, :, features]
    h, w, d = x.shape
    lab = predict(scaler_transform(x.reshape(h * w, d), mean, scale), centers).reshape(h, w)
    lab = lab.astype(float)
    lab[mask == 0] = np.nan
    return lab


def confidence_mxif(img_hwc, mask, features, centers, mean, scale, tissue_id):
    """``estimate_confidence_score_mxif`` (MILWRM.py:389-450)."""
    x = np.asarray(img_hwc, dtype=np.float64)[:, :, features]
    h, w, d = x.shape
    xs = scaler_transform(x.reshape(h * w, d), mean, scale).reshape(h, w, d)
    dist = np.zeros((h, w, len(centers)))
    for i, c in enumerate(centers):
        dist[:, :, i] += np.sum((xs - c) ** 2, axis=2)
    s = np.sort(dist, axis=2)
    with np.errstate(divide="ignore", invalid="ignore"):
        cid = (s[:, :, 1] - s[:, :, 0]) / s[:, :, 1]
    cid[mask == 0] = np.nan
    means = {}
    with np.errstate(invalid="ignore", divide="ignore"):
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            for i in range(len(centers)):
                means[i] = np.mean(cid[tissue_id == i])
    return cid, means


def percentage_variance_mxif(img_hwc, features, centers, mean, scale, tissue_id):
    """``estimate_percentage_variance_mxif`` (MILWRM.py:280-333)."""
    x = np.asarray(img_hwc, dtype=np.float64)[:, :, features]
    h, w, d = x.shape
    xs = scaler_transform(x.reshape(h * w, d), mean, scale)
    tid = np.asarray(tissue_id).reshape(h * w)
    dc = np.zeros(xs.shape)
    for i in range(centers.shape[0]):
        dc[tid == i] = (xs[tid == i] - centers[i]) ** 2
    dm = (xs - xs.mean(axis=0)) ** 2
    return np.sum(dc) / np.sum(dm) * 100


def mse_mxif(imgs, tissue_ids, features, centers, mean, scale, k):
    """``estimate_mse_mxif`` (MILWRM.py:453-515)."""
    out = {}
    for im, ar in zip(imgs, tissue_ids):
        x = np.asarray(im, dtype=np.float64)[:, :, features]
        h, w, d = x.shape
        xs = scaler_transform(x.reshape(h * w, d), mean, scale).reshape(h, w, d)
        for i in range(k):
            v = (xs[ar == i] - centers[i]) ** 2
            out.setdefault(i, []).append(np.zeros(centers.shape[1]) if len(v) == 0 else v.mean(axis=0))
    return out


def percentage_variance_st(X, centers, labels):
    """``estimate_percentage_variance_st`` (MILWRM.py:518-554): labels are the
    section's tissue_IDs (every spot has one)."""
    X = np.asarray(X, dtype=np.float64)
    dc = np.concatenate([(X[labels == i] - centers[i]) ** 2 for i in pd_unique(labels)])
    dm = (X - X.mean(axis=0)) ** 2
    return np.sum(dc) / np.sum(dm) * 100


def pd_unique(a):
    """Unique values in order of appearance (pandas.unique)."""
    _, first = np.unique(a, return_index=True)
    return np.asarray(a)[np.sort(first)]


def mse_st(X, label_list, n_obs, centers, k):
    """``estimate_mse_st`` (MILWRM.py:601-644), including its slice offsets:
    section m >= 1 reads rows from n_obs[m-1] (``i_slice = adata.n_obs``)."""
    X = np.asarray(X, dtype=np.float64)
    out = {}
    for i in range(k):
        i0, j0, diff = 0, 0, []
        for lab, n in zip(label_list, n_obs):
            j0 += n
            data = X[i0:j0]
            x = (data[np.where(lab == i)[0]] - centers[i]) ** 2
            diff.append(np.zeros(centers.shape[1]) if len(x) == 0 else x.mean(axis=0))
            i0 = n
        out[i] = diff
    return out


def tissue_id_proportions(tissue_ids, k):
    """``plot_tissue_ID_proportions_mxif``'s table (MILWRM.py:2040-2063):
    domains x images, each column the domains' share of the image's labelled
    pixels."""
    counts = np.array([[np.sum(np.asarray(t) == j) for t in tissue_ids] for j in range(k)],
                      dtype=np.float64)
    return counts / counts.sum(axis=0)


def create_tissue_mask(img_hwc, features=None, fract=0.2, return_gap=False):
    """``img.create_tissue_mask`` (MxIF.py:543-589): lognorm with the
    whole-image channel means, Gaussian sigma 2, subsample, KMeans(2, 18) on
    unscaled rows, predict all pixels, background flip.  ``return_gap``: also
    the per-pixel relative gap (d2 - d1) / d2 of the squared distances to the
    two centers (the near-tie measure of the 2-means labels)."""
    x = np.asarray(img_hwc, dtype=np.float64)
    h, w, d = x.shape
    x = log_normalize(x, None)
    x = gaussian_blur(x, 2.0)
    mask = np.ones((h, w))
    feats = list(range(d)) if features is None else list(features)
    X, _ = subsample_pixels(x, mask, feats, fract, 16)
    km = kmeans_fit(X, 2, random_state=18)
    c = km["cluster_centers_"]
    lab = predict(x.reshape(h * w, d), c).astype(float).reshape(h, w)
    z = (c - c.mean()) / c.std()
    if z[0].mean() > 0:
        lab = np.where(lab == 0.0, 0.5, lab)
        lab = np.where(lab == 1.0, 0.0, lab)
        lab = np.where(lab == 0.5, 1.0, lab)
    if not return_gap:
        return lab
    xf = x.reshape(h * w, d)
    dd = np.sort(np.stack([((xf - cc) ** 2).sum(1) for cc in c], 1), axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        gap = ((dd[:, 1] - dd[:, 0]) / dd[:, 1]).reshape(h, w)
    return lab, gap


def confidence_st(X, centers, labels):
    """``estimate_confidence_score_st`` (MILWRM.py:557-598)."""
    X = np.asarray(X, dtype=np.float64)
    d = np.zeros((X.shape[0], len(centers)))
    for i, c in enumerate(centers):
        d[:, i] += np.sum((X - c) ** 2, axis=1)
    s = np.sort(d, axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        cid = (s[:, 1] - s[:, 0]) / s[:, 1]
    means = {}
    for i in range(len(centers)):
        sel = labels == i
        means[i] = float(np.mean(cid[sel])) if sel.any() else np.nan
    return cid, means


def blur_features_st(features: np.ndarray, adjacency) -> np.ndarray:
    """``blur_features_st`` (ST.py:25-77): mean over the non-zero neighbours
    of each spot plus the spot itself (a self-loop counts twice)."""
    import scipy.sparse as sp

    A = sp.csr_matrix(adjacency)
    A.eliminate_zeros()
    out = np.empty_like(np.asarray(features, dtype=np.float64))
    F = np.asarray(features, dtype=np.float64)
    for x in range(F.shape[0]):
        nb = list(A.indices[A.indptr[x]:A.indptr[x + 1]]) + [x]
        out[x] = F[nb].mean(axis=0)
    return out


def mxif_pipeline(slides, masks, batches, features, k=8, sigma=2.0, fract=0.2,
                  random_state=18, confidence=True):
    """End-to-end reference pipeline (call stacks A, C, D, E of SURVEY §3):
    non-zero means → batch means → per image lognorm+blur+subsample →
    row_stack → StandardScaler → KMeans(k).fit → predict every pixel →
    confidence.  Used as the CPU baseline and as the end-to-end oracle."""
    ests, pix = zip(*[non_zero_mean(s) for s in slides])
    bm = batch_means(ests, pix, batches)
    pre, sub = [], []
    for s, m, b in zip(slides, masks, batches):
        x = gaussian_blur(log_normalize(s, bm[b]), sigma)
        pre.append(x)
        sub.append(subsample_pixels(x, m, features, fract)[0])
    X = np.vstack(sub)
    mean, scale, _ = scaler_fit(X)
    Xs = scaler_transform(X, mean, scale)
    km = kmeans_fit(Xs, k, random_state=random_state)
    tids, cids, cms = [], [], []
    for x, m in zip(pre, masks):
        t = tissue_ids(x, m, features, km["cluster_centers_"], mean, scale)
        tids.append(t)
        if confidence:
            c, cm = confidence_mxif(x, m, features, km["cluster_centers_"], mean, scale, t)
            cids.append(c)
            cms.append(cm)
    return dict(batch_means=bm, cluster_data=Xs, scaler_mean=mean, scaler_scale=scale,
                kmeans=km, tissue_IDs=tids, confidence_IDs=cids, confidence_means=cms,
                preprocessed=pre)


def synth_slide(h, w, c, seed, mode="hard", n_seeds=32, n_domains=8, bg_frac=0.15):
    """Synthetic structured MxIF slide (SURVEY §8d generator): Voronoi domains,
    lognormal per-domain channel profiles, gamma noise, top rows background
    (x0.05, mask 0); uint16 HWC + uint8 mask."""
    rng = np.random.default_rng(seed)
    sp_, shape = {"hard": (0.15, 1.0), "easy": (0.8, 4.0), "design": (0.07, 1.0)}[mode]
    sy = rng.uniform(0, h, n_seeds)
    sx = rng.uniform(0, w, n_seeds)
    dom_of_seed = np.arange(n_seeds) % n_domains
    prof = rng.lognormal(4.0, sp_, size=(n_domains, c))
    yy, xx = np.mgrid[0:h, 0:w]
    best = np.full((h, w), np.inf)
    dom = np.zeros((h, w), dtype=np.int64)
    for s in range(n_seeds):
        d = (yy - sy[s]) ** 2 + (xx - sx[s]) ** 2
        sel = d < best
        best[sel] = d[sel]
        dom[sel] = dom_of_seed[s]
    noise = rng.gamma(shape, 1.0 / shape, size=(h, w, c))
    img = prof[dom] * noise
    nbg = int(round(bg_frac * h))
    img[:nbg] *= 0.05
    mask = np.ones((h, w), dtype=np.uint8)
    mask[:nbg] = 0
    return np.clip(np.rint(img), 0, 65535).astype(np.uint16), mask
