"""sklearn-shaped estimators whose numerics run on the MI355X kernels.

``KMeans`` reproduces ``sklearn.cluster.KMeans(algorithm='lloyd')`` 1.7.2
(``_kmeans.py:1427-1554``): tolerance scaled by the mean feature variance
(:279-287), ``n_init='auto'`` → 1 for k-means++ (:879-881), k-means++ seeding
(:174-272), Lloyd with strict label-equality convergence or the center-shift
test (:624-752), empty-cluster relocation and averaging
(``_k_means_common.pyx:181-311``), the extra E-step when not strictly
converged, and inertia.  The data stay in HBM as fp32 rows with the
StandardScaler folded in as a per-feature affine (``DeviceRows``); the host
only sees k x F centers and a handful of scalars per iteration.

``StandardScaler`` carries sklearn's fitted attributes (mean_, var_, scale_,
n_samples_seen_) computed from device column statistics (Chan merge, fp64).
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from . import _native as N
from . import device as D
from . import profiling
from .rng import as_random_state, first_center_index, kpp_draws


class DeviceRows:
    """S x F fp32 rows in HBM, with x' = (x - mu) * inv applied on the fly."""

    def __init__(self, X: torch.Tensor, mu=None, inv=None, feature_var=None):
        assert X.dtype == torch.float32 and X.dim() == 2 and X.is_contiguous()
        self.X = X
        self.S, self.F = X.shape
        self.mu = np.zeros(self.F) if mu is None else np.asarray(mu, dtype=np.float64)
        self.inv = np.ones(self.F) if inv is None else np.asarray(inv, dtype=np.float64)
        dev = X.device
        self.mu64 = D.h2d(self.mu, dev)
        self.inv64 = D.h2d(self.inv, dev)
        self.a32 = D.h2d(self.inv.astype(np.float32), dev)
        self.b32 = D.h2d((-self.mu * self.inv).astype(np.float32), dev)
        self._feature_var = feature_var

    @classmethod
    def from_host(cls, X: np.ndarray) -> "DeviceRows":
        X = np.asarray(X)
        if X.ndim != 2:
            raise ValueError(f"Expected 2D array, got {X.ndim}D array instead")
        t = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(D.device())
        var = np.var(np.asarray(X, dtype=np.float64), axis=0)
        return cls(t, feature_var=var)

    def feature_var(self) -> np.ndarray:
        """Per-feature variance of the scaled rows (ddof=0)."""
        if self._feature_var is None:
            raise RuntimeError("feature variance unknown for these rows")
        return self._feature_var

    def scaled_rows(self, idx) -> np.ndarray:
        idx = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=self.X.device)
        x = D.d2h(self.X.index_select(0, idx).double())
        return (x - self.mu) * self.inv

    def to_host_scaled(self) -> np.ndarray:
        return (self.X.double().cpu().numpy() - self.mu) * self.inv


class StandardScaler:
    """Fitted-attribute twin of sklearn's StandardScaler (_data.py)."""

    def __init__(self, *, copy=True, with_mean=True, with_std=True):
        self.copy, self.with_mean, self.with_std = copy, with_mean, with_std

    def _set(self, n, mean, var):
        self.n_samples_seen_ = int(n)
        self.mean_ = np.asarray(mean, dtype=np.float64)
        self.var_ = np.asarray(var, dtype=np.float64)
        self.n_features_in_ = self.mean_.shape[0]
        eps = np.finfo(np.float64).eps
        constant = self.var_ <= n * eps * self.var_ + (n * self.mean_ * eps) ** 2  # _data.py:76-89
        scale = np.sqrt(self.var_)
        scale[constant] = 1.0
        self.scale_ = scale
        return self

    @classmethod
    def from_stats(cls, stats: np.ndarray) -> "StandardScaler":
        """From device Chan statistics [n, mean[F], M2[F]]."""
        n = stats[0]
        F = (len(stats) - 1) // 2
        return cls()._set(n, stats[1:1 + F], stats[1 + F:] / n)

    def fit(self, X, y=None):
        X = np.asarray(X, dtype=np.float64)
        return self._set(X.shape[0], X.mean(axis=0), X.var(axis=0))

    def transform(self, X, copy=None):
        X = np.array(X, dtype=np.float64, copy=True)
        if self.with_mean:
            X -= self.mean_
        if self.with_std:
            X /= self.scale_
        return X

    def fit_transform(self, X, y=None):
        return self.fit(X).transform(X)

    def inverse_transform(self, X, copy=None):
        X = np.array(X, dtype=np.float64, copy=True)
        if self.with_std:
            X *= self.scale_
        if self.with_mean:
            X += self.mean_
        return X

    def affine(self):
        """(mu, inv) of x' = (x - mu) * inv."""
        return self.mean_.copy(), 1.0 / self.scale_


# ----------------------------------------------------------------- k-means

def _kmeans_plusplus_device(rows: DeviceRows, k: int, random_state, n_local_trials=None):
    S, F = rows.S, rows.F
    T = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
    u0, steps = kpp_draws(random_state, k, T)
    first = first_center_index(S, u0)
    ws = D.WS.get("kpp", N.query("mw_kpp_ws_bytes", S, T))
    st = D.stream()
    with profiling.timed("kpp_init", S * (F * 4 + 8)):
        N.call("mw_kpp_init", D.P(rows.X), S, F, D.P(rows.mu64), D.P(rows.inv64),
               D.P(rows.X) + int(first) * F * 4, T, D.P(ws), st)
    for c in range(1, k):
        u = np.ascontiguousarray(steps[c - 1], dtype=np.float64)
        with profiling.timed("kpp_step", S * (F * 4 + 8 + 8 * T)):
            N.call("mw_kpp_step", D.P(rows.X), S, F, D.P(rows.mu64), D.P(rows.inv64), c,
                   u.ctypes.data, T, D.P(ws), st)
    idx = torch.empty(k, dtype=torch.int64, device=rows.X.device)
    N.call("mw_kpp_indices", D.P(ws), S, T, k, D.P(idx), st)
    idx = D.d2h(idx).copy()
    idx[0] = first
    return rows.scaled_rows(idx), idx


from .dist import LOCAL_COMM as LOCAL  # noqa: E402


def _relocate_empty(rows: DeviceRows, labels: torch.Tensor, centers_old, centers_new, weight,
                    comm):
    """_relocate_empty_clusters_dense (_k_means_common.pyx:181-226)."""
    empty = np.where(weight == 0)[0]
    n_empty = empty.size
    if n_empty == 0:
        return
    if comm.sharded():
        far_idx, far_val, xs, old_lab = comm.farthest(rows, labels, centers_old, n_empty)
    else:
        S, F = rows.S, rows.F
        k = centers_old.shape[0]
        c64 = D.h2d(centers_old, rows.X.device)
        top_i = torch.empty(n_empty, dtype=torch.int64, device=rows.X.device)
        top_v = torch.empty(n_empty, dtype=torch.float64, device=rows.X.device)
        ws = D.WS.get("far", N.query("mw_farthest_ws_bytes", S))
        N.call("mw_farthest", D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), D.P(c64), k,
               D.P(labels), int(n_empty), D.P(top_i), D.P(top_v), D.P(ws), D.stream())
        far_idx = top_i.cpu().numpy()
        far_val = top_v.cpu().numpy()
        xs = rows.scaled_rows(far_idx)
        old_lab = labels.index_select(0, top_i).cpu().numpy().astype(np.int64)
    if far_val.max() == 0:
        return
    for e, x, old in zip(empty, xs, old_lab):
        centers_new[old] -= x
        centers_new[e] = x
        weight[e] = 1.0
        weight[old] -= 1.0


def _average_centers(centers, weight):
    amax = int(np.argmax(weight))
    for j in range(centers.shape[0]):
        if weight[j] > 0:
            centers[j] *= 1.0 / weight[j]
        else:
            centers[j] = centers[amax]


def lloyd_device(rows: DeviceRows, centers_init: np.ndarray, max_iter=300, tol=0.0, verbose=False,
                 comm=LOCAL):
    """``_kmeans_single_lloyd`` on device.  Returns (labels u8 tensor, inertia,
    centers fp64, n_iter)."""
    S, F = rows.S, rows.F
    k = centers_init.shape[0]
    dev = rows.X.device
    labels = torch.full((S,), 255, dtype=torch.uint8, device=dev)  # = -1: nothing assigned
    ws = D.WS.get("lloyd", N.query("mw_lloyd_ws_bytes", S, k, F))
    rl = k * F + k + 2
    out = torch.empty(rl, dtype=torch.float64, device=dev)
    c32 = torch.empty((k, F), dtype=torch.float32, device=dev)
    centers = np.array(centers_init, dtype=np.float64)
    strict = False
    st = D.stream()

    def step(mode):
        D.h2d_into(c32, centers.astype(np.float32))
        with profiling.timed(f"lloyd_step_mode{mode}", S * (F * 4 + (2 if mode < 2 else 1))):
            N.call("mw_lloyd_step", D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), D.P(c32), k,
                   D.P(labels), mode, D.P(ws), st)
        N.call("mw_lloyd_reduce", D.P(ws), S, k, F, D.P(out), st)
        comm.all_reduce_(out)
        return D.d2h(out)

    i = 0
    for i in range(max_iter):
        rec = step(0)
        centers_new = rec[:k * F].reshape(k, F).copy()
        weight = rec[k * F:k * F + k].copy()
        changed = rec[k * F + k]
        _relocate_empty(rows, labels, centers, centers_new, weight, comm)
        _average_centers(centers_new, weight)
        shift = np.sqrt(((centers_new - centers) ** 2).sum(axis=1))
        centers = centers_new
        if verbose:
            print(f"Iteration {i}: {int(changed)} labels changed.")
        if changed == 0:
            strict = True
            if verbose:
                print(f"Converged at iteration {i}: strict convergence.")
            break
        if (shift ** 2).sum() <= tol:
            if verbose:
                print(f"Converged at iteration {i}: center shift within tolerance {tol}.")
            break
    rec = step(2 if strict else 1)
    inertia = float(rec[k * F + k + 1])
    return labels, inertia, centers, i + 1


def _mb_class(k: int) -> int:
    return 1 if k <= 16 else 2 if k <= 32 else 4


def lloyd_device_multi(rows: DeviceRows, inits, max_iter=300, tol=0.0, comm=LOCAL):
    """``lloyd_device`` for several independent fits over the same rows, run in
    lockstep: every iteration is ONE pass over the rows for all the fits
    still running (``mw_lloyd_step_multi``, fits of one M-step class per
    launch), one all-reduce and one device-to-host copy of all their records.
    Each fit's arithmetic is the single-fit kernel's, so every fit returns
    exactly what ``lloyd_device`` returns for it.  Returns a list of
    (labels u8 tensor, inertia, centers fp64, n_iter)."""
    S, F = rows.S, rows.F
    dev = rows.X.device
    n = len(inits)
    ks = [int(np.asarray(c).shape[0]) for c in inits]
    rls = [k * F + k + 2 for k in ks]
    roff = np.concatenate([[0], np.cumsum(rls)]).astype(np.int64)
    coff = np.concatenate([[0], np.cumsum([k * F for k in ks])]).astype(np.int64)
    out_all = torch.zeros(int(roff[-1]), dtype=torch.float64, device=dev)
    c32_all = torch.empty(int(coff[-1]), dtype=torch.float32, device=dev)
    host_c = np.zeros(int(coff[-1]), dtype=np.float32)
    labels = [torch.full((S,), 255, dtype=torch.uint8, device=dev) for _ in range(n)]
    wss = [torch.empty(N.query("mw_lloyd_ws_bytes", S, k, F), dtype=torch.uint8, device=dev)
           for k in ks]
    centers = [np.array(c, dtype=np.float64) for c in inits]
    done = [False] * n
    strict = [False] * n
    n_iter = [max_iter] * n
    st = D.stream()
    import ctypes

    def launch(group, mode):
        m = len(group)
        P = ctypes.c_void_p * m
        cp = P(*[D.P(c32_all) + int(coff[g]) * 4 for g in group])
        kk = (ctypes.c_int * m)(*[ks[g] for g in group])
        lp = P(*[D.P(labels[g]) for g in group])
        wp = P(*[D.P(wss[g]) for g in group])
        op = P(*[D.P(out_all) + int(roff[g]) * 8 for g in group])
        nbytes = sum(S * (F * 4 + (2 if mode < 2 else 1)) for _ in group)
        with profiling.timed(f"lloyd_multi_mode{mode}", nbytes):
            N.call("mw_lloyd_step_multi", D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), m,
                   ctypes.addressof(cp), ctypes.addressof(kk), ctypes.addressof(lp), mode,
                   ctypes.addressof(wp), ctypes.addressof(op), st)

    def run(sel, mode_of):
        """One pass for the fits in ``sel``; returns the host records."""
        for g in sel:
            host_c[coff[g]:coff[g + 1]] = centers[g].ravel()
        D.h2d_into(c32_all, host_c)
        classes = {}
        for g in sel:
            classes.setdefault((mode_of(g), _mb_class(ks[g])), []).append(g)
        for (mode, _), group in sorted(classes.items()):
            for i in range(0, len(group), 24):
                launch(group[i:i + 24], mode)
        comm.all_reduce_(out_all)
        return D.d2h(out_all)

    for it in range(max_iter):
        active = [g for g in range(n) if not done[g]]
        if not active:
            break
        rec_all = run(active, lambda g: 0)
        for g in active:
            k = ks[g]
            rec = rec_all[roff[g]:roff[g + 1]]
            centers_new = rec[:k * F].reshape(k, F).copy()
            weight = rec[k * F:k * F + k].copy()
            changed = rec[k * F + k]
            _relocate_empty(rows, labels[g], centers[g], centers_new, weight, comm)
            _average_centers(centers_new, weight)
            shift = np.sqrt(((centers_new - centers[g]) ** 2).sum(axis=1))
            centers[g] = centers_new
            if changed == 0:
                strict[g], done[g], n_iter[g] = True, True, it + 1
            elif (shift ** 2).sum() <= tol:
                done[g], n_iter[g] = True, it + 1
    rec_all = run(list(range(n)), lambda g: 2 if strict[g] else 1)
    return [(labels[g], float(rec_all[roff[g] + ks[g] * F + ks[g] + 1]), centers[g], n_iter[g])
            for g in range(n)]


def fit_many(rows: DeviceRows, k_values, random_state=None, comm=None, **kw):
    """``KMeans(n_clusters=k, random_state=random_state, **kw).fit(rows)`` for
    every k, with the Lloyd iterations of all fits batched
    (``lloyd_device_multi``); k-means++ seeding per fit as in ``KMeans.fit``.
    Returns the fitted estimators (bitwise equal to separate fits)."""
    comm = LOCAL if comm is None else comm
    models, inits = [], []
    for k in k_values:
        km = KMeans(n_clusters=int(k), random_state=random_state, **kw)
        km._check(rows.S)
        if km.n_init not in ("auto", 1) or not isinstance(km.init, str) or km.init != "k-means++":
            raise NotImplementedError("fit_many: k-means++ with a single init only")
        km._tol = float(np.mean(rows.feature_var()) * km.tol) if km.tol else 0.0
        seeded = isinstance(km.random_state, (int, np.integer)) and not isinstance(km.random_state, bool)
        c0, km.init_indices_ = km._kpp(rows, km.random_state if seeded else
                                       as_random_state(km.random_state), comm)
        models.append(km)
        inits.append(c0)
    tols = {km._tol for km in models}
    max_iters = {km.max_iter for km in models}
    assert len(tols) == 1 and len(max_iters) == 1
    res = lloyd_device_multi(rows, inits, max_iters.pop(), tols.pop(), comm)
    for km, (labels, inertia, centers, n_iter) in zip(models, res):
        km._set_fitted(rows, labels, inertia, centers, n_iter)
    return models


class KMeans:
    """Drop-in for ``sklearn.cluster.KMeans`` (lloyd) on the MI355X kernels.

    ``fit`` accepts a host array (standardised features, as MILWRM passes
    ``cluster_data``) or ``DeviceRows`` (HBM-resident rows with the scaler
    folded in).  Fitted attributes match sklearn's: ``cluster_centers_``
    (fp64), ``labels_`` (int32), ``inertia_``, ``n_iter_``."""

    def __init__(self, n_clusters=8, *, init="k-means++", n_init="auto", max_iter=300, tol=1e-4,
                 verbose=0, random_state=None, copy_x=True, algorithm="lloyd"):
        self.n_clusters = n_clusters
        self.init = init
        self.n_init = n_init
        self.max_iter = max_iter
        self.tol = tol
        self.verbose = verbose
        self.random_state = random_state
        self.copy_x = copy_x
        self.algorithm = algorithm

    # sklearn get_params/set_params subset (used by joblib-style callers)
    def get_params(self, deep=True):
        return dict(n_clusters=self.n_clusters, init=self.init, n_init=self.n_init,
                    max_iter=self.max_iter, tol=self.tol, verbose=self.verbose,
                    random_state=self.random_state, copy_x=self.copy_x, algorithm=self.algorithm)

    def set_params(self, **p):
        for k, v in p.items():
            setattr(self, k, v)
        return self

    def _check(self, S):
        if not isinstance(self.n_clusters, (int, np.integer)) or self.n_clusters < 1:
            raise ValueError(f"n_clusters must be a positive int, got {self.n_clusters!r}")
        if S < self.n_clusters:
            raise ValueError(f"n_samples={S} should be >= n_clusters={self.n_clusters}.")
        if self.algorithm not in ("lloyd", "auto", "full"):
            raise NotImplementedError("only algorithm='lloyd' is implemented on the device")
        if self.n_clusters > 64:
            raise NotImplementedError("n_clusters > 64 is not supported by the device kernels")

    def fit(self, X, y=None, sample_weight=None, comm=None):
        comm = LOCAL if comm is None else comm
        if sample_weight is not None and not np.all(np.asarray(sample_weight) == 1):
            raise NotImplementedError("non-unit sample_weight")
        rows = X if isinstance(X, DeviceRows) else DeviceRows.from_host(X)
        self._check(rows.S)
        k = int(self.n_clusters)
        self._tol = float(np.mean(rows.feature_var()) * self.tol) if self.tol else 0.0
        init = self.init
        arraylike = not isinstance(init, str) and not callable(init)
        if self.n_init == "auto":
            n_init = 1 if (arraylike or init == "k-means++") else 10
        else:
            n_init = int(self.n_init)
        if arraylike and n_init != 1:
            warnings.warn(f"Explicit initial center position passed: performing only one init in "
                          f"KMeans instead of n_init={n_init}.", RuntimeWarning, stacklevel=2)
            n_init = 1
        rs_box = []

        def rs():  # created on first use (a seeded single k-means++ init never needs it)
            if not rs_box:
                rs_box.append(as_random_state(self.random_state))
            return rs_box[0]

        best = None
        for _ in range(n_init):
            if arraylike:
                centers0 = np.array(init, dtype=np.float64)
                if centers0.shape != (k, rows.F):
                    raise ValueError(f"The shape of the initial centers {centers0.shape} does not "
                                     f"match the number of clusters {k} / features {rows.F}.")
                self.init_indices_ = None
            elif init == "k-means++":
                # a single init from an int seed draws from a fresh
                # RandomState(seed): pass the seed (memoised draws, rng.kpp_draws)
                seeded = n_init == 1 and isinstance(self.random_state, (int, np.integer)) \
                    and not isinstance(self.random_state, bool)
                centers0, self.init_indices_ = self._kpp(rows, self.random_state if seeded else rs(),
                                                         comm)
            elif init == "random":
                if comm.sharded():
                    raise NotImplementedError("init='random' with sharded rows")
                seeds = rs().choice(rows.S, size=k, replace=False,
                                  p=np.full(rows.S, 1.0 / rows.S))
                centers0, self.init_indices_ = rows.scaled_rows(seeds), seeds
            elif callable(init):
                raise NotImplementedError("callable init")
            else:
                raise ValueError(f"init should be 'k-means++', 'random' or an array, got {init!r}")
            labels, inertia, centers, n_iter = lloyd_device(rows, centers0, self.max_iter,
                                                            self._tol, bool(self.verbose), comm)
            if best is None or inertia < best[1]:
                best = (labels, inertia, centers, n_iter)
        return self._set_fitted(rows, *best)

    def _kpp(self, rows, rs, comm):
        if comm.sharded():
            return comm.kpp(rows, int(self.n_clusters), rs)
        return _kmeans_plusplus_device(rows, int(self.n_clusters), rs)

    def _set_fitted(self, rows, labels, inertia, centers, n_iter):
        self._labels_dev = labels
        self.cluster_centers_ = centers
        self.inertia_ = inertia
        self.n_iter_ = n_iter
        self.n_features_in_ = rows.F
        self._n_features_out = int(self.n_clusters)
        self._labels_host = None
        return self

    @property
    def labels_(self):
        if self._labels_host is None:
            self._labels_host = self._labels_dev.cpu().numpy().astype(np.int32)
        return self._labels_host

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight).labels_

    def predict(self, X):
        """Closest center per row (device pass, lowest index wins ties)."""
        from .assign import assign_rows

        X = np.asarray(X, dtype=np.float64)
        if X.ndim != 2 or X.shape[1] != self.cluster_centers_.shape[1]:
            raise ValueError("X has the wrong shape")
        lab, _, _ = assign_rows(X, self.cluster_centers_)
        return lab.astype(np.int32)
