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

import ctypes as C
import os
import warnings

import numpy as np
import torch

from . import _native as N
from . import device as D
from . import profiling
from .rng import as_random_state, first_center_index, kpp_draws


class DeviceRows:
    """S x F fp32 rows in HBM, with x' = (x - mu) * inv applied on the fly."""

    def __init__(self, X: torch.Tensor, mu=None, inv=None, feature_var=None, xmax_local=None):
        assert X.dtype == torch.float32 and X.dim() == 2 and X.is_contiguous()
        self.X = X
        self.S, self.F = X.shape
        self.mu = np.zeros(self.F) if mu is None else np.asarray(mu, dtype=np.float64)
        self.inv = np.ones(self.F) if inv is None else np.asarray(inv, dtype=np.float64)
        self.a_host = self.inv.astype(np.float32)
        self.b_host = (-self.mu * self.inv).astype(np.float32)
        self._dev_affine = None  # (mu64, inv64, a32, b32) on the device, uploaded on first use
        self._feature_var = feature_var
        self.xmax = None      # per-feature max |x| over all rows (all shards)
        # max |x| of this shard's rows when the producer already took it
        # (mw_col_stats_absmax beside the scaler statistics), else a pass
        self._xmax_local = None if xmax_local is None else np.asarray(xmax_local, np.float32)
        self.qexp_dev = None  # fixed-point exponents of the Lloyd M-step (int32, device)
        # the rows' draws (prep_cluster_data: [(row offset, rows, rank draws,
        # rank base)]): their order in the slides, for spatial_order()
        self.draws = None

    def spatial_order(self):
        """The permutation that puts the rows in slide (pixel) order, or None
        when the draws are not known.  Rows of neighbouring pixels have
        neighbouring values, so the rows the Lloyd bounds leave undecided (near
        domain boundaries) come in runs: the list passes' row gathers then
        read runs of consecutive rows instead of scattered ones."""
        if not self.draws or sum(S for _, S, _, _ in self.draws) != self.S:
            return None
        keys = torch.empty(self.S, dtype=torch.int64, device=self.X.device)
        for off, S, idx, base in self.draws:
            keys[off:off + S].copy_(idx)
            keys[off:off + S] += base
        return torch.sort(keys, stable=True)[1]

    def _affine(self):
        if self._dev_affine is None:  # one staged copy (the C fit driver uploads its own)
            self._dev_affine = D.h2d_many([self.mu, self.inv, self.a_host, self.b_host], self.X.device)
        return self._dev_affine

    @property
    def mu64(self):
        return self._affine()[0]

    @property
    def inv64(self):
        return self._affine()[1]

    @property
    def a32(self):
        return self._affine()[2]

    @property
    def b32(self):
        return self._affine()[3]

    def fixed_point(self, comm=None) -> np.ndarray:
        """Exponents e_f with max|x_f| * 2^e_f <= 2^40 (global over the shards
        of ``comm``), uploaded once; returns the fp64 factors 2^-e_f that turn
        a fixed-point sum back into a sum of x (lloyd.hip M-step)."""
        if self.qexp_dev is None:
            m = torch.empty(self.F, dtype=torch.float32, device=self.X.device)
            if self._xmax_local is not None:
                xmax = self._xmax_local.astype(np.float64)
            elif self.S:
                N.call("mw_col_absmax", D.P(self.X), self.S, self.F, D.P(m), D.stream())
                xmax = D.d2h(m).astype(np.float64)
            else:
                xmax = np.zeros(self.F)
            if comm is not None and comm.sharded():
                xmax = comm.all_reduce_max_np(xmax)
            self.xmax = xmax.astype(np.float32)
            e = np.array([_exp_below(float(v)) for v in xmax], dtype=np.int32)
            self.qexp = e
            self.qexp_dev = D.h2d(e, self.X.device)
        return np.ldexp(1.0, -self.qexp.astype(np.int64)).astype(np.float64)

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


def _round_f32(x, up: bool) -> np.ndarray:
    """fp64 -> fp32 rounded toward +inf (up) or -inf (down), elementwise."""
    x = np.asarray(x, dtype=np.float64)
    f = x.astype(np.float32)
    if up:
        bad = f.astype(np.float64) < x
        f[bad] = np.nextafter(f[bad], np.float32(np.inf))
    else:
        bad = f.astype(np.float64) > x
        f[bad] = np.nextafter(f[bad], np.float32(-np.inf))
    return f


def _bound_tables(c32: np.ndarray, prev32):
    """Per-center drift |c - c_prev| (rounded up), its max, and half the
    separation to the nearest other center (rounded down), from the fp32
    centers the device uses (lloyd.hip bound test).  MW_LLOYD_NOBOUND=1 (A/B
    and parity checks) makes every bound test fail: full E-step each pass."""
    c = c32.astype(np.float64)
    if os.environ.get("MW_LLOYD_NOBOUND") == "1":
        k = c.shape[0]
        return np.full(k, np.inf, np.float32), float("inf"), np.zeros(k, np.float32)
    k = c.shape[0]
    drift = np.zeros(k) if prev32 is None else np.sqrt(((c - prev32.astype(np.float64)) ** 2).sum(1))
    if k > 1:
        d2 = ((c[:, None, :] - c[None, :, :]) ** 2).sum(-1)
        np.fill_diagonal(d2, np.inf)
        half = 0.5 * np.sqrt(d2.min(1))
    else:
        half = np.full(1, np.inf)
    drift32 = _round_f32(drift, up=True)
    return drift32, float(drift32.max()), _round_f32(half, up=False)


def _exp_below(bound: float, bits: int = 40) -> int:
    """e with bound * 2^e <= 2^bits (0 for bound 0)."""
    if not np.isfinite(bound) or bound <= 0:
        return 0
    return bits - int(np.frexp(bound)[1])


def fit_memory_need(rows: DeviceRows, ks) -> int:
    """HBM bytes the Lloyd fits of ``ks`` allocate (labels, bounds, workspaces)."""
    S, F = rows.S, rows.F
    return sum(S * 9 + lloyd_ws_bytes(S, k, F) for k in ks)


def sort_memory_need(rows: DeviceRows) -> int:
    """HBM bytes of ``fit_many``'s row sort beside the rows: the sorted copy
    (S x F fp32), the int64 keys, the sort's values and indices (and its
    temporaries, ~ one more int64 pair per row)."""
    return rows.S * (rows.F * 4 + 8 + 16 + 16)


def _check_fit_memory(rows: DeviceRows, ks) -> None:
    """HBM for the fits run in lockstep (per fit: uint8 labels + fp32 upper /
    lower bounds per row, 9 bytes, and its pass workspace), checked before
    any allocation so a too-large sweep raises with the remedy instead of
    failing inside torch (find_optimal_k runs 19 fits together)."""
    from .stream import RESIDENCY

    need = fit_memory_need(rows, ks)
    free = RESIDENCY.release(need)  # resident copies of host-backed slides go first (stream.py)
    if need > free and rows.draws:
        rows.draws = None  # the rows' subsample draws (kept only for the sweep's row sort) go next
        torch.cuda.empty_cache()
        free = RESIDENCY.release(need)
    if need > free:
        S = rows.S
        raise MemoryError(
            f"{len(ks)} k-means fits over {S} rows need {need / 2**30:.1f} GiB of HBM for their "
            f"labels, bounds and workspaces and {free / 2**30:.1f} GiB are free: shard the rows "
            f"over more GPUs (milwrm_amd.dist) or lower fract")


class _FitState:
    """Host side of one Lloyd fit: fp64 centers, exact fixed-point cluster
    sums (int64 hi/lo limbs, value = hi * 2^32 + lo) and sizes, device labels
    and distance bounds."""

    def __init__(self, rows, centers, dev):
        S, F = rows.S, rows.F
        self.k = k = int(centers.shape[0])
        self.centers = np.array(centers, dtype=np.float64)
        self.prev32 = None
        self.q_hi = np.zeros((k, F), dtype=np.int64)
        self.q_lo = np.zeros((k, F), dtype=np.int64)
        self.count = np.zeros(k, dtype=np.int64)
        self.labels = torch.full((S,), 255, dtype=torch.uint8, device=dev)  # 255 = no label yet
        self.ub = torch.empty(S, dtype=torch.float32, device=dev)
        self.lb = torch.empty(S, dtype=torch.float32, device=dev)
        self.ws = torch.empty(lloyd_ws_bytes(S, k, F), dtype=torch.uint8, device=dev)
        self.done = False
        self.strict = False
        self.n_iter = 0
        self.recomputed = 0
        self.history = []  # (changed, recomputed) per pass
        self.iexp = 0
        self.drift_max = 0.0
        self.prev_dmax = 0.0
        self.bounds_ok = True  # ub / lb hold valid bounds (a dense pass does not keep them)

    def add(self, rec, F, qscale, a64, b64):
        """Apply a pass's record (mode 0): exact sums, sizes; returns the
        scaled per-cluster sums (fp64), the sizes and the changed count."""
        k = self.k
        hi = rec[:k * F].reshape(k, F).astype(np.int64)
        lo = rec[k * F:2 * k * F].reshape(k, F).astype(np.int64)
        self.q_hi += hi
        self.q_lo += lo
        carry = self.q_lo >> 32  # keep lo in [0, 2^32): every limb stays exact in fp64
        self.q_hi += carry
        self.q_lo -= carry << 32
        self.count += rec[2 * k * F:2 * k * F + k].astype(np.int64)
        tail = rec[2 * k * F + k:]
        self.recomputed += int(tail[1])
        self.history.append((int(tail[0]), int(tail[1])))
        sums_x = (self.q_hi.astype(np.float64) * 4294967296.0 + self.q_lo.astype(np.float64)) * qscale
        cnt = self.count.astype(np.float64)
        return a64[None, :] * sums_x + b64[None, :] * cnt[:, None], cnt, tail[0]


KIND_FIRST, KIND_TILE, KIND_QUEUE, KIND_LIST, KIND_DENSE = 0, 1, 2, 4, 5
# the batched sweep's dense pass (lloyd_dense2.h at F <= 30: x . C^T of every
# fit in the launch on the matrix cores, the norms folded into the two spare
# features, keyed top two, exact fp32 recheck of near ties) while at least this
# many fits run together; fewer -> the bounded passes.  Default at F <= 30
# (round 5, config 4 sweep: 0.50 s against 0.65 s with the bounded passes;
# DESIGN.md section 5); MW_LLOYD_DENSE=1 also takes F <= 64 (the grouped form,
# lloyd_dense.h: slower than the bounded passes there), 0 turns it off
DENSE_MIN_FITS = int(os.environ.get("MW_LLOYD_DENSE_MIN", "3"))
# fit_many's Lloyd passes over the rows in slide order (DeviceRows.spatial_order)
SWEEP_SORT = os.environ.get("MW_SWEEP_SORT", "1") != "0"
DENSE_MODE = os.environ.get("MW_LLOYD_DENSE", "auto")
USE_DENSE = DENSE_MODE != "0"
# the few-undecided pass: kList (bound test and list in one launch, the listed
# rows in a second) unless MW_LLOYD_LIST=0 (kQueue: both phases chunk by chunk
# in one kernel)
QUEUE_KIND = KIND_QUEUE if os.environ.get("MW_LLOYD_LIST") == "0" else KIND_LIST


def lloyd_ws_bytes(S: int, k: int, F: int) -> int:
    """A fit's pass workspace: the per-block records, plus the kList row lists
    (4 bytes per row) only when the passes can take kList."""
    return N.query("mw_lloyd_ws_bytes_kinds", S, k, F, int(QUEUE_KIND == KIND_LIST))
# a mode-0 pass streams every row (kTile) while the previous pass recomputed
# more than this fraction of the rows, else only the undecided ones (kQueue):
# the k = 2..20 sweep at 10k^2 x 30 (tools/sweep_bench.py) took 0.77 / 0.69 s
# at 0.12 / 0.3 (round 1: 1.05 / 1.03 / 0.90 s at 0.03 / 0.06 / 0.12).  Round
# 4, config 2 (profiles/r04/tried/queue_below): fit 7.44 ms at 0.3 against
# 7.6-8.1 at 0.1 / 0.2 / 0.5 / 0.7 / 1.0; the I = 17 design point 14.6 at 0.2,
# 14.9 at 0.3; the sweep 0.63 s at 0.3 / 0.5, 0.66 at 0.2
QUEUE_BELOW = float(os.environ.get("MW_LLOYD_QUEUE_BELOW", "0.3"))
# KMeans.fit through the C++ driver (mw_kmeans_fit) where it applies; MW_KMEANS_C=0
# keeps the Python loop (A/B and the per-pass trace)
USE_C_FIT = os.environ.get("MW_KMEANS_C", "1") != "0"


def _launch_pass(rows, fits_g, mode, kind, par, poff, outs, st, label="lloyd_pass"):
    """One mw_lloyd_pass over the rows for the fits in ``fits_g`` (list of
    (g, _FitState)), records folded into ``outs[g]``."""
    S, F = rows.S, rows.F
    arr = (N.LloydFit * len(fits_g))()
    nbytes = 0
    for i, (g, fs) in enumerate(fits_g):
        base = D.P(par) + int(poff[g]) * 4
        k = fs.k
        arr[i] = N.LloydFit(base, base + k * F * 4, base + (k * F + k) * 4, D.P(fs.labels),
                            D.P(fs.ub), D.P(fs.lb), D.P(fs.ws), D.P(outs[g]), k,
                            float(fs.drift_max), int(fs.iexp))
        if kind == KIND_DENSE:  # rows once per launch (counted with the first fit), labels per fit
            nbytes += 2 * S + (S * F * 4 if i == 0 else 0)
        else:
            nbytes += S * 9 + (S * F * 4 if (mode or kind not in (KIND_QUEUE, KIND_LIST)) else 0)
    tag = "" if mode else ("_first", "_tile", "_queue", "_first_atomic", "_list", "_dense", "_dense")[kind]
    ev = None
    if TRACE is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    with profiling.timed(f"{label}_mode{mode}{tag}", nbytes):
        N.call("mw_lloyd_pass", D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), D.P(rows.qexp_dev),
               len(fits_g), C.addressof(arr), int(mode), int(kind), st)
    if ev is not None:
        ev[1].record()
        TRACE.append({"mode": mode, "kind": tag.strip("_"), "fits": [g for g, _ in fits_g], "ev": ev})


TRACE = [] if os.environ.get("MW_LLOYD_TRACE") == "1" else None  # per-launch timing (diagnostics)


def trace_summary(fits_hist=None):
    """Resolve TRACE into [{mode, kind, n_fits, ms}] and clear it."""
    if TRACE is None:
        return []
    torch.cuda.synchronize()
    out = [{"mode": t["mode"], "kind": t["kind"], "n_fits": len(t["fits"]),
            "ms": round(t["ev"][0].elapsed_time(t["ev"][1]), 4)} for t in TRACE]
    TRACE.clear()
    return out


def lloyd_fits(rows: DeviceRows, inits, max_iter=300, tol=0.0, verbose=False, comm=LOCAL):
    """``_kmeans_single_lloyd`` (_kmeans.py:624-752) for one or several
    independent fits over the same rows, run in lockstep: every iteration is
    ONE mw_lloyd_pass for all the fits still running (up to 24 per launch),
    one all-reduce and one device-to-host copy of their records.  Each fit's
    arithmetic does not depend on which others run beside it, so a fit
    returns exactly what it returns alone.  Returns a list of (labels u8
    tensor, inertia, centers fp64, n_iter)."""
    S, F = rows.S, rows.F
    dev = rows.X.device
    n = len(inits)
    qscale = rows.fixed_point(comm)
    a64 = rows.a_host.astype(np.float64)
    b64 = rows.b_host.astype(np.float64)
    _check_fit_memory(rows, [int(np.asarray(c).shape[0]) for c in inits])
    fits = [_FitState(rows, c, dev) for c in inits]
    ks = [fs.k for fs in fits]
    rls = [N.query("mw_lloyd_rec_len", k, F) for k in ks]
    roff = np.concatenate([[0], np.cumsum(rls)]).astype(np.int64)
    S_glob, sizes = S, None
    if comm.sharded():
        sizes = comm.all_gather_np(np.array([S], dtype=np.int64))[:, 0]
        S_glob = int(sizes.sum())
    # the C driver on every rank (the same decision everywhere): one process, or
    # row shards that all hold rows (mw_lloyd_fits_sharded, the collectives
    # through _CommHook); the Python loop below otherwise (and for the trace)
    use_c = USE_C_FITS and TRACE is None and not verbose and (sizes is None or int(sizes.min()) >= 1)
    msg = None
    if use_c and sizes is not None:  # the records at the head of the message buffer
        msg = torch.zeros(N.query("mw_lloyd_fits_msg_len", int(roff[-1]), F, comm.world), dtype=torch.float64,
                          device=dev)
        out_all = msg[:int(roff[-1])]
    else:
        out_all = torch.zeros(int(roff[-1]), dtype=torch.float64, device=dev)
    outs = [out_all[roff[g]:roff[g + 1]] for g in range(n)]
    plen = [k * F + 2 * k for k in ks]  # per fit: centers | drift | half_sep (fp32)
    poff = np.concatenate([[0], np.cumsum(plen)]).astype(np.int64)
    par = torch.empty(int(poff[-1]), dtype=torch.float32, device=dev)
    host_par = np.zeros(int(poff[-1]), dtype=np.float32)
    st = D.stream()

    def upload(sel):
        for g in sel:
            fs = fits[g]
            k = fs.k
            c32 = fs.centers.astype(np.float32)
            drift, dmax, half = _bound_tables(c32, fs.prev32)
            if not fs.bounds_ok:  # after dense passes: every row recomputed, bounds rewritten
                drift, dmax = np.full(k, np.inf, np.float32), float("inf")
            fs.prev_dmax = fs.drift_max if fs.prev32 is not None else 0.0
            fs.prev32, fs.drift_max = c32, dmax
            o = int(poff[g])
            host_par[o:o + k * F] = c32.ravel()
            host_par[o + k * F:o + k * F + k] = drift
            host_par[o + k * F + k:o + k * F + 2 * k] = half
        D.h2d_into(par, host_par)

    def run(sel, mode, kind_of):
        by_kind = {}
        for g in sel:
            by_kind.setdefault(kind_of(g), []).append(g)
        for kind, gs in sorted(by_kind.items()):
            for i in range(0, len(gs), 24):
                _launch_pass(rows, [(g, fits[g]) for g in gs[i:i + 24]], mode, kind, par, poff,
                             outs, st)
        comm.all_reduce_(out_all)
        return D.d2h(out_all)

    first = 3 if os.environ.get("MW_LLOYD_FIRST_ATOMIC") == "1" else KIND_FIRST

    dense_now = [False]

    def kind_of(g):
        """First pass; then the dense pass while enough fits run together;
        else kTile or kQueue by the predicted share of undecided rows: the
        last pass's share scaled by how far the centers moved now relative to
        then (rows fail the bound test about in proportion to the drift)."""
        fs = fits[g]
        if not fs.history:
            return first
        if dense_now[0]:
            return KIND_DENSE
        if not fs.bounds_ok:
            return KIND_TILE
        frac = fs.history[-1][1] / max(S_glob, 1)
        if fs.prev_dmax > 0 and np.isfinite(fs.drift_max):
            frac *= min(1.0, fs.drift_max / fs.prev_dmax)
        return KIND_TILE if frac > QUEUE_BELOW else QUEUE_KIND

    # lloyd_dense2.h: F <= 30 (kD2MaxK 32); lloyd_dense.h: F <= 64, kDenseMaxFitK = 20
    dense_ok = USE_DENSE and F <= (64 if DENSE_MODE == "1" else 30) and max(ks) <= 20
    if use_c:
        hook = None
        if sizes is not None:
            hook = _CommHook(comm, msg, S_glob, int(sizes[:comm.rank].sum()))
        return _lloyd_fits_c(rows, fits, rls, out_all, par, max_iter, tol, dense_ok, first, st, hook)
    for it in range(max_iter):
        active = [g for g in range(n) if not fits[g].done]
        if not active:
            break
        dense_now[0] = dense_ok and it > 0 and len(active) >= DENSE_MIN_FITS
        upload(active)
        rec_all = run(active, 0, kind_of)
        for g in active:
            fs = fits[g]
            if it > 0:
                fs.bounds_ok = not dense_now[0]
            sums, weight, changed = fs.add(rec_all[roff[g]:roff[g + 1]], F, qscale, a64, b64)
            centers_new = sums.copy()
            _relocate_empty(rows, fs.labels, fs.centers, centers_new, weight, comm)
            _average_centers(centers_new, weight)
            shift = np.sqrt(((centers_new - fs.centers) ** 2).sum(axis=1))
            fs.centers = centers_new
            fs.n_iter = it + 1
            if verbose:
                print(f"Iteration {it}: {int(changed)} labels changed.")
            if changed == 0:
                fs.strict = fs.done = True
                if verbose:
                    print(f"Converged at iteration {it}: strict convergence.")
            elif (shift ** 2).sum() <= tol:
                fs.done = True
                if verbose:
                    print(f"Converged at iteration {it}: center shift within tolerance {tol}.")
            if fs.done:
                out_all[roff[g]:roff[g + 1]].zero_()
    for fs in fits:
        fs.n_iter = fs.n_iter if fs.done else max_iter
    # final pass: the extra E-step when not strictly converged, and inertia,
    # each fit in a fixed point from a bound on any row's squared distance
    xs = np.abs(a64) * rows.xmax.astype(np.float64) + np.abs(b64)
    xnorm = float(np.sqrt((xs ** 2).sum()))
    for fs in fits:
        cmax = float(np.sqrt((fs.centers ** 2).sum(1)).max())
        fs.iexp = _exp_below((xnorm + cmax) ** 2 * 1.01)
    upload(list(range(n)))
    for mode in (1, 2):
        sel = [g for g in range(n) if (2 if fits[g].strict else 1) == mode]
        for i in range(0, len(sel), 24):
            _launch_pass(rows, [(g, fits[g]) for g in sel[i:i + 24]], mode, KIND_FIRST, par, poff,
                         outs, st)
    comm.all_reduce_(out_all)
    rec_all = D.d2h(out_all)
    res = []
    for g, fs in enumerate(fits):
        tail = rec_all[roff[g + 1] - 4:roff[g + 1]]
        inertia = float((tail[2] * 4294967296.0 + tail[3]) * 2.0 ** -fs.iexp)
        res.append((fs.labels, inertia, fs.centers, fs.n_iter))
    LAST_STATS["recomputed"] = [fs.recomputed for fs in fits]
    LAST_STATS["history"] = [fs.history for fs in fits]
    return res


LAST_STATS = {}  # diagnostics of the last lloyd_fits call (rows recomputed per fit)
# lloyd_fits through the C++ driver (mw_lloyd_fits, csrc/fit.cpp) on one
# process; MW_LLOYD_FITS_C=0 keeps the Python loop (A/B, per-launch trace)
USE_C_FITS = os.environ.get("MW_LLOYD_FITS_C", "1") != "0"
_PASS_NAMES = ["lloyd_pass_mode0_first", "lloyd_pass_mode0_tile", "lloyd_pass_mode0_queue",
               "lloyd_pass_mode0_first_atomic", "lloyd_pass_mode0_list", "lloyd_pass_mode0_dense",
               "lloyd_pass_mode0_dense", "lloyd_pass_mode1", "lloyd_pass_mode2"]


FITS_C_USED = {"local": 0, "sharded": 0}  # lloyd_fits calls that ran the C driver (tests)


class _CommHook:
    """``mw_fit_comm`` over a ``dist.DistComm``: the C driver's collectives as
    the Python loop runs them (``comm.all_reduce_`` of the records, the
    relocation's all-gather), on slices of the message buffer ``msg`` whose
    head holds the fits' records."""

    def __init__(self, comm, msg: torch.Tensor, rows_total: int, row_offset: int):
        self.comm, self.msg, self.err = comm, msg, None
        self._ar = N.ALL_REDUCE_SUM_FN(self._all_reduce)
        self._ag = N.ALL_GATHER_FN(self._all_gather)
        self.struct = N.FitComm(None, comm.world, comm.rank, int(rows_total), int(row_offset), D.P(msg),
                                msg.numel(), self._ar, self._ag)
        self.reduces = 0

    def _all_reduce(self, ctx, off, n, stream):
        try:
            self.comm.all_reduce_(self.msg[off:off + n])
            self.reduces += 1
            return 0
        except BaseException as e:  # noqa: BLE001  (re-raised after the C call returns)
            self.err = e
            return 1

    def _all_gather(self, ctx, in_off, n, out_off, stream):
        try:
            g = self.comm.all_gather_t(self.msg[in_off:in_off + n])
            self.msg[out_off:out_off + self.comm.world * n].copy_(
                torch.from_numpy(np.ascontiguousarray(g, dtype=np.float64).reshape(-1)))
            return 0
        except BaseException as e:  # noqa: BLE001
            self.err = e
            return 1


def _lloyd_fits_c(rows, fits, rls, out_all, par, max_iter, tol, dense_ok, first, st, hook=None):
    """lloyd_fits' iterations in mw_lloyd_fits (the same host arithmetic and
    pass-kind policy in C++: no Python between the passes); over row shards
    (``hook``) in mw_lloyd_fits_sharded, one all-reduce of the records per
    pass through the hook."""
    S, F = rows.S, rows.F
    n = len(fits)
    ptrs = lambda ts: (C.c_void_p * n)(*[D.P(t) for t in ts])  # noqa: E731
    h_k = np.array([fs.k for fs in fits], dtype=np.int32)
    h_init = np.ascontiguousarray(np.concatenate([fs.centers.ravel() for fs in fits]), dtype=np.float64)
    centers = np.empty_like(h_init)
    inertia = np.empty(n, dtype=np.float64)
    n_iter = np.empty(n, dtype=np.int32)
    hist = np.zeros((n, max_iter, 2), dtype=np.int64)
    hist_len = np.zeros(n, dtype=np.int32)
    timing = np.zeros(30, dtype=np.float64) if profiling.enabled() else None
    a32 = np.ascontiguousarray(rows.a_host, dtype=np.float32)
    b32 = np.ascontiguousarray(rows.b_host, dtype=np.float32)
    qexp = np.ascontiguousarray(rows.qexp, dtype=np.int32)
    xmax = np.ascontiguousarray(rows.xmax, dtype=np.float32)
    mu = np.ascontiguousarray(rows.mu, dtype=np.float64)
    inv = np.ascontiguousarray(rows.inv, dtype=np.float64)
    nobound = int(os.environ.get("MW_LLOYD_NOBOUND") == "1")
    args = (D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), D.P(rows.qexp_dev),
            a32.ctypes.data, b32.ctypes.data, qexp.ctypes.data, xmax.ctypes.data, mu.ctypes.data,
            inv.ctypes.data, n, h_k.ctypes.data, h_init.ctypes.data,
            ptrs([fs.labels for fs in fits]), ptrs([fs.ub for fs in fits]), ptrs([fs.lb for fs in fits]),
            ptrs([fs.ws for fs in fits]), D.P(par), D.P(out_all), int(max_iter), float(tol), int(first),
            int(QUEUE_KIND), float(QUEUE_BELOW), int(DENSE_MIN_FITS) if dense_ok else -1, nobound,
            centers.ctypes.data, inertia.ctypes.data, n_iter.ctypes.data, hist.ctypes.data, int(max_iter),
            hist_len.ctypes.data, None if timing is None else timing.ctypes.data)
    if hook is None:
        N.call("mw_lloyd_fits", *args, st)
        FITS_C_USED["local"] += 1
    else:
        status = N.load().mw_lloyd_fits_sharded(*args, C.byref(hook.struct), st)
        if hook.err is not None:
            raise hook.err
        N.check(status, "mw_lloyd_fits_sharded")
        FITS_C_USED["sharded"] += 1
    if timing is not None:
        for slot, name in enumerate(_PASS_NAMES):
            profiling.add_measured(name, int(timing[3 * slot]), timing[3 * slot + 1], timing[3 * slot + 2])
        # host time between passes (no device work): per-iteration overhead of the driver
        profiling.add_measured("lloyd_fits_host", int(timing[27]), timing[28], 0)
        if hook is not None:
            profiling.add_measured("lloyd_fits_comm", int(timing[27]), timing[29], 0)
    res = []
    o = 0
    for g, fs in enumerate(fits):
        kF = fs.k * F
        fs.centers = centers[o:o + kF].reshape(fs.k, F).copy()
        o += kF
        fs.history = [tuple(int(v) for v in h) for h in hist[g, :hist_len[g]]]
        fs.recomputed = int(hist[g, :hist_len[g], 1].sum())
        res.append((fs.labels, float(inertia[g]), fs.centers, int(n_iter[g])))
    LAST_STATS["recomputed"] = [fs.recomputed for fs in fits]
    LAST_STATS["history"] = [fs.history for fs in fits]
    return res


def lloyd_device(rows: DeviceRows, centers_init: np.ndarray, max_iter=300, tol=0.0, verbose=False,
                 comm=LOCAL):
    """``_kmeans_single_lloyd`` on device.  Returns (labels u8 tensor, inertia,
    centers fp64, n_iter)."""
    return lloyd_fits(rows, [centers_init], max_iter, tol, verbose, comm)[0]


def lloyd_step_device(rows: DeviceRows, centers: np.ndarray, comm=LOCAL):
    """One Lloyd iteration from ``centers`` with no prior labels
    (lloyd_iter_chunked_dense): (labels u8 tensor, per-cluster sums of the
    scaled rows fp64, cluster sizes)."""
    qscale = rows.fixed_point(comm)
    fs = _FitState(rows, centers, rows.X.device)
    F = rows.F
    rl = N.query("mw_lloyd_rec_len", fs.k, F)
    out = torch.zeros(rl, dtype=torch.float64, device=rows.X.device)
    c32 = fs.centers.astype(np.float32)
    drift, dmax, half = _bound_tables(c32, None)
    fs.drift_max = dmax
    par = D.h2d(np.concatenate([c32.ravel(), drift, half]).astype(np.float32), rows.X.device)
    _launch_pass(rows, [(0, fs)], 0, KIND_FIRST, par, np.zeros(1, dtype=np.int64), [out], D.stream())
    comm.all_reduce_(out)
    sums, weight, _ = fs.add(D.d2h(out), F, qscale, rows.a_host.astype(np.float64),
                             rows.b_host.astype(np.float64))
    return fs.labels, sums, weight


def lloyd_device_multi(rows: DeviceRows, inits, max_iter=300, tol=0.0, comm=LOCAL):
    """``lloyd_device`` for several fits, batched (see lloyd_fits)."""
    return lloyd_fits(rows, inits, max_iter, tol, False, comm)


def fit_many(rows: DeviceRows, k_values, random_state=None, comm=None, **kw):
    """``KMeans(n_clusters=k, random_state=random_state, **kw).fit(rows)`` for
    every k, with the Lloyd iterations of all fits batched (``lloyd_fits``).

    k-means++ with an int seed draws from a fresh RandomState(seed) per fit:
    the first center and each step's n_local_trials = 2 + int(ln k) uniforms
    (_kmeans.py:225-243) are the same for every k with the same
    n_local_trials, so the centers of such a k are a prefix of the largest k's
    (groups {2}, {3..7}, {8..20} for k = 2..20).  One seeding per group serves
    all its k.  Returns the fitted estimators (bitwise equal to separate
    fits)."""
    comm = LOCAL if comm is None else comm
    models = []
    for k in k_values:
        km = KMeans(n_clusters=int(k), random_state=random_state, **kw)
        km._check(rows.S)
        if km.n_init not in ("auto", 1) or not isinstance(km.init, str) or km.init != "k-means++":
            raise NotImplementedError("fit_many: k-means++ with a single init only")
        km._tol = float(np.mean(rows.feature_var()) * km.tol) if km.tol else 0.0
        models.append(km)
    seeded = isinstance(random_state, (int, np.integer)) and not isinstance(random_state, bool)
    inits = [None] * len(models)
    if seeded:
        groups = {}
        for i, km in enumerate(models):
            groups.setdefault(2 + int(np.log(km.n_clusters)), []).append(i)
        for T, idx in groups.items():
            kmax = max(models[i].n_clusters for i in idx)
            big = KMeans(n_clusters=kmax, random_state=random_state)
            c0, ii = big._kpp(rows, random_state, comm)
            for i in idx:
                k = models[i].n_clusters
                inits[i], models[i].init_indices_ = c0[:k].copy(), ii[:k].copy()
    else:
        for i, km in enumerate(models):
            inits[i], km.init_indices_ = km._kpp(rows, as_random_state(km.random_state), comm)
    tols = {km._tol for km in models}
    max_iters = {km.max_iter for km in models}
    assert len(tols) == 1 and len(max_iters) == 1
    # the Lloyd passes over the rows in slide order (same scaler and fixed
    # point: the M-step sums are exact integers and every other output is per
    # row, so the fits are bit for bit those over the draw order; labels go
    # back to draw order below)
    # (only when HBM holds the sorted copy and its sort beside the fits'
    # state: otherwise the fits run over the draw order, the same bits)
    perm = None
    if SWEEP_SORT and len(models) > 1 and rows.draws:
        from .stream import RESIDENCY
        need = fit_memory_need(rows, [km.n_clusters for km in models]) + sort_memory_need(rows)
        if RESIDENCY.release(need) >= need:
            perm = rows.spatial_order()
    lrows = rows
    if perm is not None:
        lrows = DeviceRows(rows.X.index_select(0, perm), rows.mu, rows.inv, feature_var=rows._feature_var,
                           xmax_local=rows._xmax_local)
        lrows.xmax, lrows.qexp_dev = rows.xmax, rows.qexp_dev
        if rows.qexp_dev is not None:
            lrows.qexp = rows.qexp
    res = lloyd_fits(lrows, inits, max_iters.pop(), tols.pop(), False, comm)
    del lrows
    for km, (labels, inertia, centers, n_iter) in zip(models, res):
        if perm is not None:
            back = torch.empty_like(labels)
            back[perm] = labels
            labels = back
        km._set_fitted(rows, labels, inertia, centers, n_iter)
    return models


class _Inertia:
    """The inertia of a fit whose final E-step is still queued: its record in
    page-locked memory and the event after its copy (mw_kmeans_fit_async)."""

    def __init__(self, event, rec: torch.Tensor, iexp: int):
        self.event, self.rec, self.iexp = event, rec, int(iexp)

    def value(self) -> float:
        self.event.synchronize()
        r = self.rec.numpy()
        return float((r[-2] * 4294967296.0 + r[-1]) * 2.0 ** -self.iexp)


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

        # the C driver draws k-means++ from RandomState(seed) itself: an int
        # seed NumPy accepts (0 <= seed < 2^32; others go through
        # check_random_state on the Python path and raise as sklearn does)
        seeded_int = isinstance(self.random_state, (int, np.integer)) \
            and not isinstance(self.random_state, bool) and 0 <= int(self.random_state) < 2**32
        if (n_init == 1 and not comm.sharded() and not self.verbose and USE_C_FIT
                and (arraylike or (init == "k-means++" and seeded_int))):
            return self._set_fitted(rows, *self._fit_c(rows, k, init if arraylike else None))
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

    def _fit_c(self, rows, k, init):
        """The whole fit in the C++ driver (mw_kmeans_fit, csrc/fit.cpp): the
        same control flow and fp64 host arithmetic as the Python path below
        (bitwise the same result, tests/test_gpu_fit_c.py), without a Python
        round trip per Lloyd iteration."""
        S, F = rows.S, rows.F
        mu = np.ascontiguousarray(rows.mu, dtype=np.float64)
        inv = np.ascontiguousarray(rows.inv, dtype=np.float64)
        var = np.ascontiguousarray(rows.feature_var(), dtype=np.float64) if self.tol else None
        xmax = None if rows._xmax_local is None else np.ascontiguousarray(rows._xmax_local, np.float32)
        c0 = None
        if init is not None:
            c0 = np.ascontiguousarray(np.array(init, dtype=np.float64))
            if c0.shape != (k, F):
                raise ValueError(f"The shape of the initial centers {c0.shape} does not "
                                 f"match the number of clusters {k} / features {F}.")
        labels = torch.empty(S, dtype=torch.uint8, device=rows.X.device)
        centers = np.zeros((k, F))
        n_iter, iexp = C.c_int(), C.c_int()
        idx = np.full(k, -1, dtype=np.int64)
        nb = N.query("mw_kmeans_fit_ws_bytes", S, F, k)
        from .stream import RESIDENCY

        RESIDENCY.release(nb + S + (64 << 20))  # workspace + labels; host-backed slide copies go first
        ws = D.WS.get("kfit", nb)
        # the final E-step's record lands here when the stream gets there: the
        # fit returns with that pass queued, so whatever the caller queues next
        # (the label pass) follows it without a host round trip (_Inertia)
        rec = torch.empty(N.query("mw_lloyd_rec_len", k, F), dtype=torch.float64, pin_memory=True)
        with profiling.timed("kmeans_fit", 0):
            N.call("mw_kmeans_fit_async", D.P(rows.X), S, F, mu.ctypes.data, inv.ctypes.data,
                   None if var is None else var.ctypes.data,
                   None if xmax is None else xmax.ctypes.data, k,
                   None if c0 is None else c0.ctypes.data,
                   0 if c0 is not None else int(self.random_state),  # unused with an array init
                   int(self.max_iter), float(self.tol or 0.0), D.P(labels), centers.ctypes.data,
                   C.addressof(n_iter), idx.ctypes.data, D.P(ws), ws.numel(), rec.data_ptr(),
                   C.addressof(iexp), D.stream())
            done = torch.cuda.Event()
            done.record()
        self.init_indices_ = None if c0 is not None else idx
        return labels, _Inertia(done, rec, iexp.value), centers, n_iter.value

    def _kpp(self, rows, rs, comm):
        if comm.sharded():
            return comm.kpp(rows, int(self.n_clusters), rs)
        return _kmeans_plusplus_device(rows, int(self.n_clusters), rs)

    def _set_fitted(self, rows, labels, inertia, centers, n_iter):
        self._labels_dev = labels
        self.cluster_centers_ = centers
        self._inertia = inertia
        self.n_iter_ = n_iter
        self.n_features_in_ = rows.F
        self._n_features_out = int(self.n_clusters)
        self._labels_host = None
        return self

    @property
    def inertia_(self) -> float:
        """sklearn's inertia_ (a fit through mw_kmeans_fit_async reads its final
        record on first access, after the stream has reached it)."""
        if isinstance(self._inertia, _Inertia):
            self._inertia = self._inertia.value()
        return self._inertia

    @inertia_.setter
    def inertia_(self, v):
        self._inertia = v

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
