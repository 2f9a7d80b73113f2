"""Pixel-sharded multi-GPU execution (one process per GPU, RCCL over xGMI via
``torch.distributed`` backend "nccl").

Sharding: each rank owns whole slides (image_df rows); the clustering rows
of a rank are its slides' subsamples, and the global row order is rank order
(= image_df order when slides are dealt to ranks in order).  Every exchange
is a small fixed-size message:

  * batch means            all-gather of (C+1) fp64 per batch, once
  * scaler statistics      all-gather of each image's (1+2F) fp64, Chan-merged
                           in global image order (the single-process sequence)
  * k-means++ per step     all-gather of T local potentials; all-reduce of the
                           T candidate rows (owner contributes, others zero)
  * Lloyd fixed point      one MAX all-reduce of the F column maxima
  * Lloyd per iteration    ONE all-reduce of the fits' records: 2kF + k + 4
                           integer-valued fp64 limbs each (fixed-point sums,
                           counts, changed labels, inertia) -- exact, so
                           centers, labels and inertia are bitwise those of
                           one process for any sharding
  * empty-cluster relocation (rare) all-gather of local top-n (dist, index)

With world_size 1 every method is the identity (``LocalComm``), so the
single-GPU path runs the same code.  Tested with ``gloo`` on CPU tensors for
the host-side logic (tests/test_dist_gloo.py).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist


class LocalComm:
    world = 1
    rank = 0

    def batch_stats(self, est, pix):
        return est, pix

    def sum_batches(self, per_batch):
        return per_batch

    def merge_stats(self, stats: np.ndarray, F: int) -> np.ndarray:
        return stats

    def merge_image_stats(self, per_image: np.ndarray, F: int) -> np.ndarray:
        """[n, mean[F], M2[F]] of all images from per-image rows, Chan-merged
        in image order (images with n = 0 contribute nothing)."""
        return chan_merge(per_image, F)

    def all_reduce_(self, t: torch.Tensor):
        return t

    def all_reduce_max_np(self, a: np.ndarray) -> np.ndarray:
        return np.asarray(a)

    def sharded(self) -> bool:
        return False


def _chan(n_a, m_a, q_a, n_b, m_b, q_b):
    if n_b == 0:
        return n_a, m_a, q_a
    if n_a == 0:
        return n_b, m_b.copy(), q_b.copy()
    n = n_a + n_b
    d = m_b - m_a
    return n, m_a + d * (n_b / n), q_a + q_b + d * d * (n_a * n_b / n)


def chan_merge(per_image: np.ndarray, F: int) -> np.ndarray:
    n, m, q = 0.0, np.zeros(F), np.zeros(F)
    for row in np.asarray(per_image, dtype=np.float64).reshape(-1, 1 + 2 * F):
        n, m, q = _chan(n, m, q, row[0], row[1:1 + F], row[1 + F:])
    return np.concatenate([[n], m, q])


class DistComm(LocalComm):
    """Collectives on the default process group.  ``device`` is where the
    message tensors live (cuda for RCCL, cpu for gloo tests)."""

    def __init__(self, device=None, group=None, force=False):
        """``force``: run the sharded code path (every collective) even on a
        one-rank group -- how the RCCL message path is exercised on a single
        GPU (tests/test_gpu_nccl.py); results must equal ``LocalComm``'s."""
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) \
                if dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.device = device
        self.force = bool(force)

    def sharded(self) -> bool:
        return self.world > 1 or self.force

    # -- primitives ------------------------------------------------------
    def all_gather_np(self, a: np.ndarray) -> np.ndarray:
        """[world, *a.shape] in rank order."""
        return self.all_gather_t(torch.as_tensor(np.ascontiguousarray(a)))

    def all_gather_t(self, t: torch.Tensor) -> np.ndarray:
        """All-gather of a tensor living anywhere (device results stay on the
        device until the one host copy of the gathered block): [world, *shape]
        host array in rank order."""
        t = t.to(self.device).contiguous()
        out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=self.device)
        dist.all_gather_into_tensor(out, t.reshape(-1), group=self.group)
        return out.reshape((self.world,) + tuple(t.shape)).cpu().numpy()

    def all_reduce_(self, t: torch.Tensor):
        if t.device != self.device:
            tmp = t.to(self.device)
            dist.all_reduce(tmp, group=self.group)
            t.copy_(tmp)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def all_to_all_counts(self, counts):
        """counts[d] sent to rank d -> counts received from each rank."""
        t = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=self.device)
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=self.group)
        return out.cpu().tolist()

    def all_to_all_single(self, out, src, out_splits, in_splits):
        dist.all_to_all_single(out, src, out_splits, in_splits, group=self.group)

    def all_reduce_max_np(self, a: np.ndarray) -> np.ndarray:
        t = torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=self.device).clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.cpu().numpy()

    # -- preprocessing statistics --------------------------------------
    def batch_stats(self, est, pix):
        """Single-batch convenience: global (sum of estimators, sum of pixels)."""
        g = self.all_gather_np(np.concatenate([np.asarray(est, dtype=np.float64), [float(pix)]]))
        tot = np.zeros_like(g[0])
        for r in range(self.world):
            tot = tot + g[r]
        return list(tot[:-1]), int(round(tot[-1]))

    def sum_batches(self, per_batch: dict) -> dict:
        """{batch: (est_sum[C], pixels)} summed over ranks in rank order."""
        names = sorted(self.all_gather_names(list(per_batch)))
        C = len(next(iter(per_batch.values()))[0]) if per_batch else 0
        C = int(max(self.all_gather_np(np.array([C], dtype=np.int64))[:, 0]))
        vec = np.zeros((len(names), C + 1))
        for i, n in enumerate(names):
            if n in per_batch:
                vec[i, :C] = per_batch[n][0]
                vec[i, C] = per_batch[n][1]
        g = self.all_gather_np(vec)
        out = {}
        for i, n in enumerate(names):
            tot = np.zeros(C + 1)
            for r in range(self.world):
                tot = tot + g[r, i]
            out[n] = (tot[:C], tot[C])
        return out

    def all_gather_names(self, names):
        objs = [None] * self.world
        dist.all_gather_object(objs, names, group=self.group)
        return set(x for o in objs for x in o)

    def merge_image_stats(self, per_image: np.ndarray, F: int) -> np.ndarray:
        """Per-image statistics of every rank (ranks hold consecutive images),
        Chan-merged in global image order: the single-process sequence."""
        lists = [None] * self.world
        dist.all_gather_object(lists, np.asarray(per_image, dtype=np.float64).reshape(-1, 1 + 2 * F),
                               group=self.group)
        return chan_merge(np.concatenate(lists, axis=0), F)

    def merge_stats(self, stats: np.ndarray, F: int) -> np.ndarray:
        """Chan-merge per-rank [n, mean[F], M2[F]] in rank order."""
        g = self.all_gather_np(np.asarray(stats, dtype=np.float64))
        n, m, q = 0.0, np.zeros(F), np.zeros(F)
        for r in range(self.world):
            n, m, q = _chan(n, m, q, g[r, 0], g[r, 1:1 + F], g[r, 1 + F:])
        return np.concatenate([[n], m, q])

    # -- k-means++ over row shards -------------------------------------
    def kpp(self, rows, k, random_state, n_local_trials=None, engine=None):
        """sklearn ``_kmeans_plusplus`` (_kmeans.py:174-272) over row shards.
        Per step: each rank's local potentials of the T trial arrays are
        all-gathered and summed in rank order (global argmin, first wins);
        each target ``u_t * pot`` is owned by the first rank whose prefix of
        the best array's local potentials reaches it, and that rank searches
        its shard for ``target - prefix``; the candidates' global indices and
        raw rows travel as ONE all-reduced T x (1 + F) fp64 message (owner
        contributes, others zero; fp32 rows and indices < 2^53 are exact in
        fp64).  One host synchronisation per step (the gathered potentials,
        which the host needs for the targets); the chosen indices and rows
        stay on the device until the end.  ``engine`` holds the local
        distance arrays (``DeviceKpp``: the mw_kpp_* kernels; tests substitute
        a host one)."""
        from .rng import first_center_index, kpp_draws

        S, F = rows.S, rows.F
        T = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
        eng = DeviceKpp(rows, T) if engine is None else engine
        sizes = self.all_gather_np(np.array([S], dtype=np.int64))[:, 0]
        offs = np.concatenate([[0], np.cumsum(sizes)])
        S_tot = int(offs[-1])
        off = int(offs[self.rank])
        u0, steps = kpp_draws(random_state, k, T)

        first = first_center_index(S_tot, u0)
        msg = self._owned_rows(eng, [first - off if off <= first < off + S else -1], off)
        chosen = [msg[0, 0]]
        chosen_rows = [msg[0, 1:]]
        eng.init(msg[0, 1:].float().contiguous())
        cand = None
        self.kpp_host_ms = []  # per step: host time from the sync to the next trial pass queued
        for c in range(1, k + 1):
            n_arr = 1 if c == 1 else T
            g = self.all_gather_t(eng.pots_t(c, n_arr))  # [world, n_arr]: the step's one sync
            t_sync = time.perf_counter()
            tot = np.zeros(n_arr)
            for r in range(self.world):
                tot = tot + g[r]
            best = int(np.argmin(tot)) if c >= 2 else 0
            if c >= 2:
                chosen.append(cand[best, 0])
                chosen_rows.append(cand[best, 1:])
            if c == k:
                break
            rv_local = kpp_targets(np.asarray(steps[c - 1], dtype=np.float64) * tot[best],
                                   g[:, best], self.rank)
            cand = self._owned_rows(eng, eng.search_t(c, best, rv_local), off)
            eng.trial(c, best, cand[:, 1:].float().contiguous())
            self.kpp_host_ms.append((time.perf_counter() - t_sync) * 1e3)
        out = torch.cat([torch.stack(chosen)[:, None], torch.stack(chosen_rows)], 1).cpu().numpy()
        return (out[:, 1:] - rows.mu) * rows.inv, out[:, 0].astype(np.int64)

    def _owned_rows(self, eng, loc, off):
        """[n, 1 + F] fp64 on the engine's device: (global index, raw row) of
        the entries this rank owns (``loc`` = local row or -1), summed over the
        ranks (exactly one owner per entry, zeros elsewhere)."""
        loc = torch.as_tensor(loc, dtype=torch.int64).to(eng.device)
        have = loc >= 0
        X = eng.rows_at(loc.clamp(min=0))
        X = torch.where(have[:, None], X, torch.zeros_like(X)).double()
        gi = torch.where(have, loc + off, torch.zeros_like(loc)).double()
        msg = torch.cat([gi[:, None], X], 1)
        self.all_reduce_(msg)
        return msg

    # -- empty-cluster relocation --------------------------------------
    def farthest(self, rows, labels, centers_old, n, local_top=None):
        """The n rows farthest from their own center over all shards
        (_relocate_empty_clusters_dense's argpartition, _k_means_common.pyx:
        181-226): each rank's local top n (``mw_farthest``; ``local_top(m)``
        -> (values, local indices) substitutes it in tests) are all-gathered
        and ordered by (distance desc, global index asc); the winners' raw
        rows and labels are all-reduced from their owners.  Returns (global
        indices, distances, scaled rows, old labels)."""
        S, F = rows.S, rows.F
        dev = rows.X.device
        sizes = self.all_gather_np(np.array([S], dtype=np.int64))[:, 0]
        off = int(np.concatenate([[0], np.cumsum(sizes)])[self.rank])
        m = min(n, S)
        vi = np.full((n, 2), -1.0)
        if m > 0:
            top_v, top_i = (local_top or _device_far(rows, labels, centers_old))(m)
            vi[:m, 0] = top_v[:m]
            vi[:m, 1] = top_i[:m] + off
        g = self.all_gather_np(vi).reshape(-1, 2)
        g = g[g[:, 1] >= 0]
        order = np.lexsort((g[:, 1], -g[:, 0]))[:n]
        sel = g[order]
        far_idx = sel[:, 1].astype(np.int64)
        far_val = sel[:, 0]
        # the winners' raw rows and labels from their owners: one message
        loc = np.where((far_idx >= off) & (far_idx < off + S), far_idx - off, -1)
        loc_t = torch.as_tensor(loc, dtype=torch.int64, device=dev)
        have = (loc_t >= 0)[:, None]
        li = loc_t.clamp(min=0)
        part = torch.cat([rows.X.index_select(0, li).double(),
                          torch.as_tensor(labels).to(dev).index_select(0, li).double()[:, None]], 1)
        buf = torch.where(have, part, torch.zeros_like(part))
        self.all_reduce_(buf)
        b = buf.cpu().numpy()
        xs = (b[:, :F] - rows.mu) * rows.inv
        return far_idx, far_val, xs, b[:, F].astype(np.int64)


def _device_far(rows, labels, centers_old):
    def top(m):
        from . import _native as N
        from . import device as D

        dev = rows.X.device
        c64 = torch.from_numpy(np.ascontiguousarray(centers_old)).to(dev)
        top_i = torch.empty(m, dtype=torch.int64, device=dev)
        top_v = torch.empty(m, dtype=torch.float64, device=dev)
        ws = D.WS.get("far", N.query("mw_farthest_ws_bytes", rows.S))
        N.call("mw_farthest", D.P(rows.X), rows.S, rows.F, D.P(rows.a32), D.P(rows.b32), D.P(c64),
               centers_old.shape[0], D.P(labels), int(m), D.P(top_i), D.P(top_v), D.P(ws),
               D.stream())
        return top_v.cpu().numpy(), top_i.cpu().numpy()
    return top


def kpp_targets(rv, local_pots, rank):
    """Local search targets of this rank: target t belongs to the first rank
    whose inclusive prefix of local potentials (rank order) reaches rv[t]
    (the last rank if rounding leaves it unreached) and is searched there
    for rv[t] - prefix; -1 on every other rank."""
    pre = np.concatenate([[0.0], np.cumsum(local_pots)])
    world = len(local_pots)
    out = np.full(len(rv), -1.0)
    for t, v in enumerate(rv):
        owner = world - 1
        for r in range(world):
            if pre[r + 1] >= v:
                owner = r
                break
        if owner == rank:
            out[t] = max(v - pre[owner], 0.0)
    return out


class DeviceKpp:
    """Local k-means++ state of one shard on the device (mw_kpp_* kernels):
    the ping-pong banks of T candidate-min distance arrays and their
    per-block sums live in the kernel workspace."""

    def __init__(self, rows, T):
        from . import _native as N
        from . import device as D

        self.N, self.D, self.rows, self.T = N, D, rows, T
        self.ws = D.WS.get("kpp", N.query("mw_kpp_ws_bytes", rows.S, T))
        dev = rows.X.device
        self.pots_dev = torch.empty(T, dtype=torch.float64, device=dev)
        self.rv_dev = torch.empty(T, dtype=torch.float64, device=dev)
        self.loc_dev = torch.empty(T, dtype=torch.int64, device=dev)

    @property
    def device(self):
        return self.rows.X.device

    def rows_at(self, idx: torch.Tensor) -> torch.Tensor:
        return self.rows.X.index_select(0, idx)

    def init(self, center_row):
        r, D = self.rows, self.D
        self.N.call("mw_kpp_init", D.P(r.X), r.S, r.F, D.P(r.mu64), D.P(r.inv64), D.P(center_row),
                    self.T, D.P(self.ws), D.stream())

    def pots_t(self, c, n_arr) -> torch.Tensor:
        D = self.D
        self.N.call("mw_kpp_pots", D.P(self.ws), self.rows.S, self.T, c, D.P(self.pots_dev),
                    D.stream())
        return self.pots_dev[:n_arr]

    def search_t(self, c, best, rv_local) -> torch.Tensor:
        """Local rows of this rank's targets (-1 where rv_local < 0), on the device."""
        D = self.D
        D.h2d_into(self.rv_dev, np.asarray(rv_local, dtype=np.float64))
        r = self.rows
        self.N.call("mw_kpp_search", D.P(r.X), r.S, r.F, D.P(self.ws), self.T, c, best,
                    D.P(self.rv_dev), D.P(self.loc_dev), D.stream())
        return self.loc_dev

    def trial(self, c, best, cand_rows):
        r, D = self.rows, self.D
        self.N.call("mw_kpp_trial", D.P(r.X), r.S, r.F, D.P(r.mu64), D.P(r.inv64), c, best,
                    D.P(cand_rows), self.T, D.P(self.ws), D.stream())


LOCAL_COMM = LocalComm()


def make_comm():
    """DistComm on an initialised process group with world > 1, else local."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return DistComm()
    return LOCAL_COMM
