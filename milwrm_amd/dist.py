"""Pixel-sharded multi-GPU execution (one process per GPU, RCCL over xGMI via
``torch.distributed`` backend "nccl").

Sharding: each rank owns whole slides (image_df rows); the clustering rows
of a rank are its slides' subsamples, and the global row order is rank order
(= image_df order when slides are dealt to ranks in order).  Every exchange
is a small fixed-size message:

  * batch means            all-gather of (C+1) fp64 per batch, once
  * scaler statistics      all-gather of (1+2F) fp64, Chan-merged in rank order
  * k-means++ per step     all-gather of T local potentials; all-reduce of the
                           T candidate rows (owner contributes, others zero)
  * Lloyd per iteration    ONE all-reduce of k*F + k + 2 fp64 (sums, counts,
                           changed labels, inertia)
  * empty-cluster relocation (rare) all-gather of local top-n (dist, index)

With world_size 1 every method is the identity (``LocalComm``), so the
single-GPU path runs the same code.  Tested with ``gloo`` on CPU tensors for
the host-side logic (tests/test_dist_gloo.py).
"""
from __future__ import annotations

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


class DistComm(LocalComm):
    """Collectives on the default process group.  ``device`` is where the
    message tensors live (cuda for RCCL, cpu for gloo tests)."""

    def __init__(self, device=None, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) \
                if dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.device = device

    def sharded(self) -> bool:
        return self.world > 1

    # -- primitives ------------------------------------------------------
    def all_gather_np(self, a: np.ndarray) -> np.ndarray:
        """[world, *a.shape] in rank order."""
        t = torch.as_tensor(np.ascontiguousarray(a), device=self.device).contiguous()
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

    def merge_stats(self, stats: np.ndarray, F: int) -> np.ndarray:
        """Chan-merge per-rank [n, mean[F], M2[F]] in rank order."""
        g = self.all_gather_np(np.asarray(stats, dtype=np.float64))
        n, m, q = 0.0, np.zeros(F), np.zeros(F)
        for r in range(self.world):
            n, m, q = _chan(n, m, q, g[r, 0], g[r, 1:1 + F], g[r, 1 + F:])
        return np.concatenate([[n], m, q])

    # -- k-means++ over row shards -------------------------------------
    def kpp(self, rows, k, random_state, n_local_trials=None):
        from . import _native as N
        from . import device as D
        from .rng import first_center_index, kpp_draws

        S, F = rows.S, rows.F
        sizes = self.all_gather_np(np.array([S], dtype=np.int64))[:, 0]
        offs = np.concatenate([[0], np.cumsum(sizes)])
        S_tot = int(offs[-1])
        off = int(offs[self.rank])
        T = 2 + int(np.log(k)) if n_local_trials is None else int(n_local_trials)
        u0, steps = kpp_draws(random_state, k, T)
        dev = rows.X.device
        ws = D.WS.get("kpp", N.query("mw_kpp_ws_bytes", S, T))
        st = D.stream()

        def rows_of(gidx):
            """Raw fp32 rows for global indices (owner contributes, all-reduce)."""
            buf = torch.zeros((len(gidx), F), dtype=torch.float32, device=dev)
            for i, g in enumerate(gidx):
                if g >= 0 and off <= g < off + S:
                    buf[i] = rows.X[g - off]
            self.all_reduce_(buf)
            return buf

        first = first_center_index(S_tot, u0)
        chosen = [first]
        chosen_rows = [rows_of([first])[0].clone()]
        N.call("mw_kpp_init", D.P(rows.X), S, F, D.P(rows.mu64), D.P(rows.inv64),
               D.P(chosen_rows[0]), T, D.P(ws), st)
        pots_dev = torch.empty(T, dtype=torch.float64, device=dev)
        rv_dev = torch.empty(T, dtype=torch.float64, device=dev)
        loc_dev = torch.empty(T, dtype=torch.int64, device=dev)
        cand_g = None
        cand_rows = None
        for c in range(1, k + 1):
            n_arr = 1 if c == 1 else T
            N.call("mw_kpp_pots", D.P(ws), S, T, c, D.P(pots_dev), st)
            local = pots_dev[:n_arr].cpu().numpy()
            g = self.all_gather_np(local)  # [world, n_arr]
            tot = np.zeros(n_arr)
            for r in range(self.world):
                tot = tot + g[r]
            best = int(np.argmin(tot)) if c >= 2 else 0
            if c >= 2:
                chosen.append(int(cand_g[best]))
                chosen_rows.append(cand_rows[best].clone())
            if c == k:
                break
            pot = tot[best]
            rv = np.asarray(steps[c - 1], dtype=np.float64) * pot
            pre = np.concatenate([[0.0], np.cumsum(g[:, best])])
            rv_local = np.full(T, -1.0)
            for t in range(T):
                owner = self.world - 1
                for r in range(self.world):
                    if pre[r + 1] >= rv[t]:
                        owner = r
                        break
                if owner == self.rank:
                    rv_local[t] = max(rv[t] - pre[owner], 0.0)
            rv_dev.copy_(torch.from_numpy(rv_local))
            N.call("mw_kpp_search", D.P(ws), S, T, c, best, D.P(rv_dev), D.P(loc_dev), st)
            loc = loc_dev.cpu().numpy()
            gl = np.where(loc >= 0, loc + off, 0).astype(np.int64)
            gsum = torch.from_numpy(gl).to(dev)
            self.all_reduce_(gsum)
            cand_g = gsum.cpu().numpy()
            buf = torch.zeros((T, F), dtype=torch.float32, device=dev)
            for t in range(T):
                if loc[t] >= 0:
                    buf[t] = rows.X[int(loc[t])]
            self.all_reduce_(buf)
            cand_rows = buf
            N.call("mw_kpp_trial", D.P(rows.X), S, F, D.P(rows.mu64), D.P(rows.inv64), c, best,
                   D.P(buf), T, D.P(ws), st)
        X0 = torch.stack(chosen_rows).double().cpu().numpy()
        return (X0 - rows.mu) * rows.inv, np.asarray(chosen, dtype=np.int64)

    # -- empty-cluster relocation --------------------------------------
    def farthest(self, rows, labels, centers_old, n):
        from . import _native as N
        from . import device as D

        S, F = rows.S, rows.F
        k = centers_old.shape[0]
        dev = rows.X.device
        sizes = self.all_gather_np(np.array([S], dtype=np.int64))[:, 0]
        off = int(np.concatenate([[0], np.cumsum(sizes)])[self.rank])
        c64 = torch.from_numpy(np.ascontiguousarray(centers_old)).to(dev)
        m = min(n, S)
        top_i = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
        top_v = torch.empty(max(m, 1), dtype=torch.float64, device=dev)
        if m > 0:
            ws = D.WS.get("far", N.query("mw_farthest_ws_bytes", S))
            N.call("mw_farthest", D.P(rows.X), S, F, D.P(rows.a32), D.P(rows.b32), D.P(c64), k,
                   D.P(labels), int(m), D.P(top_i), D.P(top_v), D.P(ws), D.stream())
        vi = np.full((n, 2), -1.0)
        if m > 0:
            vi[:m, 0] = top_v[:m].cpu().numpy()
            vi[:m, 1] = top_i[:m].cpu().numpy() + off
        g = self.all_gather_np(vi).reshape(-1, 2)
        g = g[g[:, 1] >= 0]
        order = np.lexsort((g[:, 1], -g[:, 0]))[:n]
        sel = g[order]
        far_idx = sel[:, 1].astype(np.int64)
        far_val = sel[:, 0]
        buf = torch.zeros((n, F + 1), dtype=torch.float64, device=dev)
        for i, gi in enumerate(far_idx):
            if off <= gi < off + S:
                li = int(gi - off)
                buf[i, :F] = rows.X[li].double()
                buf[i, F] = float(labels[li].item())
        self.all_reduce_(buf)
        b = buf.cpu().numpy()
        xs = (b[:, :F] - rows.mu) * rows.inv
        return far_idx, far_val, xs, b[:, F].astype(np.int64)


LOCAL_COMM = LocalComm()


def make_comm():
    """DistComm on an initialised process group with world > 1, else local."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return DistComm()
    return LOCAL_COMM
