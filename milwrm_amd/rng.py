"""Host-side random-number plumbing that must reproduce NumPy's legacy
``RandomState`` draws exactly (the reference seeds it: MxIF.py:484,
MILWRM.py:52/735 → sklearn ``check_random_state``).

* ``subsample_indices``: ``np.random.seed(16); np.random.choice(M, S)`` →
  the library's bit-exact MT19937 masked-rejection generator (C, host).
* ``kpp_draws``: the uniform doubles sklearn's ``_kmeans_plusplus`` consumes,
  drawn up front (they do not depend on the data), so k-means++ runs on the
  device with no host round trip.
* ``first_center_index``: ``choice(n, p=ones/n)`` without materialising the
  n-element cdf: the sequential fp64 running sum of 1/n advances by a constant
  increment inside each binade (after one step), so it is evaluated run by run.
"""
from __future__ import annotations

import functools
import math

import numpy as np


def subsample_indices(M: int, fract: float, random_state: int = 16, out=None) -> np.ndarray:
    """Indices of ``img.subsample_pixels`` (MxIF.py:484,490) as int32."""
    from . import _native as N

    S = int(M * fract)
    if out is None:
        out = np.empty(S, dtype=np.int32)
    if S == 0:
        return out[:0]
    if M > 2**31:
        raise NotImplementedError("subsample over more than 2^31 masked pixels")
    N.call("mw_legacy_randint_host", int(random_state) & 0xFFFFFFFF, int(M), int(S),
           out.ctypes.data)
    return out


# ---- device generator (MT19937 jump-ahead, csrc/rng.hip) -------------------
# words per segment: 32 regenerations of the 624-word window.  mt_gen runs one
# wave per segment through its regenerations in order, so the segment length
# is its serial chain: ~1,150 segments for the config-2 draw (~23 M words),
# 4-5 waves per CU.  The start states (one 2.5-KB window per segment, built
# once per process by the jump prefix): 5 MB at config 2, 82 MB for a
# 40k^2-pixel slide's draw.
MT_SEGMENT = 624 * 32
MT_LEVELS = 24           # jump tables t^(L 2^j) mod phi, j < 24 (2^24 segments)
_tables = {}


def _jump_tables(device):
    """Host-computed jump polynomials (Berlekamp-Massey + squarings, ~0.1 s,
    once per process) uploaded to ``device``."""
    import torch

    from . import _native as N

    key = str(device)
    if key not in _tables:
        h = np.zeros((MT_LEVELS, 312), dtype=np.uint64)
        N.call("mw_mt_jump_tables", MT_SEGMENT, MT_LEVELS, h.ctypes.data)
        _tables[key] = torch.from_numpy(h.view(np.int64)).to(device)
    return _tables[key]


def subsample_indices_device(M: int, fract: float, random_state: int = 16, device=None):
    """Device twin of ``subsample_indices``: returns (int32 tensor of
    int(M*fract) indices, int64 device tensor with the number of accepted
    draws produced, to be checked >= S after the next synchronisation)."""
    import torch

    from . import _native as N
    from . import device as D

    dev = device if device is not None else D.device()
    S = int(M * fract)
    _release_last_draw()
    out = torch.empty(S, dtype=torch.int32, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    if S == 0:
        return out, total
    if M > 2**31:
        raise NotImplementedError("subsample over more than 2^31 masked pixels")
    seed = int(random_state) & 0xFFFFFFFF
    W = N.query("mw_legacy_randint_segments", int(M), S, MT_SEGMENT)
    states, W_avail = _segment_states(dev, seed, W)
    ws = D.WS.get("mtrng", N.query("mw_legacy_randint_gen_ws_bytes", int(M), S, MT_SEGMENT))
    N.call("mw_legacy_randint_from_states", D.P(states), W_avail, int(M), S, MT_SEGMENT, D.P(out),
           D.P(total), D.P(ws), D.stream())
    # the per-segment accepted counts go to the host behind an event of their
    # own, so set_global_state_after_draws waits for them, not for the kernels
    # queued after the draw (the host replay then overlaps the gather)
    cnt = ws[int(W) * MT_SEGMENT * 4:int(W) * MT_SEGMENT * 4 + int(W) * 8].view(torch.int64)
    slot = D._PINNED.take(int(W) * 8)  # pooled page-locked buffer, held until the replay
    slot[1] = D._Busy
    cnt_host = slot[0][:int(W) * 8].view(torch.int64)
    cnt_host.copy_(cnt, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    _LAST_DRAW.update(M=int(M), S=S, seed=seed, W=int(W), cnt_host=cnt_host, ev=ev, slot=slot,
                      states_key=(str(dev), seed))
    return out, total


_LAST_DRAW = {}  # the newest device draw: what the global NumPy state must be advanced past


def _release_last_draw():
    slot = _LAST_DRAW.get("slot")
    if slot is not None:
        _LAST_DRAW["ev"].synchronize()  # the copy into the slot has landed
        slot[1] = None
    _LAST_DRAW.clear()


def set_global_state_after_draws() -> None:
    """Leave NumPy's global RandomState where the reference leaves it after
    ``np.random.seed(16); np.random.choice(M, S)`` (MxIF.py:484,490): advanced
    past every 32-bit word the masked rejection consumed (one word per
    attempt, accepted or not).  From the device generator's per-segment
    accepted counts (exclusive offsets after its scan) the segment holding the
    S-th accepted draw is known; its start state is the MT19937 recurrence
    window after w*L words, i.e. NumPy's key with pos = 624; the host replays
    at most one segment (L = 19,968 words) to find the word that
    accepted draw S came from.  Call after the draw has been synchronised."""
    import torch

    from . import device as D

    last = dict(_LAST_DRAW)
    if not last or last["S"] == 0 or last["M"] < 2:
        _release_last_draw()
        return
    L, S = MT_SEGMENT, last["S"]
    last["ev"].synchronize()
    off = last["cnt_host"].numpy().copy()
    _release_last_draw()
    w = int(np.searchsorted(off, S - 1, side="right")) - 1
    need = S - int(off[w])  # accepted draws still needed inside segment w
    key = _segment_states_host(last["states_key"])[w * 624:(w + 1) * 624].view(np.uint32)
    r = np.uint64(last["M"] - 1)
    m = r
    for s in (1, 2, 4, 8, 16):
        m |= m >> np.uint64(s)
    rs = np.random.RandomState()
    rs.set_state(("MT19937", key.copy(), 624))
    words = rs.randint(0, 2**32, size=L, dtype=np.uint64)  # full range: one word per draw
    hit = np.nonzero((words & m) <= r)[0]
    used = int(hit[need - 1]) + 1
    rs.set_state(("MT19937", key.copy(), 624))
    if used:
        rs.randint(0, 2**32, size=used, dtype=np.uint64)
    np.random.set_state(rs.get_state())


_states = {}


def _segment_states(dev, seed: int, W: int):
    """MT19937 start states of the first >= W stream segments for ``seed``
    (a pure function of (seed, MT_SEGMENT)), built on the device by the jump
    prefix and memoised per (device, seed): every image reseeds with the same
    constant (MxIF.py:484), so the jumps run once per process, not per image.
    Grown to the next power of two when a larger draw needs more segments."""
    import torch

    from . import _native as N
    from . import device as D

    key = (str(dev), seed)
    hit = _states.get(key)
    if hit is not None and hit[1] >= W:
        return hit
    W_new = 1 << max(0, int(W - 1).bit_length())
    if hit is not None:
        W_new = max(W_new, 2 * hit[1])
    states = torch.empty(W_new * 624, dtype=torch.int32, device=dev)
    N.call("mw_mt_segment_states", seed, W_new, D.P(_jump_tables(dev)), MT_LEVELS, D.P(states),
           D.stream())
    _states[key] = (states, W_new)
    return _states[key]


_states_host = {}


def _segment_states_host(key):
    """Host copy of the memoised segment start states (copied once per
    (device, seed, size): they never change once built)."""
    from . import device as D

    states, W = _states[key]
    hit = _states_host.get(key)
    if hit is None or hit[1] != W:
        hit = (D.d2h(states), W)
        _states_host[key] = hit
    return hit[0]


def check_total(total, S: int):
    """``total``: the device count (one sync) or its host value."""
    if S and int(total.item() if hasattr(total, "item") else total) < S:  # pragma: no cover - 16-sigma margin
        raise RuntimeError("device MT19937 produced too few accepted draws; increase the margin")


def as_random_state(random_state):
    """sklearn ``check_random_state`` semantics."""
    if random_state is None or random_state is np.random:
        return np.random.mtrand._rand
    if isinstance(random_state, (int, np.integer)):
        return np.random.RandomState(int(random_state))
    if isinstance(random_state, np.random.RandomState):
        return random_state
    raise ValueError(f"{random_state!r} cannot be used to seed a RandomState instance")


def kpp_draws(random_state, n_clusters: int, n_local_trials: int):
    """(u0, [u_c for c in 1..k-1]) consumed by ``_kmeans_plusplus``
    (_kmeans.py:225 choice → one random_sample; :243 uniform(size=T)).
    An int seed means a fresh ``RandomState(seed)`` whose draws do not depend
    on the data: memoised (constructing the generator alone costs ~0.1 ms)."""
    if isinstance(random_state, (int, np.integer)) and not isinstance(random_state, bool):
        u0, steps = _kpp_draws_seeded(int(random_state), int(n_clusters), int(n_local_trials))
        return u0, [u.copy() for u in steps]
    rs = as_random_state(random_state)
    u0 = float(rs.random_sample())
    steps = [rs.uniform(size=n_local_trials).astype(np.float64) for _ in range(1, n_clusters)]
    return u0, steps


@functools.lru_cache(maxsize=256)
def _kpp_draws_seeded(seed: int, n_clusters: int, n_local_trials: int):
    rs = np.random.RandomState(seed)
    u0 = float(rs.random_sample())
    steps = tuple(rs.uniform(size=n_local_trials).astype(np.float64) for _ in range(1, n_clusters))
    return u0, steps


def _runs(n: int):
    """Yield (i0, s0, inc, m) runs: s_{i0+j} = s0 + j*inc for j in [0, m) where
    s_i = fl(s_{i-1} + c), s_0 = c, c = 1/n (numpy sequential cumsum)."""
    c = 1.0 / float(n)
    i, s = 0, c
    while i < n:
        # one explicit step fixes the parity (round-half-even ties)
        yield i, s, 0.0, 1
        i += 1
        if i >= n:
            return
        t = s + c
        u = t + c
        inc = u - t
        m_exp = math.frexp(t)[1]  # t in [2^(m_exp-1), 2^m_exp)
        top = math.ldexp(1.0, m_exp)
        if inc > 0:
            # largest j with t + j*inc < top, verified exactly below
            j = int((top - t) / inc)
            while j > 0 and t + float(j) * inc >= top:
                j -= 1
            while t + float(j + 1) * inc < top:
                j += 1
            m = min(j + 1, n - i)
        else:
            m = n - i
        # the run t, t+inc, ..., holds while increments stay constant (same binade)
        yield i, t, inc, m
        i += m
        s = (t + float(m - 1) * inc) + c  # s_i = fl(s_{i-1} + c)


def _s_at(run, j):
    i0, s0, inc, m = run
    return s0 + float(j) * inc


@functools.lru_cache(maxsize=256)
def first_center_index(n: int, u: float) -> int:
    """``RandomState.choice(n, p=ones(n)/n)`` given its uniform draw ``u``
    (memoised: a pure function of (n, u))."""
    if n <= 0:
        raise ValueError("n must be positive")
    runs = list(_runs(n))
    last = runs[-1]
    total = _s_at(last, last[3] - 1)
    for run in runs:
        i0, s0, inc, m = run
        if _s_at(run, m - 1) / total > u:
            lo, hi = 0, m - 1  # first j with s_j/total > u
            while lo < hi:
                mid = (lo + hi) // 2
                if _s_at(run, mid) / total > u:
                    hi = mid
                else:
                    lo = mid + 1
            return i0 + lo
    return n  # u >= 1 is impossible for random_sample; numpy would return n
