"""Per-launch HIP-event timing on the stream the kernels run on (torch's
current stream).  Disabled by default; bench.py enables it to measure the
dominant kernel's average launch duration live."""
from __future__ import annotations

from collections import defaultdict
from contextlib import contextmanager

import torch

_enabled = False
_events = defaultdict(list)
_bytes = defaultdict(float)
_measured = defaultdict(lambda: [0, 0.0])  # name -> [launches, ms] timed by native code


def enable(on: bool = True):
    global _enabled
    _enabled = on


def reset():
    _events.clear()
    _bytes.clear()
    _measured.clear()


def enabled() -> bool:
    return _enabled


def add_measured(name: str, count: int, total_ms: float, nbytes: float = 0.0):
    """Launches a native driver timed itself (HIP events on its stream)."""
    if not _enabled or count <= 0:
        return
    m = _measured[name]
    m[0] += int(count)
    m[1] += float(total_ms)
    _bytes[name] += nbytes


@contextmanager
def timed(name: str, nbytes: float = 0.0):
    if not _enabled:
        yield
        return
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    yield
    e.record()
    _events[name].append((s, e))
    _bytes[name] += nbytes


def summary():
    """{name: dict(count, total_ms, mean_ms, bytes)} (synchronises)."""
    torch.cuda.synchronize()
    out = {}
    for name, evs in _events.items():
        ms = [s.elapsed_time(e) for s, e in evs]
        out[name] = dict(count=len(ms), total_ms=sum(ms), mean_ms=sum(ms) / max(len(ms), 1),
                         bytes=_bytes[name])
    for name, (cnt, tot) in _measured.items():
        r = out.setdefault(name, dict(count=0, total_ms=0.0, mean_ms=0.0, bytes=0.0))
        r["count"] += cnt
        r["total_ms"] += tot
        r["mean_ms"] = r["total_ms"] / max(r["count"], 1)
        r["bytes"] = _bytes[name]
    return out
