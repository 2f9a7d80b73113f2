"""Dense-pass diagnostics for the config-4 sweep: per-launch device times by
kind (MW_LLOYD_TRACE) and the share of (row, fit) pairs rechecked exactly."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
os.environ.setdefault("MW_LLOYD_TRACE", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from milwrm_amd import kmeans as K  # noqa: E402
from milwrm_amd import stream  # noqa: E402,F401

H = W = 20000
C = 30
slides = bench.Slides(H, W, C, [20251015], "device", "hard")
from milwrm_amd.dist import make_comm  # noqa: E402

step = bench.make_step(slides, C, 8, make_comm(), sweep=True)
step()  # prep + one sweep (warm)
K.trace_summary()
torch.cuda.synchronize()
t0 = time.perf_counter()
lab = step()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
tr = K.trace_summary()
agg = {}
for t in tr:
    a = agg.setdefault(t["kind"] + f"_m{t['mode']}", {"n": 0, "ms": 0.0, "fits": 0})
    a["n"] += 1
    a["ms"] += t["ms"]
    a["fits"] += t["n_fits"]
S = lab._rows.S
hist = K.LAST_STATS.get("history", [])
rec = [[h[1] for h in hh] for hh in hist]
print(json.dumps({"wall_s": wall, "S": S, "by_kind": agg,
                  "dense_launch_ms": [t["ms"] for t in tr if t["kind"] == "dense"][:200:10],
                  "dense_fits": [t["n_fits"] for t in tr if t["kind"] == "dense"][:200:10],
                  "recomputed_frac_first3": [[round(x / S, 5) for x in r[:3]] for r in rec],
                  "recomputed_frac_late": [[round(x / S, 5) for x in r[-3:]] for r in rec]}, indent=1))
