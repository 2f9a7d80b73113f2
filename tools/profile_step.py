"""Host-side profile of bench steps (cProfile, cumulative) + wall time per
step.  Usage: python tools/profile_step.py [--size N]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from milwrm_amd import device as D  # noqa: E402
from milwrm_amd.dist import make_comm  # noqa: E402

size = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 10000
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, 30, seed=20251015, mode="hard")
step = bench.make_step(raw, mask, 8, make_comm())
for _ in range(2):
    step()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    step()
torch.cuda.synchronize()
print(f"wall per step: {(time.perf_counter() - t) / 3 * 1e3:.1f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(25)
