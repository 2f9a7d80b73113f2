"""Host-side (Python) cost of one bench step: cProfile over a few steps of
bench.py's step at config 2.  Time inside Tensor.cpu / .item is the host
waiting for the device; everything else is host overhead that the device
may idle behind.

  python tools/host_profile.py [--steps 3] [--size 10000]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--size", type=int, default=10000)
    a = ap.parse_args()
    import bench
    from milwrm_amd import device as D
    from milwrm_amd.dist import make_comm

    torch.cuda.set_device(0)
    raw, mask = D.synth_slide(a.size, a.size, 30, seed=20251015, mode="hard")
    step = bench.make_step(raw, mask, 8, make_comm())
    step()
    step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
    ps.print_stats(35)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue())


if __name__ == "__main__":
    main()
