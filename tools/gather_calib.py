"""Calibration of the gather's HBM counters: the same
kernel (mw_gather_rows, identity rank table so X[j] = img[idx[j]]) over three
draw patterns of known algorithmic bytes on a 10k x 10k x 30 fp32 image,
S = 1.7e7 draws (config 2's sample):
  seq    idx = 0..S-1             (a streaming read of 2.04 GB of rows)
  rand   idx uniform on [0, H*W)  (config 2's pattern: random 120-B rows)
  sorted rand, sorted ascending   (the "sort the draws by pixel" idea)
Prints per-launch time (HIP events on the launch stream) and, under
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, the dispatch order is seq, rand,
sorted (x REPS).  usage: python tools/gather_calib.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milwrm_amd import device as D  # noqa: E402

REPS = 3
H = W = 10000
C = F = 30
S = 17_000_000


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    img = torch.rand((H, W, C), device=dev, generator=g)
    feat = torch.arange(F, dtype=torch.int32, device=dev)
    r2p = torch.arange(H * W, dtype=torch.int32, device=dev)
    pats = {"seq": torch.arange(S, dtype=torch.int32, device=dev),
            "rand": torch.randint(0, H * W, (S,), dtype=torch.int32, device=dev, generator=g)}
    pats["sorted"] = torch.sort(pats["rand"])[0]
    X = torch.empty((S, F), dtype=torch.float32, device=dev)
    stats = torch.zeros(1 + 2 * F, dtype=torch.float64, device=dev)
    out = {"S": S, "F": F, "algorithmic_bytes": {"read_rows": S * F * 4, "read_idx_r2p": S * 8,
                                                  "write_rows": S * F * 4}, "ms": {}}
    for _ in range(REPS):
        for name, idx in pats.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()  # the current stream: the one mw_gather_rows is launched on
            D.gather_rows(img, feat, idx, r2p, X, stats, False)
            e1.record()
            torch.cuda.synchronize()
            out["ms"].setdefault(name, []).append(e0.elapsed_time(e1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
