"""Time mw_domain_sse (the QC estimators' pass) on one synthetic slide in HBM.

    python tools/qc_bench.py [--size 4096] [--channels 30] [--k 8] [--reps 10]

Prints one JSON line: ms per launch and algorithmic GB/s = n_pix*(C*4 + 1)
bytes (fp32 slide + int8 labels) per launch, against the 8 TB/s HBM peak."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milwrm_amd import _native as N  # noqa: E402
from milwrm_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--channels", type=int, default=30)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    H = W = a.size
    C, k, F = a.channels, a.k, a.channels
    n = H * W
    g = torch.Generator(device=dev).manual_seed(0)
    img = torch.rand((H, W, C), device=dev, generator=g) * 3
    lab = torch.randint(-1, k, (n,), device=dev, generator=g).to(torch.int8)
    feat = torch.arange(F, dtype=torch.int32, device=dev)
    av = torch.ones(F, dtype=torch.float64, device=dev)
    bv = torch.zeros(F, dtype=torch.float64, device=dev)
    cen = torch.randn((k, F), dtype=torch.float64, device=dev, generator=g)
    M = k * F + 2 * F + k
    out = torch.empty(M, dtype=torch.float64, device=dev)
    ws = torch.empty(N.query("mw_domain_sse_ws_bytes", n, k, F), dtype=torch.uint8, device=dev)
    st = D.stream()

    def run():
        N.call("mw_domain_sse", D.P(img), C, D.P(feat), F, D.P(av), D.P(bv), D.P(cen), k, D.P(lab), n,
               D.P(out), D.P(ws), st)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    byts = n * (C * 4 + 1)
    cnt = out[k * F + 2 * F:].sum().item()
    print(json.dumps({"kernel": "mw_domain_sse", "H": H, "W": W, "C": C, "k": k, "ms": ms,
                      "GB_s": byts / ms / 1e6, "frac_hbm": byts / ms / 1e6 / 8000.0,
                      "labelled_pixels": cnt, "expected_labelled": int((lab >= 0).sum().item())}))


if __name__ == "__main__":
    main()
