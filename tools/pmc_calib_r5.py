"""Calibration of the HBM counters of the deferred-blur sample path (VERDICT
r4 item 4): mw_sample_map, the blur's sample epilogue (mw_blur_sample_rows)
and mw_col_stats_rows, each over two draw patterns of known algorithmic bytes
on config 2's shape (10k x 10k x 30 uint16, every pixel in the mask, the
identity rank table, S = 1.7e7 draws):
  seq    idx = 0..S-1          (the first S pixels: streaming slot / row writes)
  rand   idx uniform on [0, n)  (config 2's pattern)
Per launch: time (HIP events on the launch stream) and, under rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE (separate runs), the counters per dispatch in
the order seq, rand (x REPS).  tools/pmc_calib_r5_report.py turns both into
the per-kernel correction table.  usage: python tools/pmc_calib_r5.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from milwrm_amd import device as D  # noqa: E402
from milwrm_amd import stream  # noqa: E402

REPS = 2
H = W = 10000
C = F = 30
S = 17_000_000


def main():
    dev = torch.device("cuda")
    raw, _ = D.synth_slide(H, W, C, seed=20251015, mode="hard")
    n = H * W
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    inv_mean = torch.full((C,), 1e-3, dtype=torch.float32, device=dev)
    feat = torch.arange(F, dtype=torch.int32, device=dev)
    r2p = torch.arange(n, dtype=torch.int32, device=dev)
    pats = {"seq": torch.arange(S, dtype=torch.int32, device=dev),
            "rand": torch.randint(0, n, (S,), dtype=torch.int32, device=dev, generator=g)}
    X = torch.empty((S, F), dtype=torch.float32, device=dev)
    stats = torch.zeros(1 + 2 * F, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    out = {"S": S, "F": F, "n_pix": n, "C": C,
           "algorithmic_bytes": {
               "sample_map": {"read": S * 8, "write": n * 8 + S * 4,
                              "note": "idx + rank table reads; the slot memset (n x 8) + one 4-B slot per draw"},
               "blur_sample": {"read": n * C * 2 + n * 8, "write": S * F * 4,
                               "note": "raw uint16 slide + the slot side data; the sampled rows"},
               "col_stats": {"read": S * F * 4, "write": 0, "note": "the rows"}},
           "ms": {}}
    for _ in range(REPS):
        for name, idx in pats.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            stream.blur_gather(raw, 2.0, inv_mean, 1.0, feat, idx, r2p, X)
            ev[1].record()
            D.col_stats_rows(X, stats, False)
            ev[2].record()
            torch.cuda.synchronize()
            out["ms"].setdefault(name, []).append({"blur_gather": ev[0].elapsed_time(ev[1]),
                                                   "col_stats": ev[1].elapsed_time(ev[2])})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
