"""QC sums (estimate_percentage_variance_mxif / estimate_mse_mxif, MILWRM.py:
280-333, 453-515) as extra outputs of the label pass, against the
estimators' own passes, on one synthetic slide (device-generated):

  label            the label pass alone (_assign_img)
  label+qc         the label pass taking the QC sums (label_tissue_regions(qc=True))
  estimators       the QC pass afterwards (fixed point from img._blur_bound)
  estimators_colmax  the same without the bound: a first pass for the column
                   maxima (a second re-blur on a deferred slide)

Rows prepped and fit once (untimed); each variant run once untimed, then
the best of --reps runs, each synchronised on both sides.  Prints one JSON
line.

  python tools/qc_label_bench.py [--size 10000] [--channels 30] [--k 8] [--reps 2]
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pandas as pd  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=10000)
    ap.add_argument("--channels", type=int, default=30)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW
    from milwrm_amd import device as D

    torch.cuda.set_device(0)
    raw, mask = D.synth_slide(a.size, a.size, a.channels, seed=20251015, mode="hard")
    im = M.img.from_device(raw, mask)
    feats = list(range(a.channels))
    with contextlib.redirect_stdout(sys.stderr):
        est, pix = im.calculate_non_zero_mean()
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=feats, sigma=2, fract=0.2)
        lab.find_tissue_regions(k=a.k, random_state=18)
    cents = lab.kmeans.cluster_centers_

    def timed(fn):
        """One untimed run (the caching allocator then holds the band buffer and
        outputs: the timed runs measure the passes, not hipMalloc), then the best
        of --reps timed runs."""
        torch.cuda.synchronize()
        torch.cuda.empty_cache()  # the previous variant's blocks (the banded pass sizes its band from free HBM)
        best, out = None, None
        for r in range(a.reps + 1):
            out = None  # the previous run's outputs (a 40k^2 slide's labels: 8 GB)
            torch.cuda.synchronize()
            t = time.perf_counter()
            with contextlib.redirect_stdout(sys.stderr):
                out = fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) * 1e3
            if r > 0:
                best = dt if best is None else min(best, dt)
            print(f"qc_label_bench: {dt:.1f} ms{' (warm-up)' if r == 0 else ''}", file=sys.stderr, flush=True)
        return best, out

    res = {}
    res["label_ms"], _ = timed(lambda: MW._assign_img(im, feats, cents, lab.scaler))
    _ = None
    res["label_qc_ms"], r = timed(lambda: MW._assign_img(im, feats, cents, lab.scaler, qc=True))
    s_pass = r[3]
    tid = r[0]
    res["estimators_ms"], s_est = timed(lambda: MW._domain_stats(im, False, lab.scaler, cents, feats, tid))
    bound = im._xbound
    im._xbound = None
    try:
        res["estimators_colmax_ms"], _ = timed(
            lambda: MW._domain_stats(im, False, lab.scaler, cents, feats, tid))
    finally:
        im._xbound = bound
    same = s_pass is not None and all(np.array_equal(s_pass[q], s_est[q], equal_nan=True)
                                      for q in ("sse", "sum", "sumsq", "count"))
    pv = np.float64(np.sum(s_est["sse"])) / MW.dm_total(s_est) * 100
    print(json.dumps({"workload": f"one synthetic {a.size}^2 x {a.channels} slide, k={a.k}, "
                                  f"{'deferred' if im._pending_blur is not None else 'materialised'} blur",
                      **{k: round(v, 3) for k, v in res.items()},
                      "qc_extra_in_label_pass_ms": round(res["label_qc_ms"] - res["label_ms"], 3),
                      "label_pass_sums_equal_estimators": bool(same),
                      "pct_variance_S2": float(pv)}))


if __name__ == "__main__":
    main()
