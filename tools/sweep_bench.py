"""find_optimal_k (k = 2..20, MILWRM.py:659-704) on one synthetic slide:
batched Lloyd (all k per pass, mw_lloyd_pass) against one fit after
another (MW_SWEEP_BATCH=0).  Rows prepared once (untimed); each sweep timed
with a device synchronisation on both sides.  Prints one JSON line.

  python tools/sweep_bench.py [--size 10000] [--reps 2]
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
    ap.add_argument("--mode", default="hard")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import milwrm_amd as M
    from milwrm_amd import device as D
    from milwrm_amd import profiling

    torch.cuda.set_device(0)
    raw, mask = D.synth_slide(a.size, a.size, a.channels, seed=20251015, mode=a.mode)
    im = M.img.from_device(raw, mask)
    with contextlib.redirect_stdout(sys.stderr):
        est, pix = im.calculate_non_zero_mean()
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(a.channels)), sigma=2, fract=0.2)
    out = {"workload": f"find_optimal_k k=2..20 on {lab._rows.S} x {a.channels} rows "
                       f"({a.size}^2 synthetic {a.mode} slide, fract 0.2)"}
    for name, env in [("batched", "1"), ("sequential", "0")]:
        os.environ["MW_SWEEP_BATCH"] = env
        ts, curve = [], None
        for r in range(a.reps + 1):
            profiling.reset()
            profiling.enable(r == a.reps)
            torch.cuda.synchronize()
            t = time.perf_counter()
            with contextlib.redirect_stdout(sys.stderr):
                lab.find_optimal_k(random_state=18, alpha=0.05)
            torch.cuda.synchronize()
            if r > 0:  # first run warms up
                ts.append(time.perf_counter() - t)
            curve = lab.inertia_curve_["Scaled Inertia"].values
        prof = profiling.summary()
        profiling.enable(False)
        out[name] = {"s": min(ts), "best_k": int(lab.k),
                     "kernels_ms": {k: round(v["total_ms"], 2) for k, v in sorted(prof.items())}}
        out[name + "_curve"] = [float(x) for x in curve]
        if name == "batched":
            from milwrm_amd.kmeans import LAST_STATS
            out["rows_recomputed_per_k"] = LAST_STATS.get("recomputed")
    out["identical_curve"] = bool(np.array_equal(out["batched_curve"], out["sequential_curve"]))
    out["speedup"] = out["sequential"]["s"] / out["batched"]["s"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
