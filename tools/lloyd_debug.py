"""Lloyd engine diagnostics on the bench slide's rows (config 2 by default):
per fit the passes' (changed, recomputed) counts, bounded vs unbounded
(MW_LLOYD_NOBOUND) trajectories, run-to-run determinism, and per-pass device
times.  python tools/lloyd_debug.py [--size 10000] [--k 8,9,20]"""
import argparse
import contextlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pandas as pd  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=10000)
    ap.add_argument("--channels", type=int, default=30)
    ap.add_argument("--k", default="8")
    a = ap.parse_args()
    import milwrm_amd as M
    from milwrm_amd import device as D
    from milwrm_amd import profiling
    os.environ["MW_LLOYD_TRACE"] = "1"
    from milwrm_amd import kmeans as KM
    from milwrm_amd.kmeans import KMeans, LAST_STATS

    torch.cuda.set_device(0)
    raw, mask = D.synth_slide(a.size, a.size, a.channels, seed=20251015, mode="hard")
    im = M.img.from_device(raw, mask)
    with contextlib.redirect_stdout(sys.stderr):
        est, pix = im.calculate_non_zero_mean()
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(a.channels)), sigma=2, fract=0.2)
    rows = lab._device_rows()
    out = {"S": rows.S}
    for k in [int(x) for x in a.k.split(",")]:
        res = {}
        for name, env, first in [("bounded", "0", "0"), ("bounded_again", "0", "1"), ("full", "1", "0")]:
            os.environ["MW_LLOYD_NOBOUND"] = env
            os.environ["MW_LLOYD_FIRST_ATOMIC"] = first
            KM.trace_summary()
            profiling.reset()
            profiling.enable(True)
            km = KMeans(n_clusters=k, random_state=18).fit(rows)
            torch.cuda.synchronize()
            prof = profiling.summary()
            profiling.enable(False)
            res[name] = {"n_iter": km.n_iter_, "inertia": km.inertia_,
                         "history": LAST_STATS["history"][0],
                         "ms": {n: round(v["total_ms"], 3) for n, v in prof.items() if "lloyd" in n},
                         "trace": KM.trace_summary(),
                         "labels": km.labels_.copy(), "centers": km.cluster_centers_.copy()}
        b, b2, f = res["bounded"], res["bounded_again"], res["full"]
        out[k] = {n: {kk: vv for kk, vv in r.items() if kk not in ("labels", "centers")}
                  for n, r in res.items()}
        out[k]["deterministic"] = bool(np.array_equal(b["labels"], b2["labels"]) and
                                       np.array_equal(b["centers"], b2["centers"]))
        out[k]["bounded_equals_full"] = bool(np.array_equal(b["labels"], f["labels"]) and
                                             np.array_equal(b["centers"], f["centers"]))
        out[k]["label_diff"] = int((b["labels"] != f["labels"]).sum())
    os.environ.pop("MW_LLOYD_NOBOUND", None)
    print(json.dumps(out, default=str), flush=True)


if __name__ == "__main__":
    main()
