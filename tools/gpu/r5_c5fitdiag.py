"""Config-5 share (4 synth 40k^2 x 50 slides on one GPU): the Lloyd fit's
per-pass history (changed, recomputed rows) and per-launch device times,
through the Python loop (MW_KMEANS_C=0, MW_LLOYD_TRACE=1)."""
import contextlib
import json
import os
import sys
import time

os.environ["MW_KMEANS_C"] = "0"
os.environ["MW_LLOYD_TRACE"] = "1"
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch  # noqa: E402

import bench  # noqa: E402
from milwrm_amd import kmeans as K  # noqa: E402
from milwrm_amd.dist import make_comm  # noqa: E402

n = int(os.environ.get("C5_SLIDES", "4"))
slides = bench.Slides(40000, 40000, 50, [20251015 + i for i in range(n)], "synth", "hard")
import milwrm_amd as M  # noqa: E402
import pandas as pd  # noqa: E402

with contextlib.redirect_stdout(sys.stderr):
    ims = slides.images()
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in ims])
    df = pd.DataFrame({"Img": ims, "batch_names": ["b"] * len(ims), "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(50)), sigma=2, fract=0.2, comm=make_comm())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    km = K.KMeans(n_clusters=8, random_state=18).fit(lab._rows)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
tr = K.trace_summary()
S = lab._rows.S
hist = K.LAST_STATS.get("history", [[]])[0]
print(json.dumps({"S": S, "n_iter": int(km.n_iter_), "wall_s": wall,
                  "history_frac": [[h[0] / S, h[1] / S] for h in hist],
                  "launches": [(t["kind"], t["mode"], t["ms"]) for t in tr]}))
