"""Determinism of the Lloyd queue pass: run the same fits several times with
every bounded pass forced to kQueue and report where the per-pass histories
(changed, recomputed) first diverge.  python tools/dev/queue_race.py [size]"""
import contextlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402

import milwrm_amd as M  # noqa: E402
from milwrm_amd import device as D  # noqa: E402
from milwrm_amd import kmeans as KM  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, 30, seed=20251015, mode="hard")
im = M.img.from_device(raw, mask)
with contextlib.redirect_stdout(sys.stderr):
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(30)), sigma=2, fract=0.2)
rows = lab._rows
ks = [int(x) for x in os.environ.get("QR_KS", "13,15,17,18,19").split(",")]
KM.QUEUE_BELOW = float(os.environ.get("QR_QB", "2.0"))
runs = []
for rep in range(int(os.environ.get("QR_REPS", "4"))):
    with contextlib.redirect_stdout(sys.stderr):
        fits = KM.fit_many(rows, ks, random_state=18)
    runs.append(([np.asarray(m.labels_).copy() for m in fits], [list(h) for h in KM.LAST_STATS["history"]]))
for i, k in enumerate(ks):
    hs = [r[1][i] for r in runs]
    labs = [r[0][i] for r in runs]
    div = None
    for p in range(min(len(h) for h in hs)):
        if len({tuple(h[p]) for h in hs}) > 1:
            div = p
            break
    same = all(np.array_equal(labs[0], x) for x in labs[1:])
    print(f"k={k}: passes {[len(h) for h in hs]} labels same {same} first divergent pass {div}"
          + (f" histories there {[h[div] for h in hs]} before {[h[div - 1] for h in hs] if div else None}" if div is not None else ""))
