"""Lloyd pass kinds must not change results: fits with every bounded pass
forced to kTile vs forced to kQueue (and the default mix) must agree bit for
bit (labels, centers, n_iter).  python tools/dev/kind_check.py [size]"""
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
ks = list(range(int(os.environ.get("KC_K0", 8)), int(os.environ.get("KC_K1", 16))))
res = {}
VARIANTS = [("full", -1.0), ("tile", -1.0), ("queue", 2.0), ("mix", 0.12), ("mix3", 0.3),
            ("tile2", -1.0), ("queue2", 2.0), ("queue3", 2.0)]
for name, qb in VARIANTS:
    KM.QUEUE_BELOW = qb
    if name == "full":  # every bound test fails: the plain Lloyd E-step each pass (ground truth)
        os.environ["MW_LLOYD_NOBOUND"] = "1"
    else:
        os.environ.pop("MW_LLOYD_NOBOUND", None)
    with contextlib.redirect_stdout(sys.stderr):
        fits = KM.fit_many(rows, ks, random_state=18)
    res[name] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_) for m in fits]
ok = True
for name in [v for v, _ in VARIANTS[1:]]:
    for i, k in enumerate(ks):
        a, b = res["full"][i], res[name][i]
        same = np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
        if not same:
            ok = False
            print(f"k={k} full vs {name}: labels differ {int((a[0] != b[0]).sum())}, n_iter {a[2]} vs {b[2]}, "
                  f"max center diff {np.abs(a[1] - b[1]).max():.3e}")
print("ALL SAME" if ok else "MISMATCH")
