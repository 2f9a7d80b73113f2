"""Per-launch trace of the batched k sweep (find_optimal_k k=2..20) on one
synthetic slide: per fit n_iter and (changed, recomputed) per pass, per
launch (kind, fits, ms).  Writes JSON to argv[2] (default stdout)."""
import contextlib
import json
import os
import sys

os.environ["MW_LLOYD_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pandas as pd  # noqa: E402
import torch  # noqa: E402

import milwrm_amd as M  # noqa: E402
from milwrm_amd import device as D  # noqa: E402
from milwrm_amd import kmeans as KM  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, 30, seed=20251015, mode="hard")
im = M.img.from_device(raw, mask)
with contextlib.redirect_stdout(sys.stderr):
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(30)), sigma=2, fract=0.2)
    lab.find_optimal_k(random_state=18, alpha=0.05)  # warm
    KM.trace_summary()
    torch.cuda.synchronize()
    lab.find_optimal_k(random_state=18, alpha=0.05)
tr = KM.trace_summary()
out = {"S": int(lab._rows.S), "history": KM.LAST_STATS.get("history"), "launches": tr}
s = json.dumps(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(s)
else:
    print(s)
