"""Fingerprint of the config-2 pipeline's fit (k-means++ indices, centers,
n_iter, labels hash) for same-bits A/B checks of kernel variants selected by
environment variables: run once per variant and compare the printed lines."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402

import milwrm_amd as M  # noqa: E402
from milwrm_amd import device as D  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
C, k = 30, 8
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, C, seed=1, mode="hard")
im = M.img.from_device(raw, mask)
est, pix = im.calculate_non_zero_mean()
df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
lab = M.mxif_labeler(df)
lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
lab.label_tissue_regions(k=k, plot_out=False, random_state=18)
km = lab.kmeans
h = hashlib.sha1()
h.update(np.ascontiguousarray(km.cluster_centers_).tobytes())
h.update(lab._labels_dev[0].cpu().numpy().tobytes())
h.update(lab._conf_dev[0].cpu().numpy().tobytes())
idx = getattr(km, "init_indices_", None)
print(f"FP n_iter={km.n_iter_} inertia={km.inertia_!r} init={None if idx is None else list(map(int, idx))} "
      f"sha1={h.hexdigest()}", flush=True)
