import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, pandas as pd, torch
import milwrm_amd as M
from milwrm_amd.kmeans import KMeans, fit_many, LAST_STATS
g = dict(np.load("tests/golden/mxif_hard256.npz"))
im = M.img(g["raw"].copy(), mask=g["mask"].copy())
est, pix = im.calculate_non_zero_mean()
df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est], "pixels": [pix]})
lab = M.mxif_labeler(df)
lab.prep_cluster_data(features=list(range(g["raw"].shape[2])), sigma=2, fract=0.2)
rows = lab._device_rows()
for env in ["0", "1"]:
    os.environ["MW_LLOYD_NOBOUND"] = env
    ref = None
    for rep in range(4):
        junk = [torch.randn(rows.S * 19, device="cuda") for _ in range(3)]  # scribble the allocator pool
        del junk
        many = fit_many(rows, list(range(2, 21)), random_state=18); hm = LAST_STATS["history"]
        sig = [m.n_iter_ for m in many]
        if ref is None:
            ref = (sig, hm)
        else:
            bad = [k for k in range(19) if hm[k] != ref[1][k]]
            print("nobound", env, "rep", rep, "n_iter", sig == ref[0], "differing fits", bad, flush=True)
            for kk in bad[:2]:
                for i, (x, z) in enumerate(zip(ref[1][kk], hm[kk])):
                    if x != z: print("   k", kk + 2, "iter", i, x, z); break
