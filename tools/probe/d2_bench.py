"""Per-launch time of one dense Lloyd pass (lloyd_dense2.h) over synthetic
rows for a fixed set of fits: the A/B harness for kernel variants built with
MW_EXTRA_FLAGS into MW_LIB (tools/probe/d2_variants.sh)."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402
from milwrm_amd import kmeans as KM  # noqa: E402

S = int(os.environ.get("D2_S", 17_000_000))
F = 30
ks = [int(k) for k in os.environ.get("D2_KS", "9,10,11,12,13,14,15,16,17,18,19,20").split(",")]
rng = np.random.default_rng(5)
cent = rng.normal(0, 3, size=(16, F)).astype(np.float32)
X = torch.from_numpy(cent[rng.integers(0, 16, size=S)] + rng.normal(0, 1, size=(S, F)).astype(np.float32)).cuda()
rows = KM.DeviceRows(X)
rows.fixed_point()
dev = X.device
fits = [KM._FitState(rows, rows.scaled_rows(rng.choice(S, size=k, replace=False)), dev) for k in ks]
rls = [int(__import__("milwrm_amd._native", fromlist=["query"]).query("mw_lloyd_rec_len", k, F)) for k in ks]
roff = np.concatenate([[0], np.cumsum(rls)]).astype(np.int64)
out_all = torch.zeros(int(roff[-1]), dtype=torch.float64, device=dev)
outs = [out_all[roff[g]:roff[g + 1]] for g in range(len(ks))]
plen = [k * F + 2 * k for k in ks]
poff = np.concatenate([[0], np.cumsum(plen)]).astype(np.int64)
host = np.zeros(int(poff[-1]), dtype=np.float32)
for g, fs in enumerate(fits):
    o = int(poff[g])
    host[o:o + fs.k * F] = fs.centers.astype(np.float32).ravel()
par = D.h2d(host, dev)
st = D.stream()
sel = [(g, fits[g]) for g in range(len(ks))]
KM._launch_pass(rows, sel, 0, KM.KIND_FIRST, par, poff, outs, st)  # labels
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ms = []
for it in range(12):
    ev[0].record()
    KM._launch_pass(rows, sel, 0, KM.KIND_DENSE, par, poff, outs, st)
    ev[1].record()
    torch.cuda.synchronize()
    if it >= 2:
        ms.append(ev[0].elapsed_time(ev[1]))
print(json.dumps({"lib": os.environ.get("MW_LIB", "default"), "flags": os.environ.get("MW_EXTRA_FLAGS", ""),
                  "S": S, "ks": ks, "ms_mean": float(np.mean(ms)), "ms_min": float(np.min(ms))}))
