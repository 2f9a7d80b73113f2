"""Wall time of each phase of one pipeline step, with a device sync after
each phase (so each number = host + device time of that phase)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402
from milwrm_amd.assign import assign_image  # noqa: E402
from milwrm_amd.kmeans import DeviceRows, StandardScaler, _kmeans_plusplus_device, lloyd_device  # noqa: E402
from milwrm_amd.rng import subsample_indices_device  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, 30, seed=20251015, mode="hard")
torch.cuda.synchronize()


def run(report):
    T = {}
    t = time.perf_counter()

    def mark(name):
        nonlocal t
        torch.cuda.synchronize()
        now = time.perf_counter()
        T[name] = (now - t) * 1e3
        t = now

    s, c = D.nz_stats(raw)
    s = s.cpu().numpy(); c = c.cpu().numpy()
    mark("nz_stats+D2H")
    mean = s / c
    inv = torch.from_numpy((1 / mean).astype(np.float32)).cuda()
    mark("inv H2D")
    blurred = D.blur(raw, 2.0, inv_mean=inv)
    mark("blur")
    r2p, M = D.mask_rank(mask.reshape(-1))
    mark("mask_rank+count")
    idx, tot = subsample_indices_device(M, 0.2, 16)
    mark("device rng")
    S = idx.shape[0]
    X = torch.empty((S, 30), dtype=torch.float32, device="cuda")
    stats = torch.zeros(61, dtype=torch.float64, device="cuda")
    feat = torch.arange(30, dtype=torch.int32, device="cuda")
    mark("alloc")
    D.gather_rows(blurred, feat, idx, r2p, X, stats, False)
    mark("gather")
    st = stats.cpu().numpy()
    sc = StandardScaler.from_stats(st)
    mu, invs = sc.affine()
    rows = DeviceRows(X, mu, invs, feature_var=sc.var_ * invs * invs)
    mark("scaler+rows")
    centers, ids = _kmeans_plusplus_device(rows, 8, np.random.RandomState(18))
    mark("kpp")
    tol = float(np.mean(rows.feature_var()) * 1e-4)
    labels, inertia, cent, n_iter = lloyd_device(rows, centers, 300, tol)
    mark(f"lloyd ({n_iter} it)")
    lab, conf, dom = assign_image(blurred, np.arange(30), mu, invs, cent, mask)
    dom = dom.cpu().numpy()
    mark("assign+D2H")
    if report:
        tot_ms = sum(T.values())
        print(" | ".join(f"{k} {v:.2f}" for k, v in T.items()), f"|| total {tot_ms:.1f} ms", flush=True)


for i in range(4):
    run(i >= 2)
