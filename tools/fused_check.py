"""Fused blur epilogues vs the materialising path, bit for bit, plus device
times at the bench size:  blur + gather  vs  sample map + blur_sample + fixup,
and  blur + assign  vs  blur_assign  (+ domain records).

  python tools/fused_check.py [--size N] [--k K] [--reps R]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402
from milwrm_amd.assign import assign_image, blur_assign_image  # noqa: E402


def ev_time(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def stage(msg):
    torch.cuda.synchronize()
    print(f"  .. {msg}", flush=True)


def same(a, b):
    a = a.contiguous().view(torch.uint8)
    b = b.contiguous().view(torch.uint8)
    return bool(torch.equal(a, b))


def run(H, W, C, k, reps, feats=None, sigma=2.0, seed=7):
    torch.cuda.set_device(0)
    raw, mask = D.synth_slide(H, W, C, seed=seed, mode="hard")
    s, c = D.nz_stats(raw)
    inv = (c.double() / s).float()
    blurred = D.blur(raw, sigma, inv_mean=inv)
    r2p, M = D.mask_rank(mask.reshape(-1))
    S = int(0.2 * M)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    idx = torch.randint(0, M, (S,), device="cuda", generator=g, dtype=torch.int32)
    feats = list(range(C)) if feats is None else feats
    F = len(feats)
    feat = torch.tensor(feats, dtype=torch.int32, device="cuda")
    X0 = torch.empty((S, F), dtype=torch.float32, device="cuda")
    st0 = torch.zeros(2 * F + 1, dtype=torch.float64, device="cuda")
    D.gather_rows(blurred, feat, idx, r2p, X0, st0, False)
    stage("blur + gather")
    X1 = torch.full((S, F), float("nan"), dtype=torch.float32, device="cuda")
    ok = D.blur_gather_fused(raw, sigma, inv, 1.0, feat, idx, r2p, X1)
    stage(f"fused sample ({ok})")
    st1 = torch.zeros(2 * F + 1, dtype=torch.float64, device="cuda")
    res = {"shape": (H, W, C, F, k), "S": S, "fused_sample": ok}
    if ok:
        D.col_stats_rows(X1, st1, False)
        stage("col stats")
        res["X_equal"] = same(X0, X1)
        res["stats_equal"] = same(st0, st1)
        if not res["X_equal"]:
            bad = (X0 != X1).any(1).nonzero()
            res["X_bad_rows"] = int(bad.numel())
            j = int(bad[0])
            res["X_first_bad"] = (j, X0[j, :4].tolist(), X1[j, :4].tolist())
    mu = (st0[1:1 + F]).cpu().numpy()
    var = (st0[1 + F:]).cpu().numpy() / st0[0].item()
    invs = 1.0 / np.sqrt(var)
    cent_rows = X0[torch.arange(0, S, max(1, S // k), device="cuda")[:k]].double().cpu().numpy()
    centers = (cent_rows - mu) * invs
    if feats == list(range(C)):
        l0, c0, d0 = assign_image(blurred, feats, mu, invs, centers, mask)
        stage("assign")
        out = blur_assign_image(raw, sigma, inv, 1.0, mu, invs, centers, mask)
        stage("fused assign")
        res["fused_assign"] = out is not None
        if out is not None:
            l1, c1, d1 = out
            res["lab_equal"] = same(l0, l1)
            res["conf_equal"] = same(c0, c1)
            res["dom_equal"] = same(d0, d1)
            if not res["lab_equal"]:
                res["lab_diff"] = int((l0 != l1).sum())
            if not res["conf_equal"]:
                dd = (c0 - c1).abs()
                res["conf_maxdiff"] = float(dd[~torch.isnan(dd)].max()) if (~torch.isnan(dd)).any() else 0.0
    if reps:
        Xt = torch.empty_like(X1)
        res["t_blur"] = ev_time(lambda: D.blur(raw, sigma, inv_mean=inv, out=blurred), reps)
        res["t_gather"] = ev_time(lambda: D.gather_rows(blurred, feat, idx, r2p, X0, st0, False), reps)
        res["t_fused_sample"] = ev_time(lambda: D.blur_gather_fused(raw, sigma, inv, 1.0, feat, idx, r2p, Xt), reps)
        res["t_col_stats"] = ev_time(lambda: D.col_stats_rows(Xt, st1, False), reps)
        if feats == list(range(C)):
            res["t_assign"] = ev_time(lambda: assign_image(blurred, feats, mu, invs, centers, mask), reps)
            res["t_fused_assign"] = ev_time(
                lambda: blur_assign_image(raw, sigma, inv, 1.0, mu, invs, centers, mask), reps)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=10000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--small", action="store_true", help="also odd small shapes")
    a = ap.parse_args()
    if a.small:
        for (H, W, C, k, feats) in [(300, 260, 30, 8, None), (257, 333, 30, 5, None), (130, 64, 30, 16, None),
                                    (190, 210, 30, 8, [3, 1, 4, 15, 9, 2, 6]), (200, 200, 16, 8, None),
                                    (160, 96, 64, 12, None), (77, 101, 30, 3, [0, 1, 2, 3, 4])]:
            print(run(H, W, C, k, 0, feats), flush=True)
    print(run(a.size, a.size, 30, a.k, a.reps), flush=True)


if __name__ == "__main__":
    main()
