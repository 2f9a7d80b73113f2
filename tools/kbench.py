"""Per-kernel microbenchmark at BASELINE config-2 sizes (10k x 10k x 30 uint16
slide, S = 1.7e7 sample rows, k = 8): device time per launch from HIP events
on the launch stream, algorithmic GB/s, and an output fingerprint so kernel
variants can be compared bit for bit across builds.

  python tools/kbench.py [--only blur,lloyd,...] [--reps N]
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import _native as N  # noqa: E402
from milwrm_amd import device as D  # noqa: E402


def fp(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:12]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--size", type=int, default=10000)
    ap.add_argument("--C", type=int, default=30)
    ap.add_argument("--k", type=int, default=8)
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))
    want = lambda n: not only or n in only  # noqa: E731
    torch.cuda.set_device(0)
    H = W = a.size
    C, k = a.C, a.k
    st = D.stream()
    raw, mask = D.synth_slide(H, W, C, seed=20251015, mode="hard")
    s, c = D.nz_stats(raw)
    inv = (c.double() / s).float()
    torch.cuda.synchronize()
    res = {}
    if want("nz"):
        ms = timeit(lambda: D.nz_stats(raw), a.reps)
        res["nz_stats"] = (ms, H * W * C * 2, fp(*D.nz_stats(raw)))
    blurred = D.blur(raw, 2.0, inv_mean=inv)
    if want("blur"):
        ms = timeit(lambda: D.blur(raw, 2.0, inv_mean=inv, out=blurred), a.reps)
        res["blur"] = (ms, H * W * C * 6, fp(blurred))
        os.environ["MW_BLUR_IMPL"] = "valu"
        ref = torch.empty_like(blurred)
        ms2 = timeit(lambda: D.blur(raw, 2.0, inv_mean=inv, out=ref), a.reps)
        del os.environ["MW_BLUR_IMPL"]
        res["blur(valu kernel)"] = (ms2, H * W * C * 6, fp(ref))
        diff = (blurred - ref).abs()
        rel = (diff / ref.abs().clamp_min(1e-30)).max().item()
        print(f"blur mfma vs valu: max abs {diff.max().item():.3e} max rel {rel:.3e}", flush=True)
        del ref, diff
    # sample rows: S = 0.17 N rows of the blurred slide (fixed random pick)
    S = int(0.17 * H * W)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    r2p, M = D.mask_rank(mask)
    idx = torch.randint(0, M, (S,), device="cuda", generator=g, dtype=torch.int64)
    X = torch.empty((S, C), dtype=torch.float32, device="cuda")
    stats = torch.zeros(2 * C + 1, dtype=torch.float64, device="cuda")
    feat = torch.arange(C, dtype=torch.int32, device="cuda")
    if want("gather"):
        idx32 = idx.to(torch.int32)
        ms = timeit(lambda: D.gather_rows(blurred, feat, idx32, r2p, X, stats, False), a.reps)
        res["gather"] = (ms, S * C * 8 + S * 8, fp(X))
    else:
        D.gather_rows(blurred, feat, idx.to(torch.int32), r2p, X, stats, False)
    mu = X.double().mean(0)
    sd = X.double().std(0, unbiased=False)
    inv64 = (1.0 / sd).contiguous()
    mu64 = mu.contiguous()
    a32 = inv64.float().contiguous()
    b32 = (-mu64 * inv64).float().contiguous()
    F = C
    T = 2 + int(np.log(k))
    if want("kpp"):
        ws = D.WS.get("kpp", N.query("mw_kpp_ws_bytes", S, T))
        rs = np.random.RandomState(3)
        us = [rs.random_sample(T) for _ in range(k)]

        def kpp_all():
            N.call("mw_kpp_init", D.P(X), S, F, D.P(mu64), D.P(inv64), D.P(X) + 12345 * F * 4, T,
                   D.P(ws), st)
            for cc in range(1, k):
                u = np.ascontiguousarray(us[cc - 1])
                N.call("mw_kpp_step", D.P(X), S, F, D.P(mu64), D.P(inv64), cc, u.ctypes.data, T,
                       D.P(ws), st)
        ms = timeit(kpp_all, max(1, a.reps // 2))
        idxo = torch.empty(k, dtype=torch.int64, device="cuda")
        N.call("mw_kpp_indices", D.P(ws), S, T, k, D.P(idxo), st)
        res["kpp(init+7 steps)"] = (ms, k * (S * F * 4) + (k - 1) * S * 8 * (1 + T), fp(idxo))
    if want("lloyd"):
        # the real Lloyd sequence (first / tile / queue passes, final mode 1)
        # from evenly spaced rows, per-launch HIP event times (kmeans.TRACE)
        from milwrm_amd import kmeans as K

        rows = K.DeviceRows(X, mu64.cpu().numpy(), inv64.cpu().numpy())
        c0 = rows.scaled_rows(np.arange(0, S, S // k)[:k])
        K.lloyd_device(rows, c0)  # warm (fixed point, workspaces)
        K.TRACE = []
        labels, inertia, cents, n_iter = K.lloyd_device(rows, c0)
        per = {}
        for t in K.trace_summary():
            per.setdefault((t["mode"], t["kind"]), []).append(t["ms"])
        K.TRACE = None
        for (mode, kind), v in sorted(per.items()):
            res[f"lloyd_m{mode}_{kind or 'full'} x{len(v)}"] = (float(np.mean(v)), S * (F * 4 + 9),
                                                                fp(labels))
        print(f"lloyd n_iter {n_iter} inertia {inertia!r}", flush=True)
    cent = X[torch.arange(0, S, S // k, device="cuda")[:k]].double()
    cent = ((cent - mu64) * inv64).float().contiguous()
    if want("assign"):
        lab = torch.empty((H, W), dtype=torch.int8, device="cuda")
        conf = torch.empty((H, W), dtype=torch.float32, device="cuda")
        aws = D.WS.get("assign", N.query("mw_assign_ws_bytes", H * W, k))
        dom = torch.empty(2 * k, dtype=torch.float64, device="cuda")

        def asg():
            N.call("mw_assign_conf", D.P(blurred), C, D.P(feat), F, D.P(a32), D.P(b32), D.P(cent),
                   k, D.P(mask), H * W, D.P(lab), D.P(conf), D.P(aws), st)
        ms = timeit(asg, a.reps)
        N.call("mw_assign_reduce", D.P(aws), H * W, k, D.P(dom), st)
        res["assign_conf"] = (ms, H * W * (C * 4 + 6), fp(lab, conf, dom))
    for n, (ms, b, h) in res.items():
        print(f"{n:22s} {ms:8.3f} ms  {b / ms / 1e6:7.0f} GB/s  fp={h}", flush=True)


if __name__ == "__main__":
    main()
