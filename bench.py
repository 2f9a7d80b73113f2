"""Benchmark: MILWRM MxIF pixel clustering (preprocess + k-means fit + label)
on synthetic 30-channel slides, BASELINE.json config 2 per GPU.

One step = the whole hot path over one slide per GPU, inputs (uint16 HWC +
uint8 mask) already resident in HBM:
  calculate_non_zero_mean → batch means → fused log-normalise + Gaussian blur
  → mask rank + legacy-RNG subsample gather + column stats → StandardScaler
  → k-means++ (k=8, random_state=18) → Lloyd to convergence → label +
  confidence pass over every pixel.
Multi-GPU: one slide per rank (weak scaling), pixel-sharded fit with RCCL
all-reduce of the per-iteration partials (milwrm_amd.dist).  Launched either
by torchrun (WORLD_SIZE set) or as ``bench.py --gpus N``, which spawns the N
ranks itself (fresh processes, before any GPU call) and fails when fewer than
N GPUs are visible.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "pixels/sec (node) for preprocess+k-means fit+label, 30-ch MxIF k=8; %HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md); measured copy ceiling ~6300


def _config_name(H, W, C, n, world, sweep=False):
    """Which BASELINE.json config this workload is (``n`` slides per GPU)."""
    if sweep:
        if (H, W, C) == (20000, 20000, 30) and n == 1:
            return "BASELINE config 4: the k=2..20 sweep over config 3's slides (one 20k^2 x 30 slide per GPU)"
        return "find_optimal_k sweep k=2..20 (config 4 shape) over custom slides"
    if (H, W, C) == (10000, 10000, 30) and n == 1:
        return "BASELINE config 2 per GPU"
    if (H, W, C) == (20000, 20000, 30) and n == 1:
        return "BASELINE config 3 per GPU: one of its 8 slides"
    if (H, W, C) == (40000, 40000, 50):
        if n * world == 16:
            return f"BASELINE config 5: its 16-slide cohort, {n} slides per GPU"
        return f"BASELINE config 5 per GPU: {n} of its 16 slides per GPU"
    return "custom size"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=10000, help="slide is size x size pixels")
    ap.add_argument("--channels", type=int, default=30)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--no-design-point", action="store_true",
                    help="skip the second line on the design-point slide (--mode design, I~17)")
    ap.add_argument("--mode", default="hard", choices=["hard", "easy", "design"],
                    help="synthetic slide: hard (the headline), design (overlapping domains: "
                         "SURVEY 8d's I~17 Lloyd iterations), easy")
    ap.add_argument("--slides-per-gpu", type=int, default=1,
                    help="slides each rank labels per step (config 5: 2 on 8 GPUs)")
    ap.add_argument("--source", default="auto", choices=["auto", "device", "synth", "host"],
                    help="where the raw slides live: device = resident in HBM before the timed "
                         "region; synth = not resident, generated band by band on the device "
                         "inside the step (the stand-in for a slide reader); host = page-locked "
                         "host memory read band by band over PCIe inside the step; "
                         "auto = device when all fit in 60%% of HBM, else synth")
    ap.add_argument("--sweep", action="store_true",
                    help="time find_optimal_k (k=2..20) over the prepped rows instead of the "
                         "label pipeline (BASELINE config 4)")
    ap.add_argument("--cpu-size", type=int, default=2048, help="oracle CPU-baseline slide side")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-outputs", action="store_true",
                    help="skip the reference-format host outputs after the timed steps (timeline traces)")
    return ap.parse_args()


class Slides:
    """The raw slides of this rank, kept where ``--source`` puts them; ``img``
    objects are made fresh for every step."""

    def __init__(self, H, W, C, seeds, source, mode):
        import milwrm_amd as M
        from milwrm_amd import device as D
        from milwrm_amd import stream

        self.M, self.stream = M, stream
        self.source = source
        self.items = []
        for seed in seeds:
            if source == "device":
                self.items.append(D.synth_slide(H, W, C, seed=seed, mode=mode))
            elif source == "synth":
                self.items.append(stream.SynthSource(H, W, C, seed, mode))
            else:  # host: generated on the device into page-locked host chunks
                src = stream.SynthSource(H, W, C, seed, mode)
                chunks = stream.pinned_rows(src, progress=lambda y: print(
                    f"bench.py: slide {seed} in pinned host memory: {y}/{H} rows", file=sys.stderr,
                    flush=True))
                self.items.append((stream.HostSource(chunks), src.mask_device()))
        torch.cuda.synchronize()

    def images(self):
        M = self.M
        if self.source == "device":
            return [M.img.from_device(raw, mask) for raw, mask in self.items]
        if self.source == "synth":
            return [M.img.from_source(src) for src in self.items]
        return [M.img.from_source(hs, mask=m) for hs, m in self.items]


def make_step(slides, C, k, comm, sweep=False):
    import pandas as pd

    import milwrm_amd as M

    def step():
        with contextlib.redirect_stdout(sys.stderr):  # reference-style progress prints
            return _step()

    def prep():
        ims = slides.images()
        ests, pix = zip(*[im.calculate_non_zero_mean() for im in ims])
        # one batch over every slide of every rank (mxif_labeler sums the
        # estimators per batch over its images and, sharded, over the ranks)
        df = pd.DataFrame({"Img": ims, "batch_names": ["b"] * len(ims),
                           "mean estimators": list(ests), "pixels": list(pix)})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2, comm=comm)
        return lab

    def _step():
        lab = prep()
        lab.label_tissue_regions(k=k, plot_out=False, random_state=18, comm=comm)
        lab.confidence_score_images()
        return lab

    if not sweep:
        return step
    state = {}

    def sweep_step():
        # the rows are prepped once (the first, untimed warmup call); each
        # step is the whole find_optimal_k over them
        if "lab" not in state:
            with contextlib.redirect_stdout(sys.stderr):
                state["lab"] = prep()
        lab = state["lab"]
        with contextlib.redirect_stdout(sys.stderr):
            lab.find_optimal_k(random_state=18, alpha=0.05)
        return lab

    return sweep_step


def cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo) and its logical CPU count."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{name} ({os.cpu_count()} logical CPUs on the host; the baseline uses `cores` of them)"


def cpu_baseline(size, C, k, sweep=False):
    """Oracle (numpy/scipy restatement of the reference pipeline) on a bounded
    host sample; pixels/s on this box's cores.  ``sweep``: the oracle's
    find_optimal_k (19 sklearn-restated fits) over the rows of a smaller
    slide (prep untimed)."""
    from threadpoolctl import threadpool_info

    from oracle import milwrm_oracle as O

    threads = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    if sweep:
        size = min(size, 512)
        raw, mask = O.synth_slide(size, size, C, seed=20251015, mode="hard")
        est, pix = O.non_zero_mean(raw)
        mean = np.asarray(est) / pix
        X, _ = O.subsample_pixels(O.gaussian_blur(O.log_normalize(raw, mean)), mask, list(range(C)))
        mu, sc, _ = O.scaler_fit(X)
        Xs = O.scaler_transform(X, mu, sc)
        t = time.perf_counter()
        best = O.choose_best_k(Xs)
        dt = time.perf_counter() - t
        return dict(value=size * size / dt, unit="pixels/s", cores=int(threads), kind="port",
                    cpu_model=cpu_model(), sample=f"oracle choose_best_k (k=2..20) over the {Xs.shape[0]} rows of one "
                           f"{size}x{size}x{C} synthetic slide (best_k {best[0]}), {dt:.1f} s, "
                           f"numpy/OpenBLAS threads={threads}")
    raw, mask = O.synth_slide(size, size, C, seed=20251015, mode="hard")
    t = time.perf_counter()
    r = O.mxif_pipeline([raw], [mask], ["b"], list(range(C)), k=k)
    dt = time.perf_counter() - t
    return dict(value=size * size / dt, unit="pixels/s", cores=int(threads), kind="port",
                cpu_model=cpu_model(), sample=f"oracle mxif_pipeline on one {size}x{size}x{C} synthetic slide, k={k} "
                       f"(n_iter {r['kmeans']['n_iter_']}), {dt:.1f} s, numpy/OpenBLAS threads="
                       f"{threads}")


def pmc_traffic(kernel, suffix=""):
    """HBM bytes per launch of ``kernel`` from the newest committed rocprofv3
    FETCH_SIZE / WRITE_SIZE summary for this workload (profiles/*/pmc_traffic
    {suffix}_v*.json: "" config 2, "_c5" the config-5 slice; written by
    tools/pmc_traffic.py from tools/gpu/pmc_bench.sh's separate counter passes
    over this same bench command; corrections in that file), plus the kernel's
    SQ summary (issue / wait fractions, VALU and MFMA busy) when recorded.
    Returns (bytes or None, source or None, counters or None)."""
    import glob
    import re

    def ver(f):
        m = re.search(r"r(\d+)/pmc_traffic%s_v(\d+)\.json$" % re.escape(suffix), f)
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"pmc_traffic{suffix}_v*.json")), key=ver)
    if not files:
        return None, None, None
    d = json.load(open(files[-1]))
    rec = d.get("kernels", {}).get(kernel)
    sq = d.get("sq", {}).get(kernel)
    src = os.path.relpath(files[-1], ROOT)
    if not rec or not rec.get("calibrated", False):
        return None, (src if sq else None), sq
    return rec["traffic_bytes"], src, sq


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N fresh child processes, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment), each
    running this script; this parent never touches the GPU (it only counts
    the devices, which does not initialise HIP on this image) and exits with
    the first failing child's status.  A child that fails takes the others
    down (they would wait forever in a collective)."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in alive:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def check_devices(world: int) -> None:
    """One GPU per rank on this node: fewer visible devices than ranks is an
    error, never a silent world-1 run."""
    have = torch.cuda.device_count()
    if have < world:
        print(f"bench.py: {world} ranks (--gpus / WORLD_SIZE) need {world} GPUs on this node, "
              f"{have} visible", file=sys.stderr, flush=True)
        sys.exit(2)


def design_point(H, W, C, k, comm, lab_hard, steps=3):
    """The same step on the 'design' slide (overlapping domains: SURVEY 8d's
    I ~ 17 Lloyd iterations instead of the headline slide's ~5), timed the
    same way: a second line beside the headline, where the fit weighs as the
    survey's design point assumes."""
    from milwrm_amd import profiling
    from milwrm_amd import stream

    del lab_hard
    slides = Slides(H, W, C, [20251015], "device", "design")
    step = make_step(slides, C, k, comm)
    step()
    torch.cuda.synchronize()
    profiling.reset()
    profiling.enable(True)
    t0 = time.perf_counter()
    lab = None
    for _ in range(steps):
        lab = None
        lab = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    profiling.enable(False)
    prof = profiling.summary()
    fit = prof.get("kmeans_fit", {})
    return {"mode": "design", "spread": stream.synth_mode("design")[0], "steps": steps,
            "ms_per_step": el / steps * 1e3, "value": H * W * steps / el, "unit": "pixels/s",
            "lloyd_iters": int(lab.kmeans.n_iter_),
            "kmeans_fit_ms": round(fit.get("total_ms", 0.0) / steps, 4)}


FP32_PEAK_TFLOPS = 157.3    # MI355X vector / f32-matrix peak (MI355X_MICROARCH.md)
F16_MFMA_PEAK_TFLOPS = 2500.0  # dense f16/bf16 matrix-core peak (spec, no sparsity)


def dense_pass_roofline(rows, ks=tuple(range(9, 21)), reps=6):
    """The sweep's ALU-bound kernel (the batched k-sweep E-step
    against the ALU roofline): one dense Lloyd pass (lloyd_dense2.h) of the
    fits k = 9..20 together over the sweep's own rows, timed with HIP events
    on its stream.  Useful work = the x . c products every (row, center) pair
    needs, S * sum(k) * F * 2 flops, against the fp32 peak (what a direct
    fp32 E-step would issue); issued work = the f16 hi/lo matrix-core products
    (per 32 rows: ceil(sum of 8-aligned k / 32) tiles x 6 v_mfma_f32_32x32x16_f16
    of 32768 flops), against the f16 MFMA peak."""
    from milwrm_amd import _native as N
    from milwrm_amd import device as D
    from milwrm_amd import kmeans as KM

    S, F = rows.S, rows.F
    if F > 30:
        return None
    rows.fixed_point()
    dev = rows.X.device
    rng = np.random.default_rng(5)
    fits = [KM._FitState(rows, rows.scaled_rows(np.sort(rng.choice(S, size=k, replace=False))), dev)
            for k in ks]
    rls = [N.query("mw_lloyd_rec_len", k, F) for k in ks]
    roff = np.concatenate([[0], np.cumsum(rls)]).astype(np.int64)
    out_all = torch.zeros(int(roff[-1]), dtype=torch.float64, device=dev)
    outs = [out_all[roff[g]:roff[g + 1]] for g in range(len(ks))]
    poff = np.concatenate([[0], np.cumsum([k * F + 2 * k for k in ks])]).astype(np.int64)
    host = np.zeros(int(poff[-1]), dtype=np.float32)
    for g, fs in enumerate(fits):
        host[int(poff[g]):int(poff[g]) + fs.k * F] = fs.centers.astype(np.float32).ravel()
    par = D.h2d(host, dev)
    st = D.stream()
    sel = [(g, fits[g]) for g in range(len(ks))]
    KM._launch_pass(rows, sel, 0, KM.KIND_FIRST, par, poff, outs, st)  # labels to start from
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ms = []
    for it in range(reps + 1):
        ev[0].record()
        KM._launch_pass(rows, sel, 0, KM.KIND_DENSE, par, poff, outs, st)
        ev[1].record()
        torch.cuda.synchronize()
        if it:
            ms.append(ev[0].elapsed_time(ev[1]))
    t = float(np.mean(ms)) * 1e-3
    useful = float(S) * sum(ks) * F * 2
    ntile = -(-sum((k + 7) // 8 * 8 for k in ks) // 32)
    issued = float(-(-S // 32)) * ntile * 6 * 32768
    nbytes = float(S) * F * 4 + 2.0 * S * len(ks)
    del fits, out_all, outs
    return {"kernel": "lloyd_dense2_kernel", "fits": list(ks), "rows": S, "ms": t * 1e3,
            "useful_tflops": useful / t / 1e12, "fp32_peak_tflops": FP32_PEAK_TFLOPS,
            "frac_fp32": useful / t / 1e12 / FP32_PEAK_TFLOPS,
            "mfma_issued_tflops": issued / t / 1e12, "f16_mfma_peak_tflops": F16_MFMA_PEAK_TFLOPS,
            "frac_f16_mfma": issued / t / 1e12 / F16_MFMA_PEAK_TFLOPS,
            "hbm_GBps": nbytes / t / 1e9, "frac_hbm": nbytes / t / 1e9 / HBM_PEAK_GBPS}


def fit_rows_read(S, F, k):
    """Rows whose features the last single fit of this thread read: k
    k-means++ passes over all S rows plus, per Lloyd pass, the rows the pass
    read (mw_kmeans_fit_history); None when the fit did not run in the C
    driver (no history)."""
    import numpy as np

    from milwrm_amd import _native as N

    n = N.load().mw_kmeans_fit_history(None, 0)
    if n <= 0:
        return None
    h = np.zeros((n, 4), dtype=np.int64)
    N.load().mw_kmeans_fit_history(h.ctypes.data, n)
    return int(k * S + h[:, 3].sum())


def host_outputs(lab):
    """Cost of the reference-format outputs of one slide, outside the timed
    step: ``tissue_IDs[0]`` and ``confidence_IDs[0]`` as float64 H x W host
    arrays with NaN outside the mask (MILWRM.py:275-276, 444-445), converted
    on first access from the device's int8 labels and fp32 confidences (one
    page-locked D2H copy each, then a threaded host expansion)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tid = lab.tissue_IDs[0]
    t1 = time.perf_counter()
    cid = lab.confidence_IDs[0]
    t2 = time.perf_counter()
    n = int(tid.size)
    # the round-4 conversion (pageable .cpu(), single-threaded numpy astype /
    # NaN fill; the confidences widened to fp64 on the device first), for comparison
    t3 = time.perf_counter()
    a = lab._labels_dev[0].cpu().numpy().astype(np.float64)
    a[a < 0] = np.nan
    b = lab._conf_dev[0].double().cpu().numpy()
    t4 = time.perf_counter()
    same = bool(np.array_equal(a, tid, equal_nan=True) and np.array_equal(b, cid, equal_nan=True))
    del a, b
    return {"pixels": n, "tissue_IDs_ms": round((t1 - t0) * 1e3, 3),
            "confidence_IDs_ms": round((t2 - t1) * 1e3, 3),
            "round4_conversion_ms": round((t4 - t3) * 1e3, 3), "equal_to_round4": same,
            "d2h_bytes": 5 * n, "host_bytes_written": 16 * n,
            "note": "first access of lab.tissue_IDs[0] / lab.confidence_IDs[0] (float64, NaN outside "
                    "the mask) after the timed steps; not part of the headline step, whose outputs "
                    "stay in HBM"}


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if os.environ.get("MW_BENCH_SHARE_GPU") != "1":
            check_devices(args.gpus)  # before any GPU call
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "--gpus" in " ".join(sys.argv):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MW_BENCH_SHARE_GPU=1 with MW_BENCH_BACKEND=gloo: every rank on cuda:0 and
    # the messages over gloo (the multi-rank host path rehearsed on one GPU;
    # RCCL needs one GPU per rank)
    share = os.environ.get("MW_BENCH_SHARE_GPU") == "1"
    backend = os.environ.get("MW_BENCH_BACKEND", "nccl")
    if share:
        local = 0
    check_devices(local + 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from milwrm_amd import device as D
    from milwrm_amd import profiling
    from milwrm_amd.dist import make_comm

    comm = make_comm()
    H = W = args.size
    C = args.channels
    n_sl = args.slides_per_gpu
    source = args.source
    if source == "auto":
        total = torch.cuda.get_device_properties(local).total_memory
        source = "device" if n_sl * H * W * C * 2 <= 0.6 * total else "synth"
    seeds = [20251015 + rank * n_sl + i for i in range(n_sl)]
    slides = Slides(H, W, C, seeds, source, args.mode)
    step = make_step(slides, C, args.k, comm, sweep=args.sweep)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(max(args.warmup, 1 if args.sweep else 0)):
        step()
    barrier()
    profiling.reset()
    profiling.enable(True)
    barrier()
    prof_path = os.environ.get("MW_BENCH_CPROFILE")  # diagnostics: host profile of the timed steps
    if prof_path:
        import cProfile
        cpr = cProfile.Profile()
        cpr.enable()
    t0 = time.perf_counter()
    lab = None
    for _ in range(args.steps):
        if not args.sweep:
            lab = None  # the last step's buffers go before the next step allocates (40k^2 x 50 fits once)
        lab = step()
    barrier()
    elapsed = time.perf_counter() - t0
    if prof_path:
        cpr.disable()
        cpr.dump_stats(f"{prof_path}.{rank}")
        ms_ = torch.cuda.memory_stats()
        print(json.dumps({k: ms_.get(k) for k in ("num_alloc_retries", "num_device_alloc",
                                                  "num_device_free", "num_ooms")}),
              file=sys.stderr, flush=True)
    profiling.enable(False)
    prof = profiling.summary()
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    px_total = world * n_sl * H * W * args.steps
    value = px_total / elapsed

    S = int(lab._rows.S)  # this rank's rows (all its slides)
    F, k = C, args.k
    # dominant kernel by device time inside the timed region (timed regions
    # without an algorithmic byte count, e.g. the whole k-means fit in the C++
    # driver, are not kernels with a roofline; read_* is the slide reader)
    dom_name, dom = max(((n, r) for n, r in prof.items() if r["bytes"] > 0 and not n.startswith("read_")),
                        key=lambda kv: kv[1]["total_ms"])
    per_launch_bytes = dom["bytes"] / max(dom["count"], 1)
    achieved = per_launch_bytes / (dom["mean_ms"] * 1e-3) / 1e9
    traffic, traffic_src, counters = pmc_traffic(dom_name, "_c5" if (H, W, C) == (40000, 40000, 50) else "")
    reads = {n: r for n, r in prof.items() if n.startswith("read_")}
    read_info = None
    if reads:
        rb = sum(r["bytes"] for r in reads.values()) / args.steps
        rms = sum(r["total_ms"] for r in reads.values()) / args.steps
        read_info = {"kind": source, "bytes_per_step": rb, "ms_per_step_side_stream": rms,
                     "GBps": rb / max(rms, 1e-9) / 1e6,
                     "note": "raw slide bands read on a side stream (overlapping the passes on the "
                             "main stream) inside the timed step; synth = generated on the device, "
                             "host = host-to-device copies over PCIe"}
    workload = (f"mxif_labeler: {world} GPU(s) x {n_sl} synthetic {C}-ch {H}x{W} slide(s) per GPU, "
                f"k={k}, sigma=2, fract=0.2, random_state=18 ({_config_name(H, W, C, n_sl, world, args.sweep)})")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "pixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (fp64 accumulation)",
        "data": "synthetic (device-generated Voronoi/gamma slides, SURVEY 8d; uint16 HWC + mask)",
        "config": {"workload": workload, "source": source,
                   "blur": ("deferred (fused epilogues)" if source != "device" or D.defer_blur(H, W, C)
                            else "materialised"),
                   "slides_per_gpu": n_sl, "H": H, "W": W, "C": C, "k": k, "mode": args.mode,
                   "samples_per_slide": S // n_sl, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": achieved,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "counters": counters,
                     "launches": dom["count"], "avg_launch_ms": dom["mean_ms"],
                     "algorithmic_bytes_per_launch": per_launch_bytes},
        "slide_reads": read_info,
        "kernels": {n: {"count": v["count"], "mean_ms": round(v["mean_ms"], 4),
                        "total_ms_per_step": round(v["total_ms"] / args.steps, 4)}
                    for n, v in sorted(prof.items())},
        "cpu_baseline": None,
    }
    if args.sweep:
        curve = lab.inertia_curve_
        iters = curve.attrs.get("n_iter", {})
        passes = [n for n in prof if n.startswith("lloyd_pass") or n.startswith("lloyd_mark")]
        pass_ms = sum(prof[n]["total_ms"] for n in passes) / args.steps
        fit_passes = sum(int(v) + 1 for v in iters.values())  # Lloyd iterations + the final E-step
        S_glob = S * world
        out["metric"] = ("pixels/sec (node) through find_optimal_k (k=2..20 sweep, inertia curve) over "
                         "the prepped rows of 30-ch MxIF slides")
        hostp = prof.get("lloyd_fits_host", {})
        commp = prof.get("lloyd_fits_comm", {})
        out["sweep_driver"] = {
            "iterations": int(hostp.get("count", 0)) // max(args.steps, 1),
            "host_ms_per_iteration": hostp.get("total_ms", 0.0) / max(hostp.get("count", 0), 1),
            "comm_ms_per_iteration": commp.get("total_ms", 0.0) / max(commp.get("count", 0), 1) if commp else 0.0,
            "backend": dist.get_backend() if world > 1 else None,
            "note": "mw_lloyd_fits(_sharded): host time from a pass's records arriving to the next pass "
                    "queued, and time inside the all-reduce callback (sharded runs)"}
        out["sweep"] = {"seconds": ms / 1e3, "best_k": int(lab.k), "rows_total": S_glob,
                        "n_iter": {int(a): int(b) for a, b in iters.items()},
                        "fit_passes": fit_passes, "lloyd_device_ms": pass_ms,
                        "device_ms_per_fit_pass": pass_ms / max(fit_passes, 1),
                        "curve": [float(v) for v in curve["Scaled Inertia"].values]}
        if world == 1:
            out["sweep"]["alu_roofline"] = dense_pass_roofline(lab._device_rows())
        out["config"]["workload"] = (f"find_optimal_k k=2..20 over {world} GPU(s) x {n_sl} synthetic "
                                     f"{C}-ch {H}x{W} slide(s) per GPU ({S_glob} rows; "
                                     f"{_config_name(H, W, C, n_sl, world, True)})")
    else:
        n_iter = int(lab.kmeans.n_iter_)
        # SURVEY §8(d) whole-pipeline algorithmic bytes (per slide)
        N_pix = H * W
        S1 = S / n_sl
        B = (N_pix * C * 2 + (N_pix * C * 2 + N_pix + S1 * F * 4) + (k + n_iter + 1) * S1 * F * 4
             + (N_pix * F * 2 + N_pix + 5 * N_pix))
        pipe_gbps = B * world * n_sl / (elapsed / args.steps) / 1e9
        out["config"]["lloyd_iters"] = n_iter
        out["pipeline_roofline"] = {"algorithmic_bytes_per_slide": B, "achieved": pipe_gbps,
                                    "unit": "GB/s", "frac": pipe_gbps / (HBM_PEAK_GBPS * world)}
        # the formula counts (k + n_iter + 1) full passes over the rows; the
        # pruned Lloyd passes read only the rows their bounds leave open: the
        # rows each pass of the last fit really read (mw_kmeans_fit_history)
        fr = fit_rows_read(S, F, k)
        if fr is not None:
            formula_fit = (k + n_iter + 1) * S1 * F * 4
            read_fit = fr / n_sl * F * 4
            B_read = B - formula_fit + read_fit
            out["pipeline_roofline"].update({
                "fit_bytes_per_slide_formula": formula_fit, "fit_bytes_per_slide_read": read_fit,
                "bytes_read_per_slide": B_read,
                "achieved_bytes_read": B_read * world * n_sl / (elapsed / args.steps) / 1e9,
                "note": "fit_bytes_per_slide_read: k k-means++ passes over every row + the rows each "
                        "Lloyd pass of the rank's last fit read (its bounds skip the rest), x F x 4 B"})
            out["pipeline_roofline"]["frac_bytes_read"] = (out["pipeline_roofline"]["achieved_bytes_read"]
                                                           / (HBM_PEAK_GBPS * world))
    if not args.sweep and not args.no_host_outputs:
        out["host_outputs"] = host_outputs(lab)
    if (world == 1 and not args.sweep and args.mode == "hard" and not args.no_design_point
            and source == "device" and n_sl == 1 and H * W * C * 2 <= 20e9):
        out["design_point"] = design_point(H, W, C, args.k, comm, lab)
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_size, C, args.k, sweep=args.sweep)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
