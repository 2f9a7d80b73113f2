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


def _config_name(H, W, C):
    """Which BASELINE.json config one GPU's slice of this workload is."""
    if (H, W, C) == (10000, 10000, 30):
        return "BASELINE config 2 per GPU"
    if (H, W, C) == (20000, 20000, 30):
        return "BASELINE config 3 per GPU: one of its 8 slides"
    if (H, W, C) == (40000, 40000, 50):
        return "BASELINE config 5 per GPU: one of its 16 slides (one slide per GPU step)"
    return "custom size"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=10000, help="slide is size x size pixels")
    ap.add_argument("--channels", type=int, default=30)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--mode", default="hard", choices=["hard", "easy"])
    ap.add_argument("--cpu-size", type=int, default=2048, help="oracle CPU-baseline slide side")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def make_step(raw, mask, k, comm):
    import pandas as pd

    import milwrm_amd as M

    def step():
        with contextlib.redirect_stdout(sys.stderr):  # reference-style progress prints
            return _step()

    def _step():
        im = M.img.from_device(raw, mask)
        est, pix = im.calculate_non_zero_mean()
        est, pix = comm.batch_stats(est, pix)
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(raw.shape[2])), sigma=2, fract=0.2,
                              comm=comm)
        lab.label_tissue_regions(k=k, plot_out=False, random_state=18, comm=comm)
        lab.confidence_score_images()
        return lab

    return step


def cpu_baseline(size, C, k):
    """Oracle (numpy/scipy restatement of the reference pipeline) on a bounded
    host sample; Mpix/s on this box's cores."""
    from threadpoolctl import threadpool_info

    from oracle import milwrm_oracle as O

    raw, mask = O.synth_slide(size, size, C, seed=20251015, mode="hard")
    t = time.perf_counter()
    r = O.mxif_pipeline([raw], [mask], ["b"], list(range(C)), k=k)
    dt = time.perf_counter() - t
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    return dict(value=size * size / dt, unit="pixels/s", cores=int(threads), kind="port",
                sample=f"oracle mxif_pipeline on one {size}x{size}x{C} synthetic slide, k={k} "
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


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        check_devices(args.gpus)  # before any GPU call
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "--gpus" in " ".join(sys.argv):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_devices(local + 1)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from milwrm_amd import device as D
    from milwrm_amd import profiling
    from milwrm_amd.dist import make_comm

    comm = make_comm()
    H = W = args.size
    C = args.channels
    raw, mask = D.synth_slide(H, W, C, seed=20251015 + rank, mode=args.mode)
    torch.cuda.synchronize()
    step = make_step(raw, mask, args.k, comm)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
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
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    px_total = world * H * W * args.steps
    value = px_total / elapsed

    n_iter = int(lab.kmeans.n_iter_)
    S = int(lab._rows.S)
    # dominant kernel by device time inside the timed region
    # (timed regions without an algorithmic byte count, e.g. the whole k-means
    # fit in the C++ driver, are not kernels with a roofline)
    dom_name, dom = max(((n, r) for n, r in prof.items() if r["bytes"] > 0),
                        key=lambda kv: kv[1]["total_ms"])
    per_launch_bytes = dom["bytes"] / max(dom["count"], 1)
    achieved = per_launch_bytes / (dom["mean_ms"] * 1e-3) / 1e9
    traffic, traffic_src, counters = pmc_traffic(dom_name, "_c5" if (H, W, C) == (40000, 40000, 50) else "")
    # SURVEY §8(d) whole-pipeline algorithmic bytes (per slide)
    N_pix, F, k = H * W, C, args.k
    B = (N_pix * C * 2 + (N_pix * C * 2 + N_pix + S * F * 4) + (k + n_iter + 1) * S * F * 4
         + (N_pix * F * 2 + N_pix + 5 * N_pix))
    pipe_gbps = B * world / (elapsed / args.steps) / 1e9
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
        "config": {"workload": f"mxif_labeler: {world} x synthetic {C}-ch {H}x{W} slide (one per GPU), "
                               f"k={k}, sigma=2, fract=0.2, random_state=18 ({_config_name(H, W, C)})",
                   "blur": "deferred (fused epilogues)" if D.defer_blur(H, W, C) else "materialised",
                   "slides_per_gpu": 1, "H": H, "W": W, "C": C, "k": k, "mode": args.mode,
                   "samples_per_slide": S, "lloyd_iters": n_iter, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": achieved,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "counters": counters,
                     "launches": dom["count"], "avg_launch_ms": dom["mean_ms"],
                     "algorithmic_bytes_per_launch": per_launch_bytes},
        "pipeline_roofline": {"algorithmic_bytes_per_slide": B, "achieved": pipe_gbps,
                              "unit": "GB/s", "frac": pipe_gbps / (HBM_PEAK_GBPS * world)},
        "kernels": {n: {"count": v["count"], "mean_ms": round(v["mean_ms"], 4),
                        "total_ms_per_step": round(v["total_ms"] / args.steps, 4)}
                    for n, v in sorted(prof.items())},
        "cpu_baseline": None,
    }
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_size, C, args.k)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
