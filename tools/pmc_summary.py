"""Per-kernel PMC summary of one tools/gpu/pmc_bench.sh run (passes sq, mfma,
fetch, write under gpurun_out/pmc_<tag>/) -> the JSON bench.py reads for
roofline.traffic / roofline.counters (profiles/rNN/pmc_traffic[_c5]_vN.json).

Traffic: FETCH_SIZE / WRITE_SIZE per launch with the gfx950 corrections of
tools/pmc_traffic.py.  SQ: fractions of SQ_WAVE_CYCLES summed over a kernel's
launches (all SQ cycle counters in the same quad-cycle unit);
mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).

usage: python tools/pmc_summary.py <tag> <out.json> "<workload text>"
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_traffic as PT  # noqa: E402

SQ_KERNELS = {
    "blur": "true, 0>(",
    "blur_sample": "true, 1>(",
    "assign_conf": "assign_kernel<",
    "kpp_pass": "kpp_pass_kernel<",
    "lloyd_pass": "lloyd_pass_kernel<",
    "lloyd_mark": "lloyd_mark_kernel",
    "gather": "gather_kernel<true, false, false>",
    "col_stats_rows": "col_stats_rows_kernel",
    "nz_stats": "nz_stats_u16_kernel",
    "sample_map": "sample_map_kernel",
}


def counters(base, pas):
    """{(kernel pattern name, counter): (sum over launches, launches)}"""
    out = collections.defaultdict(lambda: [0.0, set()])
    for f in glob.glob(f"{base}/{pas}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            for name, pat in SQ_KERNELS.items():
                if pat in r["Kernel_Name"]:
                    a = out[(name, r["Counter_Name"])]
                    a[0] += float(r["Counter_Value"])
                    a[1].add(r["Dispatch_Id"])
    return {k: (v[0], len(v[1])) for k, v in out.items()}


def main():
    tag, out_path, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    base = f"gpurun_out/pmc_{tag}"
    res = {"source": f"rocprofv3 --pmc, separate passes (sq, mfma, fetch, write) over "
                     f"'bench.py --steps 1 --warmup 1' ({base})",
           "correction": "KB -> bytes; FETCH_SIZE x2 (gfx950 wide-read undercount; x1 for col_stats_rows, "
                         "calibrated round 5); WRITE_SIZE as reported",
           "workload": workload, "kernels": {}, "sq": {},
           "sq_note": "SQ_* fractions of SQ_WAVE_CYCLES; mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / "
                      "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); separate rocprofv3 --pmc passes "
                      "(tools/gpu/pmc_bench.sh passes sq, mfma)"}
    for name, pat in PT.KERNELS.items():
        f, nf = PT.per_launch(f"{base}/fetch/run_counter_collection.csv", pat)
        w, nw = PT.per_launch(f"{base}/write/run_counter_collection.csv", pat)
        if f is None or w is None:
            continue
        fb, wb = PT.FETCH_FACTOR.get(name, 2) * f * 1024, w * 1024
        cal = name not in PT.UNCALIBRATED and not (name in PT.CALIBRATED_C2_ONLY and "c5" in tag)
        res["kernels"][name] = {"symbol": pat, "launches": nf, "fetch_bytes": fb, "write_bytes": wb,
                                "traffic_bytes": fb + wb, "calibrated": cal}
    sq = counters(base, "sq")
    mf = counters(base, "mfma")
    for name in SQ_KERNELS:
        wc = sq.get((name, "SQ_WAVE_CYCLES"))
        if not wc or wc[0] <= 0:
            continue
        g = lambda c: sq.get((name, c), (0.0, 0))[0]  # noqa: E731
        e = {"wait_any_frac": g("SQ_WAIT_ANY") / wc[0], "wait_inst_frac": g("SQ_WAIT_INST_ANY") / wc[0],
             "active_inst_frac": g("SQ_ACTIVE_INST_ANY") / wc[0]}
        wc2 = mf.get((name, "SQ_WAVE_CYCLES"))
        if wc2 and wc2[0] > 0:
            m = lambda c: mf.get((name, c), (0.0, 0))[0]  # noqa: E731
            n = max(wc2[1], 1)
            e["valu_active_frac"] = m("SQ_ACTIVE_INST_VALU") / wc2[0]
            e["valu_insts_per_launch"] = g("SQ_INSTS_VALU") / max(wc[1], 1)
            e["mfma_insts_per_launch"] = m("SQ_INSTS_MFMA") / n
            grbm = m("GRBM_GUI_ACTIVE")
            e["mfma_busy_frac"] = m("SQ_VALU_MFMA_BUSY_CYCLES") / (grbm / 8 * 1024) if grbm > 0 else 0.0
        res["sq"][name] = {k: round(v, 4) if isinstance(v, float) and v < 1e6 else v for k, v in e.items()}
    json.dump(res, open(out_path, "w"), indent=1)
    for n, v in res["kernels"].items():
        print(f"{n:18s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")
    for n, v in res["sq"].items():
        print(n, v)


if __name__ == "__main__":
    main()
