"""HBM traffic per launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/gpu/pmc_bench.sh (gpurun_out/pmc_<tag>/{fetch,write}/run_counter_collection.csv)
-> a JSON table bench.py reads for roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): both counters are
in KB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
streaming stores.  Kernels whose reads are not wide coalesced streams (the
random-row gather) are uncalibrated and flagged as such.

usage: python tools/pmc_traffic.py <tag> <out.json>
"""
import collections
import csv
import json
import re
import sys

# bench.py profiling names -> substring of the HIP kernel symbol
KERNELS = {
    "blur": "true, 0>(",           # blur_mfma_kernel<T, R, CT, BT, true, kEpiStore>
    "blur_sample": "true, 1>(",    # ... kEpiSample (deferred blur: rows written by the blur)
    "blur_assign": "true, 2>(",    # ... kEpiAssign (deferred blur: labels written by the blur)
    "assign_conf": "assign_kernel<",
    "kpp_init": "kpp_pass_kernel<32, 1, 0>",
    "kpp_step1": "kpp_pass_kernel<32, 4, 1>",
    "kpp_step": "kpp_pass_kernel<32, 4, 2>",
    "lloyd_pass_mode0_first": "lloyd_pass_kernel<32, 0, 0, 1>",
    "lloyd_pass_mode0_tile": "lloyd_pass_kernel<32, 0, 1, 1>",
    "lloyd_pass_mode1": "lloyd_pass_kernel<32, 1, 0, 1>",
    "lloyd_pass_mode2": "lloyd_pass_kernel<32, 2, 0, 1>",
    "kpp_init_f64": "kpp_pass_kernel<64, 1, 0>",
    "kpp_step1_f64": "kpp_pass_kernel<64, 4, 1>",
    "kpp_step_f64": "kpp_pass_kernel<64, 4, 2>",
    "lloyd_first_f64": "lloyd_pass_kernel<64, 0, 0, 1>",
    "lloyd_first_w2": "lloyd_first_w2_kernel",
    "lloyd_tile_f64": "lloyd_pass_kernel<64, 0, 1, 1>",
    "lloyd_queue_f64": "lloyd_pass_kernel<64, 0, 2, 1>",
    "lloyd_final_f64": "lloyd_pass_kernel<64, 1, 0, 1>",
    "lloyd_list_f64": "lloyd_pass_kernel<64, 0, 4, 1>",
    "lloyd_list": "lloyd_pass_kernel<32, 0, 4, 1>",
    "lloyd_mark": "lloyd_mark_kernel",
    "sample_map": "sample_map_kernel",
    "col_stats": "col_stats_rows_kernel",
    "gather": "gather_kernel<true, false, false>",  # (round 5: the PX flag joined the template)
    "lloyd_first_w3": "lloyd_first_w3_kernel",
    "lloyd_pass_mode0_dense": "lloyd_dense2_kernel",
    "nz_stats": "nz_stats_u16_kernel",
    "mask_scatter": "mask_scatter_kernel",
}
# not wide coalesced streams: random rows / atomics, and 4-byte loads (col_stats).
# The gather was calibrated in round 4 (tools/gather_calib.py,
# profiles/r04/gather_calib/): the same kernel over a sequential draw pattern
# reads FETCH_SIZE x 2 = 2.13 GB for 2.18 GB of algorithmic reads, so the x2
# correction holds for it; over config 2's random draws x2 gives 6.17 GB =
# two 128-B lines per straddling 120-B row plus one per random rank lookup.
# Round 5 (tools/pmc_calib_r5.py, profiles/r05/calib/): over known draw patterns
# blur_sample's FETCH_SIZE x 2 is 1.35x its algorithmic reads for sequential
# and random draws alike (the blur's halo over-fetch, as the plain blur) and
# its WRITE_SIZE is exact for sequential rows (1.19x for random 120-B rows);
# sample_map's FETCH_SIZE x 2 is exact for sequential draws (random draws: a
# 128-B line per rank lookup); col_stats_rows' FETCH_SIZE is exact WITHOUT
# the x2 (its loads are not the wide streaming kind the correction is for).
UNCALIBRATED = {"lloyd_list", "lloyd_list_f64"}
FETCH_FACTOR = {"col_stats": 1}  # default 2
# calibrated on config 2's shape only: col_stats' x1 was exact at F = 30 (the
# config-5 slice's F = 50 rows read 0.86x of their bytes under it), and the
# config-5 sample map looks ranks up in the compact index, not the table the
# calibration used
CALIBRATED_C2_ONLY = {"col_stats", "sample_map"}


def per_launch(path, pat):
    tot = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if pat in r["Kernel_Name"]:
            tot[r["Dispatch_Id"]] += float(r["Counter_Value"])
    if not tot:
        return None, 0
    return sum(tot.values()) / len(tot), len(tot)


def main():
    tag, out = sys.argv[1], sys.argv[2]
    base = f"gpurun_out/pmc_{tag}"
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                     f"'bench.py --steps 1 --warmup 1' ({base})",
           "correction": "KB -> bytes; FETCH_SIZE x2 (gfx950 wide-read undercount; x1 for "
                         "col_stats_rows, calibrated round 5); WRITE_SIZE as reported",
           "kernels": {}}
    for name, pat in KERNELS.items():
        f, nf = per_launch(f"{base}/fetch/run_counter_collection.csv", pat)
        w, nw = per_launch(f"{base}/write/run_counter_collection.csv", pat)
        if f is None or w is None:
            continue
        fb, wb = FETCH_FACTOR.get(name, 2) * f * 1024, w * 1024
        cal = name not in UNCALIBRATED and not (name in CALIBRATED_C2_ONLY and "c5" in tag)
        res["kernels"][name] = {"symbol": pat, "launches": nf, "fetch_bytes": fb, "write_bytes": wb,
                                "traffic_bytes": fb + wb, "calibrated": cal}
    json.dump(res, open(out, "w"), indent=1)
    for n, v in res["kernels"].items():
        print(f"{n:18s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
