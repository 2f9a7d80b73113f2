"""Per-kernel, per-pattern FETCH_SIZE / WRITE_SIZE (KB counters, summed over
the dispatches of one kernel in dispatch order seq, rand, seq, rand) against
the algorithmic bytes of tools/pmc_calib_r5.py.
usage: python tools/pmc_calib_r5_report.py <gpurun_out dir> <calib.json> <out.json>"""
import collections
import csv
import glob
import json
import sys

KERN = {"sample_map": "sample_map_kernel<false>", "blur_sample": "true, 1>(",
        "col_stats": "col_stats_rows_kernel"}


def per_dispatch(path):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"])
    return rows


def main(d, calib, outp):
    cal = json.load(open(calib))
    pats = list(cal["ms"].keys())
    res = {}
    for cnt in ("fetch", "write"):
        f = glob.glob(f"{d}/{cnt}/**/*counter_collection.csv", recursive=True)
        if not f:
            continue
        disp = per_dispatch(f[0])
        for name, pat in KERN.items():
            vals = [v for (i, k), v in sorted(disp.items()) if pat in k]
            for j, v in enumerate(vals):
                p = pats[j % len(pats)]
                res.setdefault(name, {}).setdefault(p, {}).setdefault(cnt, []).append(v * 1024.0)
    table = {}
    for name, by in res.items():
        alg = cal["algorithmic_bytes"][name]
        for p, c in by.items():
            fb = sum(c.get("fetch", [0])) / max(len(c.get("fetch", [1])), 1)
            wb = sum(c.get("write", [0])) / max(len(c.get("write", [1])), 1)
            table.setdefault(name, {})[p] = {
                "fetch_bytes_raw": fb, "fetch_x2": 2 * fb, "write_bytes": wb,
                "alg_read": alg["read"], "alg_write": alg["write"],
                "fetch_x2_over_alg": (2 * fb / alg["read"]) if alg["read"] else None,
                "write_over_alg": (wb / alg["write"]) if alg["write"] else None}
    json.dump({"calib": cal, "table": table}, open(outp, "w"), indent=1)
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
