"""Summarise rocprofv3 counter_collection.csv files under gpurun_out/pmc_<tag>/
(last dispatch of each kernel matching a substring)."""
import collections
import csv
import glob
import sys

tag, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    names = {}
    for r in rows:
        if pat not in r["Kernel_Name"]:
            continue
        agg[(r["Kernel_Name"][:60], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        names[r["Kernel_Name"][:60]] = r["Dispatch_Id"]
    last = collections.defaultdict(dict)
    for (k, d, c), v in agg.items():
        if d == names[k]:
            last[k][c] = v
    for k, d in last.items():
        print(f.split("/")[-2], k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
