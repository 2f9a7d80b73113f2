"""Per-kernel mean of rocprofv3 --pmc counters over all dispatches, from
gpurun_out/pmc_<tag>/<pass>/**/run_counter_collection.csv.  FETCH_SIZE is
reported doubled (gfx950 tallies a 128-B streaming request as 64 B:
MI355X_MICROARCH.md §HBM); both are in kB as rocprofv3 reports them."""
import collections
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "bench"
per = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        c = r["Counter_Name"]
        per[k][c] += float(r["Counter_Value"])
        cnt[k][c].add(r["Dispatch_Id"])
for k in sorted(per):
    d = {c: v / max(len(cnt[k][c]), 1) for c, v in per[k].items()}
    if "FETCH_SIZE" in d:
        d["HBM_READ_MB"] = 2 * d.pop("FETCH_SIZE") / 1e3
    if "WRITE_SIZE" in d:
        d["HBM_WRITE_MB"] = d.pop("WRITE_SIZE") / 1e3
    print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
