"""Summary JSON of one gpu_pmc_kernel.sh output directory: per-launch counter averages of the
kernels matching a name (FETCH_SIZE doubled per the gfx950 note) and per-launch durations by grid
from its kernel-trace pass.   python scripts/pmc_kernel_summary.py DIR KERNEL_SUBSTRING [note]"""
import collections
import csv
import glob
import json
import sys

O, kname = sys.argv[1], sys.argv[2]
agg, n = collections.defaultdict(float), collections.defaultdict(set)
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(r["Dispatch_Id"])
c = {k: agg[k] / len(n[k]) for k in agg}
if "FETCH_SIZE" in c:
    c["FETCH_BYTES_corrected"] = 2 * 1024 * c["FETCH_SIZE"]
if "WRITE_SIZE" in c:
    c["WRITE_BYTES"] = 1024 * c["WRITE_SIZE"]
by = collections.defaultdict(list)
for f in glob.glob(f"{O}/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            by[r.get("Grid_Size_X", "?")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(json.dumps({
    "kernel": kname, "note": sys.argv[3] if len(sys.argv) > 3 else "",
    "launches_per_counter": max((len(v) for v in n.values()), default=0),
    "per_launch_counters": {k: round(v, 1) for k, v in sorted(c.items())},
    "per_launch_us_by_grid_threads": {g: {"launches": len(v), "median_us": round(sorted(v)[len(v) // 2], 1)}
                                      for g, v in sorted(by.items())},
}, indent=1))
