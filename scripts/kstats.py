"""Summarise a rocprofv3 kernel_stats.csv: name, calls, average (us), share, per-image ns."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
b = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} {float(r["AverageNs"]) / 1e3:9.1f} us '
          f'{100 * float(r["TotalDurationNs"]) / tot:5.1f} % {float(r["AverageNs"]) / b:8.1f} ns/img')
