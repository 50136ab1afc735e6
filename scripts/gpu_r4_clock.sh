#!/bin/bash
# Effective shader clock per GEMM dispatch (GRBM_GUI_ACTIVE / 8 XCDs / wall time, the DVFS check of
# MI355X_MICROARCH.md) in DeiT-base forwards at 64 and 512 images: are the 150-tile N = 768 GEMMs
# at 64 images (150 of 256 CUs busy) faster per K-tile because they clock higher?
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-clock}
mkdir -p $O
for B in 64 512; do
  timeout -s KILL 120 rocprofv3 --pmc ${PMC:-GRBM_GUI_ACTIVE GRBM_COUNT} --output-format csv -d $O/b$B -o run \
    -- python3 $R/bench.py --batch $B --cpu-seconds 0 --no-probe --steps 2 --warmup 1 > $O/b$B.log 2>&1 || exit 1
  python3 - "$O/b$B" "$B" <<'PY'
import csv, glob, collections, sys
O, B = sys.argv[1], sys.argv[2]
rows = collections.defaultdict(dict)
hdr = None
for f in glob.glob(f"{O}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        hdr = hdr or list(r.keys())
        d = rows[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]; d["grid"] = r.get("Grid_Size", "?")
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k in ("Start_Timestamp", "End_Timestamp"):
            if k in r: d[k] = int(r[k])
print("columns:", hdr)
by = collections.defaultdict(list)
seq = [rows[k] for k in sorted(rows)]
k197 = 0
for d in seq:
    n = d["name"]
    if "gemm_pers_kernel" not in n: continue
    role = n.split("gemm_pers_kernel<")[1].split(",")[0]
    if role == "197":
        role = "197-outproj" if k197 % 2 == 0 else "197-fc2"; k197 += 1
    if "Start_Timestamp" in d:
        us = (d["End_Timestamp"] - d["Start_Timestamp"]) / 1e3
        by[role].append((us, {c: d[c] for c in d if c.isupper()}))
for role, v in sorted(by.items()):
    v.sort(key=lambda x: x[0])
    us, c = v[len(v) // 2]
    print(f"bs{B} {role}: n {len(v)} median {us:.1f} us", " ".join(
        f"{k} {x:.4e} ({x / us / 1e3:.3f}/ns)" for k, x in sorted(c.items())))
PY
done
