"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_fc1.sh for the FC1 probe GEMM
(the persistent gemm_pers_kernel<35> since the persistent kernel became the default): per-launch HBM bytes, gfx950 FETCH_SIZE doubled (MI355X_MICROARCH.md)."""
import csv
import datetime
import glob
import json
import os
import sys

root = sys.argv[1]
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True)
    rows = [r for r in csv.DictReader(open(f[0]))
            if ("gemm_pers_kernel<35" in r["Kernel_Name"] or "gemm_big_kernel<35" in r["Kernel_Name"])
            and r["Counter_Name"] == c]
    vals["kernel_name"] = rows[0]["Kernel_Name"] if rows else None
    v = sorted(float(r["Counter_Value"]) for r in rows)
    vals[c] = v[len(v) // 2]  # median over launches (KB, rocprofv3 derived metric)
probe = [l for l in open(os.path.join(root, "FETCH_SIZE.log")) if l.startswith("{")]
shape = json.loads(probe[-1]) if probe else {}
M, K, N = shape.get("M"), shape.get("K"), shape.get("N")
fetch = 2 * vals["FETCH_SIZE"] * 1024
write = vals["WRITE_SIZE"] * 1024
algo = (M * K + K * N + M * N) * 2 if M else None
print(json.dumps({"kernel": "FC1 LNIN|BIAS|GELU (bf16): " + str(vals.get("kernel_name")), "M": M, "K": K, "N": N,
                  "FETCH_SIZE_KB_raw": vals["FETCH_SIZE"], "WRITE_SIZE_KB": vals["WRITE_SIZE"],
                  "fetch_bytes_corrected": fetch, "write_bytes": write,
                  "traffic_bytes_per_launch": fetch + write, "algorithmic_bytes": algo,
                  "commit": os.environ.get("COMMIT"),
                  "collected": datetime.datetime.utcnow().strftime("%Y-%m-%dT%H:%MZ")},
                 indent=1))
