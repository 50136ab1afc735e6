#!/bin/bash
# SQ counters of the MX8 GEMM on the DeiT QKV shape (one rocprofv3 pass, kernel-trace only)
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_mx8
timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAVE_CYCLES} --output-format csv -d $R/gpurun_out/pmc_mx8 -o run \
  -- python3 $R/scripts/mx8_bench.py --only qkv --reps 3 > $R/gpurun_out/pmc_mx8/run.log 2>&1
rc=$?; tail -3 $R/gpurun_out/pmc_mx8/run.log; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
f = glob.glob(f"{R}/gpurun_out/pmc_mx8/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    if "gemm" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v:.3e}" for c, v in d.items()})
PY
