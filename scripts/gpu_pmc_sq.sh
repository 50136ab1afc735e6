#!/bin/bash
# SQ / TA / TCP counters of the FC1 probe GEMM (bench.py --probe-only), one rocprofv3 pass per
# counter group (slot limits: 8 SQ, 2 TA, 2 TD, 4 TCP, 2 GRBM), kernel-trace only.
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_sq${TAG:-}
mkdir -p $O
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --output-format csv -d $O/p$i -o run \
    -- python3 $R/bench.py --probe-only 10 ${BENCH_ARGS:-} > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'G'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES
GRBM_GUI_ACTIVE GRBM_TA_BUSY TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
G
python3 - "$O" <<'PY'
import csv, glob, collections, sys
O = sys.argv[1]
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{O}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_pers" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
out = {k: agg[k] / n[k] for k in agg}  # per launch (each counter summed over its dispatch's rows)
import json; print(json.dumps({k: f"{v:.4e}" for k, v in sorted(out.items())}, indent=0))
PY
