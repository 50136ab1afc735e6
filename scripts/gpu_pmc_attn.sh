#!/bin/bash
# SQ counters of the bf16 attention kernel (scripts/attn_bench.py), one rocprofv3 pass per group.
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_attn${TAG:-}
mkdir -p $O
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --output-format csv -d $O/p$i -o run \
    -- python3 $R/scripts/attn_bench.py > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'G'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_ACTIVE_INST_ANY
GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
FETCH_SIZE
WRITE_SIZE
G
python3 - "$O" <<'PY'
import csv, glob, collections, sys, json
O = sys.argv[1]
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{O}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "attn_bf16" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(json.dumps({k: f"{agg[k] / n[k]:.4e}" for k in sorted(agg)}, indent=0))
PY
