#!/bin/bash
# PMC passes on the GEMM microbench (GS shapes, GV variants); one counter group per pass.
set -u
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
export GS=${GS:-fc2}
i=0
while read -r CTRS; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/pmc2/p$i -o run \
    -- python3 $R/scripts/gemm_bench.py ${GM:-100864} ${GV:-6,8} > $R/gpurun_out/pmc2/p$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc ($CTRS)"; [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
LIST
find $R/gpurun_out/pmc2 -name "*counter_collection*" | head -20
