#!/bin/bash
# PMC counters for the GEMM microbench (one counter set per pass; no trace domains).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/pmc/p1 -o run \
  -- python3 $R/scripts/gemm_bench.py ${GM:-100864} ${GV:-2} > $R/gpurun_out/pmc/p1.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc/p2 -o run \
  -- python3 $R/scripts/gemm_bench.py ${GM:-100864} ${GV:-2} > $R/gpurun_out/pmc/p2.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $R/gpurun_out/pmc/p3 -o run \
  -- python3 $R/scripts/gemm_bench.py ${GM:-100864} ${GV:-2} > $R/gpurun_out/pmc/p3.log 2>&1
rc=$?; echo "pass3 rc=$rc"
find $R/gpurun_out/pmc -name "*.csv" | head
exit $rc
