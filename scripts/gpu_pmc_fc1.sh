#!/bin/bash
# HBM traffic of the FC1 probe GEMM (bench.py --probe-only): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (TCC slots), kernel-trace only, no other trace domains.
set -u
mkdir -p gpurun_out/pmc_fc1
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_fc1/$C -o run \
    -- python3 $R/bench.py --probe-only 10 > $R/gpurun_out/pmc_fc1/$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_fc1 > $R/gpurun_out/pmc_fc1/summary.json
cat $R/gpurun_out/pmc_fc1/summary.json
