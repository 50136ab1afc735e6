#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes: TCC slots; kernel-trace only) of
#   fc1   the FC1 probe GEMM (bench.py --probe-only)  -> profiles/*_pmc_fc1.json via pmc_summary.py
#   swin  a short Swin-T bs256 bench (per-kernel table)
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_fc1 $R/gpurun_out/pmc_swin
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_fc1/$C -o run \
    -- python3 $R/bench.py --probe-only 10 > $R/gpurun_out/pmc_fc1/$C.log 2>&1
  rc=$?; echo "fc1 $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_fc1 > $R/gpurun_out/pmc_fc1/summary.json || exit 1
cat $R/gpurun_out/pmc_fc1/summary.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_swin/$C -o run \
    -- python3 $R/bench.py --model swin_tiny --batch 256 --steps 2 --warmup 1 --cpu-seconds 0 > $R/gpurun_out/pmc_swin/$C.log 2>&1
  rc=$?; echo "swin $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
