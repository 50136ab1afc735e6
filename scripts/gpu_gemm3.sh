#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
GS=${GS:-768x2304@33,768x768@197,768x3072@35,3072x768@197} timeout -k 10 300 python scripts/gemm_bench.py 100864 ${VARS:-9} > gpurun_out/gemm_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/gemm_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-probe > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-250
