#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python scripts/gemm_bench.py ${GM:-100864} ${GV:-1,2,3} > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gemm_bench.log | grep -v amdgpu.ids
exit $rc
