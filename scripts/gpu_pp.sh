#!/bin/bash
# Dense-kernel parity for all variants, then the GEMM microbench (variants in GV).
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "dense" > gpurun_out/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || exit $rc
GS=${GS:-qkv,out,fc1,fc2} timeout -k 10 300 python scripts/gemm_bench.py ${GM:-100864} ${GV:-6,8} > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.log
exit $rc
