#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -x -k dense > gpurun_out/pytest_dense.log 2>&1
rc=$?; echo "pytest dense rc=$rc"; tail -3 gpurun_out/pytest_dense.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/gemm_bench.py ${GM:-100864} ${GV:-1,2,3} > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gemm_bench.log | grep -v amdgpu.ids
exit $rc
