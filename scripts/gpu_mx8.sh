#!/bin/bash
# MXFP8 kernel parity tests, then the MX8 vs bf16 GEMM timing on the DeiT-base shapes
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mx8.py -m gpu > gpurun_out/pytest_mx8.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_mx8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/mx8_bench.py > gpurun_out/mx8_bench.log 2>&1; rc=$?
cat gpurun_out/mx8_bench.log; exit $rc
