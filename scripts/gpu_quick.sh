#!/bin/bash
# parity tests of the GEMM / model paths, then DeiT-base and Swin-T benches
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-250
TAG=swin BENCH_ARGS="--model swin_tiny --batch 256" bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
tail -1 gpurun_out/prof_swin/bench.log | cut -c1-200
python scripts/swin_seq.py gpurun_out/prof_swin/run_kernel_trace.csv
