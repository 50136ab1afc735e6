#!/bin/bash
# Round 2, first GPU call: full GPU suite, headline bench, vendor-GEMM calibration of the four
# DeiT-base bs512 GEMM shapes (hipBLASLt through torch.matmul beside our kernel), kernel trace.
set -u
mkdir -p gpurun_out/r2a
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2a
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-300
GS=qkv,out,fc1,fc2 TORCHMM=1 timeout -k 10 300 python scripts/gemm_bench.py 100864 0 > $O/gemm_torch.log 2>&1 || exit 1
cat $O/gemm_torch.log
TAG=r2a_deit bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
head -8 gpurun_out/prof_r2a_deit/kernel_stats.csv | cut -c1-160
