#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
for v in 0 1 6; do
  TAG=swin_v$v BENCH_ARGS="--model swin_tiny --batch 256 --gemm-variant $v" bash scripts/gpu_prof.sh || exit 1
done
