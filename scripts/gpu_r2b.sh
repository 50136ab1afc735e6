#!/bin/bash
# GEMM ablations on the model's four flag sets (full / no epilogue / no GELU / no stores) + FC1 SQ counters
set -u
mkdir -p gpurun_out/r2b
export PYTHONDONTWRITEBYTECODE=1
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,17,18,11 > gpurun_out/r2b/ablate.log 2>&1 || exit 1
cat gpurun_out/r2b/ablate.log
bash scripts/gpu_pmc_sq.sh 2>&1 | tail -40
