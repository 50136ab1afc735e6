#!/bin/bash
# Residual prefetch (variant 28) vs default on the residual GEMM shapes, + parity of variant 28.
set -u
mkdir -p gpurun_out/pf
export PYTHONDONTWRITEBYTECODE=1
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,30,20 > gpurun_out/pf/gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pf/gemm.log
