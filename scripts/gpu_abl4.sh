#!/bin/bash
# 0 (row-layout residual epilogue), 27 (next-tile prologue after the epilogue), 20 (no residual
# loads), 17 (no epilogue) on all four DeiT-base shapes.
set -u
mkdir -p gpurun_out/ablate
export PYTHONDONTWRITEBYTECODE=1
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,27,20,17 > gpurun_out/ablate/abl4.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ablate/abl4.log
