#!/bin/bash
# Re-run of the residual / stagger ablations with the variant actually applied (the library used
# to reject 20-25 silently in gemm_bench): 0 full, 20 no residual loads,
# 11 no stores, 17 no epilogue; then the timeline (variant 13).
set -u
mkdir -p gpurun_out/ablate
export PYTHONDONTWRITEBYTECODE=1
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,20,11,17 > gpurun_out/ablate/abl3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ablate/abl3.log
GS=768x768@197,3072x768@197 timeout -k 10 200 python scripts/probe/pers_timeline.py > gpurun_out/ablate/tl25.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ablate/tl25.log
