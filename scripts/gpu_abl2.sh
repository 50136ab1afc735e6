#!/bin/bash
# Residual-load ablation of the RESID persistent GEMMs (out-proj / FC2 shapes): 0 full, 20 no
# residual loads, 11 no stores, 17 no epilogue.
set -u
mkdir -p gpurun_out/ablate
export PYTHONDONTWRITEBYTECODE=1
GS=768x768@197,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,20,11,17 > gpurun_out/ablate/abl2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ablate/abl2.log
