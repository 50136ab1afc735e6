#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
: > gpurun_out/swin_gemm.log
GS=192x576@33,192x192@133,192x768@289,768x192@133 timeout -k 10 200 python scripts/gemm_bench.py 200704 9,1,2 >> gpurun_out/swin_gemm.log 2>&1 || exit 1
GS=384x1152@33,384x384@133,384x1536@289,1536x384@133 timeout -k 10 200 python scripts/gemm_bench.py 50176 9,1,2 >> gpurun_out/swin_gemm.log 2>&1 || exit 1
GS=768x2304@33,768x768@133,768x3072@289,3072x768@133 timeout -k 10 200 python scripts/gemm_bench.py 12544 9,1,2 >> gpurun_out/swin_gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/swin_gemm.log
