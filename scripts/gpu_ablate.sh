#!/bin/bash
# Persistent-GEMM ablations on the model's four flag sets (0 full, 17 no epilogue, 18 no GELU,
# 11 no stores) interleaved in one process, then hipBLASLt (torch.matmul) on the plain shapes.
set -u
mkdir -p gpurun_out/ablate
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/ablate
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,17,18,11 > $O/ablate.log 2>&1 || exit 1
grep -v amdgpu.ids $O/ablate.log
GS=768x2304@0,768x768@0,768x3072@0,3072x768@0 TORCHMM=1 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,17 > $O/torch.log 2>&1 || exit 1
grep -v amdgpu.ids $O/torch.log
