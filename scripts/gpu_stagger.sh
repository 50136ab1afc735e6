#!/bin/bash
# Late start of the blocks that have one tile fewer (variants 21-24: 1/4 .. 1 tile), isolated
# GEMMs (interleaved in one process) and in the model (bench per-role times).
set -u
mkdir -p gpurun_out/stag
export PYTHONDONTWRITEBYTECODE=1
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,21,22,23,24 > gpurun_out/stag/gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stag/gemm.log
for v in 0 22 24 0; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --gemm-variant $v > gpurun_out/stag/b_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/stag/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
