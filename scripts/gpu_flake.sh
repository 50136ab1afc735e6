#!/bin/bash
# Wrong-result probe of the residual-LayerNorm GEMM (each launch against the fp32 reference),
# then the headline bench.
set -u
mkdir -p gpurun_out/flake
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u scripts/probe/resln_flake.py ${REPS:-40} > gpurun_out/flake/probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/flake/probe.log
for v in 0 25 0 25; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --gemm-variant $v > gpurun_out/flake/b_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/flake/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
