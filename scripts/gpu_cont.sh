#!/bin/bash
# Next-tile prologue in the last K-tiles' DMA slots (default) vs after the main loop (variant 21):
# GEMM / model parity, the four DeiT-base shapes interleaved, the headline bench.
set -u
mkdir -p gpurun_out/cont
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "dense and not patch" > gpurun_out/cont/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/cont/pytest.log; [ $rc -eq 0 ] || exit $rc
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,24 > gpurun_out/cont/gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/cont/gemm.log
for v in 0 24 0 24; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --gemm-variant $v > gpurun_out/cont/b_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/cont/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
