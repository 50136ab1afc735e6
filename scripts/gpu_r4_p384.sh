#!/bin/bash
# 128 x 384 tiles: GPU suite, then A/B benches (variant 0 = automatic incl. 128 x 384, 31 = without).
set -u
O=gpurun_out/${TAG:-r4p384}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${SEL:-tests} -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
b() { timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe "$@" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' '.join(sys.argv[1:]), d['value'], d['ms_per_step'])" "$@"; }
for i in 1 2; do
  b --model t2t_vit_14 --batch 256 --gemm-variant 31 || exit 1
  b --model t2t_vit_14 --batch 256 || exit 1
  b --model deit_base --batch 64 --steps 50 --gemm-variant 31 || exit 1
  b --model deit_base --batch 64 --steps 50 || exit 1
  b --model swin_tiny --batch 256 --gemm-variant 31 || exit 1
  b --model swin_tiny --batch 256 || exit 1
  b --model deit_small --batch 512 --gemm-variant 31 || exit 1
  b --model deit_small --batch 512 || exit 1
done
b --model deit_base --batch 512 || exit 1
