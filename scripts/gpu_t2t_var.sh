#!/bin/bash
# T2T-ViT-14 bs256: per-role GEMM times under each GEMM kernel choice (0 auto, 1 128x128 tiles,
# 2 256x256 non-persistent, 9 persistent forced)
set -u
mkdir -p gpurun_out/t2tv
export PYTHONDONTWRITEBYTECODE=1
for v in 0 1 2 9 0; do
  timeout -k 10 200 python bench.py --model t2t_vit_14 --batch 256 --cpu-seconds 0 --gemm-variant $v > gpurun_out/t2tv/b_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/t2tv/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], d['ms_per_step'], d['roofline'].get('per_role_us'))"
done
