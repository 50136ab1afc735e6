#!/bin/bash
# Tile-rule A/B: automatic (cost rule, one block per tile below a round) vs variant 32 (round-3 rule)
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
b() { timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe "$@" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' '.join(sys.argv[1:]), d['value'], d['ms_per_step'])" "$@"; }
for i in 1 2; do
  for cfg in "deit_base --batch 64 --steps 50" "deit_base --batch 128 --steps 40" "swin_tiny --batch 256" "t2t_vit_14 --batch 256" "deit_base --batch 512"; do
    b --model $cfg --gemm-variant 32 || exit 1
    b --model $cfg || exit 1
  done
done
