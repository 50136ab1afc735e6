#!/bin/bash
# DeiT-base bs64 (the strong-scaling per-GPU share): bench lines at fusion flags 0..3, alternated.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-bs64}
mkdir -p $O
for i in 1 2; do
  for f in ${FUS:-0 2 1 3}; do
    timeout -k 10 240 python bench.py --batch 64 --steps 50 --warmup 5 --cpu-seconds 0 --no-probe --fusion $f > $O/f$f.$i.jsonl 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fusion', sys.argv[2], d['value'], d['ms_per_step'])" $O/f$f.$i.jsonl $f
  done
done
