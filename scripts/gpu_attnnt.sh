#!/bin/bash
# Experiment: attention qkv loads / O stores with the non-temporal cache policy (EVT_ATTN_NT=1),
# in the model: does the out-proj residual (x, read by QKV before) stay in the Infinity Cache?
set -u
mkdir -p gpurun_out/attnnt
export PYTHONDONTWRITEBYTECODE=1
for nt in 0 5 0 5 3; do
  EVT_ATTN_NT=$nt timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/attnnt/b_$nt.log 2>&1 || exit 1
  tail -1 gpurun_out/attnnt/b_$nt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($nt, d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
