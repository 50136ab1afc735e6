#!/bin/bash
# In-process-equivalent A/B of GEMM variants on one box with the lab library:
#   VARIANTS="0 26 0 26" ARGS="--model deit_base" bash scripts/gpu_ab.sh
set -u
O=gpurun_out/${TAG:-ab}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 EVT_LIB=$GRAFT_REPO_ROOT/edgevisiontransformer_amd/libevt_hip_lab.so
for v in ${VARIANTS:-0 26}; do
  timeout -k 10 300 python bench.py --gemm-variant $v --cpu-seconds 0 ${ARGS:-} > $O/b_$v.log 2>&1 || exit 1
  tail -1 $O/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], {k: v['us_per_launch'] for k, v in d['roofline']['per_role'].items()})"
done
