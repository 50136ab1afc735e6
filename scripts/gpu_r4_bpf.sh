#!/bin/bash
# Phase-3 B-fragment prefetch (EVT_BPF=1, product) vs the round-3 schedule (lab, -DEVT_BPF=0):
# GPU suite on the product library, then alternating same-box bench pairs.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-bpf}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS -m gpu > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra CFGS <<< "${CFG:---model deit_base}"
i=0
for c in "${CFGS[@]}"; do
  i=$((i + 1))
  echo "== $c"
  TAG=${TAG:-bpf}/c$i PAIRS=${PAIRS:-3} LIBS="product libevt_hip_lab.so" ARGS="$c" bash scripts/gpu_libab.sh || exit 1
done
