#!/bin/bash
# Product library (full GPU suite + smoke) against a lab library built with EVT_LAB_DEFS, in
# alternating same-box bench pairs on DeiT-base bs512 and then on each EXTRA config:
#   TAG=x PAIRS=3 EXTRA="--model deit_tiny --batch 256 --dtype f32" bash scripts/gpu_lab_ab.sh
set -u
T=${TAG:-labab}
O=gpurun_out/$T
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
grep -v amdgpu.ids $O/smoke.log
TAG=$T/base PAIRS=${PAIRS:-3} LIBS="product libevt_hip_lab.so" ARGS="" bash scripts/gpu_libab.sh || exit 1
if [ -n "${EXTRA:-}" ]; then
  IFS=';' read -ra CFGS <<< "$EXTRA"
  i=0
  for c in "${CFGS[@]}"; do
    i=$((i + 1))
    echo "== $c"
    TAG=$T/extra$i PAIRS=${EPAIRS:-2} LIBS="product libevt_hip_lab.so" ARGS="$c" bash scripts/gpu_libab.sh || exit 1
  done
fi
