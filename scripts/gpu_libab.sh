#!/bin/bash
# Alternating same-box A/B of the product library against lab libraries built with EVT_LAB_DEFS
# (LIBS: names under edgevisiontransformer_amd/, "product" = libevt_hip.so):
#   PAIRS=3 LIBS="product libevt_hip_lab.so" ARGS="--model deit_base" TESTS=tests PROBE=scripts/probe/std_err.py \
#     bash scripts/gpu_libab.sh
# TESTS / PROBE run against every non-product library (the probe against the product one too).
set -u
O=gpurun_out/${TAG:-libab}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
D=$GRAFT_REPO_ROOT/edgevisiontransformer_amd
LIBS=${LIBS:-product libevt_hip_lab.so}
libenv() { if [ "$1" = product ]; then echo "EVT_LIB=$D/libevt_hip.so"; else echo "EVT_LIB=$D/$1"; fi; }
for l in $LIBS; do
  if [ -n "${PROBE:-}" ]; then
    env $(libenv $l) timeout -k 10 300 python $PROBE > $O/probe_$l.log 2>&1 || { tail -20 $O/probe_$l.log; exit 1; }
    cat $O/probe_$l.log
  fi
  if [ -n "${TESTS:-}" ] && [ "$l" != product ]; then
    env $(libenv $l) timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      -m gpu $TESTS > $O/tests_$l.log 2>&1 || { tail -30 $O/tests_$l.log; exit 1; }
    echo "$l: $(tail -1 $O/tests_$l.log)"
  fi
done
summ() {
  tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], {k: v['us_per_launch'] for k, v in d['roofline']['per_role'].items()})"
}
for i in $(seq ${PAIRS:-3}); do
  for l in $LIBS; do
    env $(libenv $l) timeout -k 10 300 python bench.py --cpu-seconds 0 ${ARGS:-} > $O/b_${l}_$i.log 2>&1 || exit 1
    summ $O/b_${l}_$i.log $l
  done
done
