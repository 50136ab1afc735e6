#!/bin/bash
# Iteration helper: GPU tests selected by $1 (pytest -k expression, "all" = every GPU test), then
# the headline bench without the CPU baseline: value, ms/step and per-role in-model times.
set -u
mkdir -p gpurun_out/try
export PYTHONDONTWRITEBYTECODE=1
K=${1:-all}
if [ "$K" = "all" ]; then SEL=(); else SEL=(-k "$K"); fi
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu "${SEL[@]}" > gpurun_out/try/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/try/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/try/bench_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/try/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
