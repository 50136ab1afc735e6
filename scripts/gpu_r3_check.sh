#!/bin/bash
# Round-3 check: new GPU tests first, then the whole GPU suite, smoke and the headline bench.
set -u
O=gpurun_out/${TAG:-r3check}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $FIRST > $O/pytest_first.log 2>&1
  rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_first.log | tail -20; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
grep -v amdgpu.ids $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-seconds 3 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['model_roofline']['frac'], {k: (v['us_per_launch'], v['mfma_frac'], v['hbm_frac']) for k, v in d['roofline']['per_role'].items()})"
