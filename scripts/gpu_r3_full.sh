#!/bin/bash
# Round-3: the full-size BASELINE-config tests, then the whole GPU suite and smoke (tightened gates).
set -u
O=gpurun_out/r3full
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py > $O/pytest_full.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|max-abs|diff|passed|failed" $O/pytest_full.log | head -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
grep -v amdgpu.ids $O/smoke.log; exit $rc
