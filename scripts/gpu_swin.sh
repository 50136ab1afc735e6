#!/bin/bash
# Swin GPU check: parity tests, then a short bench of Swin-T bs256 (per-GPU share of bs2048 / 8).
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_swin.py > gpurun_out/pytest_swin.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_swin.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model swin_tiny --batch 256 --steps 10 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_swin.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_swin.log; exit $rc
