#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_gpu_t2t.py -q -m gpu -x > gpurun_out/pytest_t2t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_t2t.log; exit $rc
