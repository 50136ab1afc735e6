#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_t2t.py > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/attn_bench.py >> gpurun_out/attn_bench.log 2>&1 || exit 1
grep attn_us gpurun_out/attn_bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-300
