#!/bin/bash
# GPU suite, then the epilogue A/B (0 = current, 19 = round-1 epilogue, 17 = no epilogue) on the
# model's four GEMM flag sets, interleaved in one process, then the headline bench.
set -u
mkdir -p gpurun_out/r2c
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2c
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
GS=768x2304@33,768x768@197,768x3072@35,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,19,17 > $O/ablate.log 2>&1 || exit 1
cat $O/ablate.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-400
