#!/bin/bash
# Round-2 records: full GPU suite, smoke, headline bench (in-model FC1 roofline), and rocprofv3
# kernel stats of the SAME bench command (the FC1 average must agree with roofline.avg_launch_us).
set -u
mkdir -p gpurun_out/r2
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['model_roofline'], d['roofline'])"
TAG=r2_bench BENCH_ARGS="--cpu-seconds 0" STEPS=10 bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
tail -1 gpurun_out/prof_r2_bench/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof:', d['roofline']['avg_launch_us'])"
python scripts/kstats.py gpurun_out/prof_r2_bench/kernel_stats.csv 512 | head -8
