#!/bin/bash
# Round records: GPU parity suite, smoke, the headline bench, rocprof kernel stats of DeiT-base and
# Swin-T, and one bench line per BASELINE config. Every GPU step has its own time limit.
set -u
mkdir -p gpurun_out/rec
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/rec
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_deit_base.log 2>&1 || exit 1
tail -1 $O/bench_deit_base.log | cut -c1-200
TAG=deit bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
TAG=swin BENCH_ARGS="--model swin_tiny --batch 256" bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
timeout -k 10 300 python bench.py --model swin_tiny --batch 256 --steps 20 --cpu-seconds 10 > $O/bench_swin_t.log 2>&1 || exit 1
tail -1 $O/bench_swin_t.log | cut -c1-200
timeout -k 10 300 python bench.py --model t2t_vit_14 --batch 256 --steps 20 --cpu-seconds 10 > $O/bench_t2t14.log 2>&1 || exit 1
tail -1 $O/bench_t2t14.log | cut -c1-200
timeout -k 10 300 python bench.py --model deit_tiny --dtype f32 --batch 256 --steps 10 --cpu-seconds 5 --no-probe > $O/bench_tiny_f32.log 2>&1 || exit 1
tail -1 $O/bench_tiny_f32.log | cut -c1-200
