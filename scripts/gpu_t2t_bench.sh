#!/bin/bash
# T2T-ViT-14 bs256 bench + rocprof kernel stats.
set -u
mkdir -p gpurun_out/prof_t2t
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --model t2t_vit_14 --batch 256 --steps 20 --warmup 5 --cpu-seconds ${CPUS:-0} > gpurun_out/bench_t2t.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_t2t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_t2t -o run \
  -- python3 $R/bench.py --model t2t_vit_14 --batch 256 --steps 5 --warmup 2 --cpu-seconds 0 --no-probe > $R/gpurun_out/prof_t2t/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
