#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (per-kernel durations).
#   TAG=<name> BENCH_ARGS="--model swin_tiny --batch 256" bash scripts/gpu_prof.sh
set -u
TAG=${TAG:-run}
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run \
  -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > $R/gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?; echo "rocprof $TAG rc=$rc"; tail -1 $R/gpurun_out/prof_$TAG/bench.log
find $R/gpurun_out/prof_$TAG -name "*kernel_stats*" -exec cp {} $R/gpurun_out/prof_$TAG/kernel_stats.csv \;
exit $rc
