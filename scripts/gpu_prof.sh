#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (per-kernel durations).
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run \
  -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 2 --cpu-seconds 0 > $R/gpurun_out/prof/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $R/gpurun_out/prof/bench.log
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
