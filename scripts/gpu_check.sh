#!/bin/bash
# One GPU session: parity tests, smoke, short bench. Stops at the first crash-like exit status
# (fault/abort/segfault/timeout); ordinary test failures (pytest rc 1) do not stop the bench.
set -u
mkdir -p gpurun_out
ok_or_stop() {  # $1 = rc, $2 = step
  case "$1" in
    0|1) return 0 ;;
    *) echo "STOP: $2 exited with $1" | tee -a gpurun_out/status.log; exit "$1" ;;
  esac
}
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x --timeout=300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; ok_or_stop $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log; ok_or_stop $rc smoke
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 --cpu-seconds ${CPUS:-15} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; ok_or_stop $rc bench
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log; tail -2 gpurun_out/bench.log
