#!/bin/bash
# Round-3 baseline at HEAD: full GPU suite, smoke, headline bench.
set -u
O=gpurun_out/r3base
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log
