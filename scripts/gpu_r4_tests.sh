#!/bin/bash
# Full GPU suite + smoke (pass SEL="tests/x.py ..." to run a subset).
set -u
O=gpurun_out/${TAG:-r4tests}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${SEL:-tests} -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ -z "${SEL:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/smoke.log
fi
