#!/bin/bash
# Round 4: dequeued chained launch - chain tests, then alternating chain / no-chain benches.
set -u
O=gpurun_out/${TAG:-r4chain}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py > $O/chain_tests.log 2>&1
rc=$?; tail -12 $O/chain_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 2 0; do
    timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe --fusion $f > $O/bench_f${f}_$i.jsonl 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fusion', sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_f${f}_$i.jsonl $f
  done
done
