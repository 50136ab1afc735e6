#!/bin/bash
# Fused QKV + attention kernel: parity tests, then ablations (EVT_QA_DBG 0 full, 1 no attention,
# 2 main loop only) in the microbenchmark, then the headline bench fused / unfused.
set -u
mkdir -p gpurun_out/qa
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/qa
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qkv_attn.py > $O/pytest_qa.log 2>&1
rc=$?; tail -2 $O/pytest_qa.log; [ $rc -eq 0 ] || exit $rc
for d in 0 1 2; do
  EVT_QA_DBG=$d UNFUSED=$([ $d = 0 ] && echo 1 || echo 0) timeout -k 10 120 python scripts/qa_bench.py > $O/qa_$d.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/qa_$d.log
done
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-probe --fusion 1 > $O/bench_fused.log 2>&1 || exit 1
echo "fused $(grep -o '"value": [0-9.]*' $O/bench_fused.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-probe > $O/bench_unfused.log 2>&1 || exit 1
echo "unfused $(grep -o '"value": [0-9.]*' $O/bench_unfused.log)"
fi
