#!/bin/bash
# Row-layout residual epilogue: parity (GEMM / model / Swin tests), A/B vs the MFMA-layout
# epilogue (variant 26) on the residual GEMM shapes, then the headline bench.
set -u
mkdir -p gpurun_out/rows
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "dense or model or vit or gemm or swin or streamk or pers" > gpurun_out/rows/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/rows/pytest.log; [ $rc -eq 0 ] || exit $rc
GS=768x768@197,3072x768@197,768x768@133,3072x768@133 timeout -k 10 300 python scripts/gemm_bench.py 100864 0,26,20,17 > gpurun_out/rows/gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/rows/gemm.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 > gpurun_out/rows/bench_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/rows/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['per_role_us'])"
done
