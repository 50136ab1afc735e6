#!/bin/bash
# Channel-major patchify: op + model parity, then kernel stats of the forward (patch GEMM VAR 6
# default vs VAR 8 via --gemm-variant 8, which also moves the encoder GEMMs off the persistent
# kernel: compare only the patch-GEMM rows)
set -u
mkdir -p gpurun_out/patch
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "patchify or model or vit or profile" > gpurun_out/patch/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/patch/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 8; do
  TAG=patch_v$v BENCH_ARGS="--cpu-seconds 0 --gemm-variant $v" STEPS=5 bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
  echo "variant $v: $(grep -o '"value": [0-9.]*' gpurun_out/prof_patch_v$v/bench.log)"
  python scripts/kstats.py gpurun_out/prof_patch_v$v/kernel_stats.csv 512 > gpurun_out/patch/k_$v.txt
  grep -E "patchify|<137|gemm_nt" gpurun_out/patch/k_$v.txt
done
