#!/bin/bash
# Kernel times of the DeiT-base forward at bs 512 / 256 / 128 (does a layer's working set that
# fits the 256 MB Infinity Cache change the per-image kernel time?)
set -u
export PYTHONDONTWRITEBYTECODE=1
for b in 512 256 128; do
  TAG=b$b BENCH_ARGS="--batch $b --no-probe" STEPS=10 bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
  echo "bs $b"; tail -1 gpurun_out/prof_b$b/bench.log | cut -c100-200
  head -6 gpurun_out/prof_b$b/kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
done
