#!/bin/bash
# Swin window attention: GPU tests of the Swin path, then per-launch durations + counters of the
# kernel (gpu_pmc_kernel.sh) and bench lines of Swin-T bs256.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-swin}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_swin.py tests/test_gpu_ops.py tests/test_gpu_fullsize.py -m gpu -k "swin or window" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-swin}_pmc KNAME=window_attn_bf16_kernel ARGS="--model swin_tiny --batch 256" bash scripts/gpu_pmc_kernel.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
grep -E "grid|VALU|WAVE_CYCLES|WAIT|FETCH_BYTES|WRITE_BYTES" $O/pmc.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model swin_tiny --batch 256 --cpu-seconds 0 > $O/bench_$i.jsonl 2>&1 || exit 1
  tail -1 $O/bench_$i.jsonl | cut -c1-120
done
