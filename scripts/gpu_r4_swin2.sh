#!/bin/bash
# Swin window attention: the GPU tests of the Swin path, then per-launch durations of the kernel
# (kernel trace, 2 runs) and a Swin-T bs256 bench line.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-swin2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_swin.py tests/test_gpu_ops.py tests/test_gpu_fullsize.py tests/test_gpu_repeat_launch.py -m gpu -k "swin or window" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-swin2}_kt KNAME=${KN:-window_attn_bf16} ARGS="--model swin_tiny --batch 256" PAIRS=2 LIBS=product bash scripts/gpu_r4_kt.sh || exit 1
timeout -k 10 300 python bench.py --model swin_tiny --batch 256 --cpu-seconds 0 > $O/bench.jsonl 2>&1 || exit 1
tail -1 $O/bench.jsonl | cut -c1-100
