#!/bin/bash
# T2T performer: the GPU tests of the T2T path, per-launch durations of the performer kernels
# (kernel trace, 2 runs) and a T2T-ViT-14 bs256 bench line.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-t2t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_t2t.py tests/test_gpu_ops.py tests/test_gpu_fullsize.py tests/test_gpu_repeat_launch.py -m gpu -k "t2t or performer or unfold" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-t2t}_kt KNAME=performer ARGS="--model t2t_vit_14 --batch 256" PAIRS=2 LIBS=product bash scripts/gpu_r4_kt.sh || exit 1
timeout -k 10 300 python bench.py --model t2t_vit_14 --batch 256 --cpu-seconds 0 > $O/bench.jsonl 2>&1 || exit 1
tail -1 $O/bench.jsonl | cut -c1-100
