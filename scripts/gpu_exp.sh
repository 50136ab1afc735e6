set -u
export PYTHONDONTWRITEBYTECODE=1
#timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "dense" > gpurun_out/pytest_dense.log 2>&1
#rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || exit $rc
TV=13 timeout -k 10 300 python scripts/probe/pers_timeline.py > gpurun_out/timeline.log 2>&1
rc=$?; echo "timeline rc=$rc"; grep -v amdgpu.ids gpurun_out/timeline.log; [ $rc -eq 0 ] || exit $rc
GS=768x3072@35,768x2304@33,768x768@197,3072x768@197 timeout -k 10 300 python scripts/gemm_bench.py 100864 6,9 > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.log; exit $rc
