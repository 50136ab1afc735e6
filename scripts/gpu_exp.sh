set -u
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_streamk.py > gpurun_out/pytest_sk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sk.log; [ $rc -eq 0 ] || exit $rc
GS=${GS:-768x2304@33,768x768@197,768x3072@35,3072x768@197} timeout -k 10 300 python scripts/gemm_bench.py 100864 ${VARS:-9,16} > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.log; exit $rc
