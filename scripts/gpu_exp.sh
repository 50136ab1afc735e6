set -u
export PYTHONDONTWRITEBYTECODE=1
B="timeout -k 10 200 python scripts/gemm_bench.py"
for M in 25216 50432; do
GS=64x3072@1,768x3072@1,768x2304@1 $B $M 6 > gpurun_out/e15.log 2>&1 || exit 1; echo M=$M; grep -v amdgpu gpurun_out/e15.log
LDC0=1 GS=64x3072@1,768x3072@1,768x2304@1 $B $M 6 > gpurun_out/e16.log 2>&1 || exit 1; echo M=$M LDC0; grep -v amdgpu gpurun_out/e16.log
done
