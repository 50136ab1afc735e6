set -u
export PYTHONDONTWRITEBYTECODE=1
for E in 0 777 778 779; do
EPS=$E GS=qkv,fc1,64x3072@1 timeout -k 10 300 python scripts/gemm_bench.py 100864 40 > gpurun_out/gb_$E.log 2>&1 || exit 1; echo "EPS $E"; grep -v amdgpu.ids gpurun_out/gb_$E.log
done
