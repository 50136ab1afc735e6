#!/bin/bash
# round 6 lab: DMA-latency ablation (EVT_ABL_KT0: every K-tile DMAs K-tile 0's bytes) vs the plain
# lab build, GEMM microbenchmark variants 0 (full) and 17 (no epilogue), DeiT-base bs512 shapes
set -u
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-kt0}; mkdir -p $O
for L in labn kt0; do
  EVT_LIB=edgevisiontransformer_amd/libevt_hip_$L.so GS=qkv,nt3072,nt768x3072 timeout -k 10 200 \
    python scripts/gemm_bench.py 100864 0,17 > $O/gemm_$L.txt 2>&1 || { tail -5 $O/gemm_$L.txt; exit 1; }
  echo "== $L"; grep -v amdgpu.ids $O/gemm_$L.txt
done
