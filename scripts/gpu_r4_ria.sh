#!/bin/bash
# Buffer-descriptor DMA + residual added by the main loop (product) against variant 33 (the
# epilogue residual) and the lab build -DEVT_BDMA=0 at variant 33 (the round-3 kernels), in
# alternating same-box runs; GPU suite on the product library first (TESTS).
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-ria}
mkdir -p $O
D=$GRAFT_REPO_ROOT/edgevisiontransformer_amd
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS -m gpu > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
summ() {
  tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], {k: v['us_per_launch'] for k, v in d['roofline']['per_role'].items()})"
}
IFS=';' read -ra CFGS <<< "${CFG:---model deit_base}"
for c in "${CFGS[@]}"; do
  echo "== $c"
  for i in $(seq ${PAIRS:-3}); do
    EVT_LIB=$D/libevt_hip.so timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe $c > $O/a_$i.log 2>&1 || exit 1
    summ $O/a_$i.log product
    EVT_LIB=$D/libevt_hip.so timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe $c --gemm-variant 33 > $O/b_$i.log 2>&1 || exit 1
    summ $O/b_$i.log v33
    EVT_LIB=$D/libevt_hip_lab.so timeout -k 10 300 python bench.py --cpu-seconds 0 --no-probe $c --gemm-variant 33 > $O/c_$i.log 2>&1 || exit 1
    summ $O/c_$i.log lab_glds_v33
  done
done
