#!/bin/bash
set -u
O=gpurun_out/${TAG:-r4exp1}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step']); r=d['roofline'] or {}; [print('  ', k, v['us_per_launch'], v['mfma_frac']) for k, v in (r.get('per_role') or {}).items()]" $1; }
timeout -k 10 200 python scripts/blas_ref.py 512 64 > $O/blas_ref.jsonl 2>&1 || exit 1
cat $O/blas_ref.jsonl
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench512.jsonl 2>&1 || exit 1
summ $O/bench512.jsonl
timeout -k 10 300 python bench.py --cpu-seconds 0 --batch 64 --steps 50 > $O/bench64.jsonl 2>&1 || exit 1
summ $O/bench64.jsonl
timeout -k 10 300 python bench.py --cpu-seconds 0 --batch 64 --steps 50 --gemm-variant 9 > $O/bench64_v9.jsonl 2>&1 || exit 1
summ $O/bench64_v9.jsonl
