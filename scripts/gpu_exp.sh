set -u
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu -k "attention or golden or batch" > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-probe > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-150; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh > /dev/null 2>&1; python3 - <<'PY'
import csv, collections
rows=list(csv.DictReader(open('gpurun_out/prof/run_kernel_trace.csv')))
d=collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name'][:60]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(d.items(), key=lambda kv:-sum(kv[1])):
    if len(v)<5: continue
    v=sorted(v); print(f"{k:60s} n={len(v)} med={v[len(v)//2]:.1f}")
PY
