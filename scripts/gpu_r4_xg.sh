#!/bin/bash
# XCD groups of the persistent walk (gemm.hip pers_tile): variant 34 = one group (round-3 order),
# 0 = default (2 groups where the panels divide), 35 = 4 groups. DeiT-base bs512: per-launch
# durations of the GEMM roles (kernel trace, alternating), FETCH_SIZE of FC1 per variant, bench lines.
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-xg}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fullsize.py tests/test_gpu_model.py -m gpu > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for v in ${VARS:-34 0 35}; do
    rm -rf $O/kt_$v
    timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o run \
      -- python3 $R/bench.py ${ARGS:-} --gemm-variant $v --cpu-seconds 0 --no-probe --steps 3 --warmup 1 > $O/kt_$v.log 2>&1 || exit 1
    python3 - "$O/kt_$v" "$v" <<'PY'
import csv, glob, collections, sys
O, v = sys.argv[1], sys.argv[2]
by = collections.defaultdict(list)
for f in glob.glob(f"{O}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm_pers_kernel<" in n:
            by[n.split("gemm_pers_kernel<")[1].split(",")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("variant", v, "  ".join(f"<{k}> n {len(x)} med {sorted(x)[len(x)//2]:.1f}" for k, x in sorted(by.items())))
PY
  done
done
for v in ${VARS:-34 0 35}; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run \
    -- python3 $R/bench.py ${ARGS:-} --gemm-variant $v --cpu-seconds 0 --no-probe --steps 2 --warmup 1 > $O/pmc_$v.log 2>&1 || exit 1
  python3 - "$O/pmc_$v" "$v" <<'PY'
import csv, glob, collections, sys
O, v = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{O}/**/*counter_collection.csv", recursive=True):
    d = collections.defaultdict(float); name = {}
    for r in csv.DictReader(open(f)):
        d[int(r["Dispatch_Id"])] += float(r["Counter_Value"]); name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    for k, x in d.items():
        if "gemm_pers_kernel<" in name[k]:
            agg[name[k].split("gemm_pers_kernel<")[1].split(",")[0]].append(x * 2 * 1024 / 1e6)
print("variant", v, "FETCH MB per launch (x2 gfx950):", "  ".join(f"<{k}> {sorted(x)[len(x)//2]:.0f}" for k, x in sorted(agg.items())))
PY
done
for v in ${VARS:-34 0}; do
  timeout -k 10 300 python bench.py ${ARGS:-} --gemm-variant $v --cpu-seconds 0 --no-probe > $O/bench_$v.jsonl 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench variant', sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_$v.jsonl $v
done
