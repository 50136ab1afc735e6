#!/bin/bash
# Round-3 records at one commit (pass COMMIT=<hash>): full GPU suite, smoke, headline bench
# (per-role MFMA + HBM roofline fractions), rocprofv3 kernel stats of the same bench command, the
# FC1 PMC traffic pass, and the other BASELINE configs with their CPU baselines.
set -u
O=gpurun_out/${TAG:-r3rec}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline'] or {}; print(d['config']['model'], d['value'], d['ms_per_step'], 'model', d['model_roofline']['frac'], 'dom', r.get('role'), r.get('frac'), 'hbm', r.get('hbm_frac'), 'cpu', (d['cpu_baseline'] or {}).get('value')); [print('  ', k, v) for k, v in (r.get('per_role') or {}).items()]" $1; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
  rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/smoke.log
fi
timeout -k 10 300 python bench.py > $O/bench_deit_base.jsonl 2>&1 || exit 1
summ $O/bench_deit_base.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run \
  -- python3 $R/bench.py --cpu-seconds 0 > $O/bench_deit_base_prof.jsonl 2>&1 || exit 1
find $R/$O/prof -name "*kernel_stats*" -exec cp {} $R/$O/deit_base_kernel_stats.csv \;
summ $O/bench_deit_base_prof.jsonl
python3 scripts/kstats.py $O/deit_base_kernel_stats.csv 512 | head -12
mkdir -p $O/pmc_fc1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/$O/pmc_fc1/$C -o run \
    -- python3 $R/bench.py --probe-only 10 > $R/$O/pmc_fc1/$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_summary.py $R/$O/pmc_fc1 > $O/pmc_fc1.json || exit 1
grep -E "traffic|commit" $O/pmc_fc1.json
for cfg in "deit_tiny --batch 256 --dtype f32" "t2t_vit_14 --batch 256" "swin_tiny --batch 256"; do
  n=$(echo $cfg | cut -d' ' -f1)
  timeout -k 10 400 python bench.py --model $cfg --cpu-seconds 10 > $O/bench_$n.jsonl 2>&1 || exit 1
  summ $O/bench_$n.jsonl
done
