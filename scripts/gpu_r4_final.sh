#!/bin/bash
# Round-4 records at one commit: full GPU suite, smoke, the driver-style headline bench line,
# rocprofv3 kernel stats of the same bench command, the bs64 (strong-scaling share) line and its
# kernel stats, the other BASELINE configs with their CPU baselines, and the final window-attention
# counters. Every GPU step has its own time limit; the script stops at the first failure.
set -u
O=gpurun_out/${TAG:-r4final}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline'] or {}; print(d['config'].get('model', d['config'].get('workload')), d['value'], d['ms_per_step'], 'model', d['model_roofline']['frac'], 'dom', r.get('role'), r.get('frac'), 'traffic', r.get('traffic'), 'cpu', (d['cpu_baseline'] or {}).get('value'))" $1; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
  rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/smoke.log | tail -3
fi
timeout -k 10 300 python bench.py > $O/bench_deit_base.jsonl 2>&1 || exit 1
summ $O/bench_deit_base.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run \
  -- python3 $R/bench.py --cpu-seconds 0 > $O/bench_deit_base_under_rocprof.jsonl 2>&1 || exit 1
find $R/$O/prof -name "*kernel_stats*" -exec cp {} $R/$O/deit_base_kernel_stats.csv \;
python3 scripts/kstats.py $O/deit_base_kernel_stats.csv 512 > $O/deit_base_kstats.txt; head -10 $O/deit_base_kstats.txt
timeout -k 10 300 python bench.py --batch 64 --steps 50 --cpu-seconds 0 > $O/bench_deit_base_bs64.jsonl 2>&1 || exit 1
summ $O/bench_deit_base_bs64.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof64 -o run \
  -- python3 $R/bench.py --batch 64 --steps 50 --cpu-seconds 0 --no-probe > $O/bench_bs64_under_rocprof.jsonl 2>&1 || exit 1
find $R/$O/prof64 -name "*kernel_stats*" -exec cp {} $R/$O/deit_base_bs64_kernel_stats.csv \;
python3 scripts/kstats.py $O/deit_base_bs64_kernel_stats.csv 64 > $O/deit_base_bs64_kstats.txt; head -8 $O/deit_base_bs64_kstats.txt
for cfg in "t2t_vit_14 --batch 256" "swin_tiny --batch 256" "deit_tiny --batch 256 --dtype f32"; do
  n=$(echo $cfg | cut -d' ' -f1)
  timeout -k 10 400 python bench.py --model $cfg --cpu-seconds 10 > $O/bench_$n.jsonl 2>&1 || exit 1
  summ $O/bench_$n.jsonl
done
TAG=${TAG:-r4final}_swinwa KNAME=window_attn_bf16_kernel ARGS="--model swin_tiny --batch 256" bash scripts/gpu_pmc_kernel.sh > $O/swinwa_pmc.log 2>&1 || exit 1
grep grid $O/swinwa_pmc.log
