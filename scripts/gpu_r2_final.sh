#!/bin/bash
# Round-2 records at HEAD: every GPU test, smoke(), the headline bench (with the CPU baseline),
# rocprofv3 kernel stats of the same bench command, FC1 PMC traffic (FETCH_SIZE / WRITE_SIZE
# passes), and the other BASELINE configs' benches (T2T-ViT-14 bs256, Swin-T bs256, DeiT-tiny f32).
set -u
O=gpurun_out/r2v5
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
grep smoke $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['model_roofline'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['per_role_us'], d['cpu_baseline']['value'])"
TAG=r2v5_bench BENCH_ARGS="--cpu-seconds 0" STEPS=10 bash scripts/gpu_prof.sh > /dev/null 2>&1 || exit 1
grep '^{' gpurun_out/prof_r2v5_bench/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof: fc1', d['roofline']['avg_launch_us'])"
python scripts/kstats.py gpurun_out/prof_r2v5_bench/kernel_stats.csv 512 > $O/kstats.txt; head -10 $O/kstats.txt
bash scripts/gpu_pmc_fc1.sh > $O/pmc.log 2>&1 || exit 1
tail -3 $O/pmc.log
for cfg in "--model t2t_vit_14 --batch 256" "--model swin_tiny --batch 256" "--model deit_tiny --batch 256 --dtype f32"; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 $cfg > $O/b.log 2>&1 || exit 1
  tail -1 $O/b.log >> $O/other_benches.jsonl
  tail -1 $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'], d['value'], d['ms_per_step'])"
done
