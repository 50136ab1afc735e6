#!/bin/bash
# Round-4 baseline: headline bench, bs64 (strong-scaling per-GPU share) bench and its kernel stats.
set -u
O=gpurun_out/${TAG:-r4base}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench_deit_base.jsonl 2>&1 || exit 1
tail -1 $O/bench_deit_base.jsonl | cut -c1-300
timeout -k 10 300 python bench.py --cpu-seconds 0 --batch 64 --steps 50 > $O/bench_deit_base_bs64.jsonl 2>&1 || exit 1
tail -1 $O/bench_deit_base_bs64.jsonl | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof64 -o run \
  -- python3 $R/bench.py --cpu-seconds 0 --batch 64 --steps 50 > $O/bench_bs64_prof.jsonl 2>&1 || exit 1
find $R/$O/prof64 -name "*kernel_stats*" -exec cp {} $R/$O/deit_base_bs64_kernel_stats.csv \;
python3 scripts/kstats.py $O/deit_base_bs64_kernel_stats.csv 64 | head -14
