#!/bin/bash
# MX8 vs bf16 in one process, and rocprofv3 kernel stats of the T2T-ViT-14 and Swin-T benches.
set -u
O=gpurun_out/${TAG:-r3other}
mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/mx8_model_bench.py > $O/mx8_model.log 2>&1 || exit 1
tail -2 $O/mx8_model.log
for m in t2t_vit_14 swin_tiny; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$m -o run \
    -- python3 $R/bench.py --model $m --batch 256 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_$m.log 2>&1 || exit 1
  find $R/$O/prof_$m -name "*kernel_stats*" -exec cp {} $R/$O/${m}_kernel_stats.csv \;
  python3 scripts/kstats.py $O/${m}_kernel_stats.csv 256 | head -24
done
