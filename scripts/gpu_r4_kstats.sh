#!/bin/bash
# rocprofv3 kernel stats of bench configurations: KS="name|bench args;name|bench args"
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r4ks}
mkdir -p $O
IFS=';' read -ra ITEMS <<< "$KS"
for it in "${ITEMS[@]}"; do
  NAME=${it%%|*}; ARGS=${it#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$NAME -o run \
    -- python3 $R/bench.py $ARGS --cpu-seconds 0 --no-probe > $O/$NAME.jsonl 2>&1 || exit 1
  f=$(find $O/$NAME -name "*kernel_stats*" | head -1)
  echo "== $NAME: $(tail -1 $O/$NAME.jsonl | cut -c1-150)"
  python3 $R/scripts/kstats.py $f ${BATCH:-256} | head -${TOP:-10}
done
