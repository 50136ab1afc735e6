#!/bin/bash
# Round 4: per-role HBM traffic (FETCH_SIZE / WRITE_SIZE, one rocprofv3 pass each, kernel trace
# only) of every BASELINE config's dominant role over real forwards, then the SQ counter passes
# of the FC1 probe GEMM. COMMIT=<hash> is recorded in the summaries.
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r4pmc}
mkdir -p $O
while read -r NAME ROLE ARGS; do
  [ -z "$NAME" ] && continue
  if [ -n "${ONLY:-}" ] && ! echo " $ONLY " | grep -q " $NAME "; then continue; fi
  mkdir -p $O/$NAME
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/$NAME/$C -o run \
      -- python3 $R/bench.py $ARGS --cpu-seconds 0 --no-probe --steps 3 --warmup 1 > $O/$NAME/$C.log 2>&1
    rc=$?; echo "$NAME $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  set -- $ARGS
  python3 $R/scripts/pmc_roles.py $O/$NAME $2 $4 $6 $ROLE > $O/pmc_$NAME.json || exit 1
  grep -E '"role"|traffic_bytes' $O/pmc_$NAME.json
done <<'L'
deit_base fc1 --model deit_base --dtype bf16 --batch 512
t2t_vit_14 fc1 --model t2t_vit_14 --dtype bf16 --batch 256
swin_tiny fc2 --model swin_tiny --dtype bf16 --batch 256
deit_tiny_f32 fc2 --model deit_tiny --dtype f32 --batch 256
deit_base_bs64 fc1 --model deit_base --dtype bf16 --batch 64
L
if [ -n "${SQ:-}" ]; then TAG=_r4 bash $R/scripts/gpu_pmc_sq.sh > $O/sq.log 2>&1 || exit 1; tail -40 $O/sq.log; fi
