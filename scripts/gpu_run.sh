#!/bin/bash
# One parameterised GPU driver (round 5: replaces the round-2..4 one-off gpu_*.sh scripts).
#
#   TAG=<dir> bash scripts/gpu_run.sh STEP [STEP ...]      (run on the box through gpurun)
#
# Outputs go to gpurun_out/$TAG/. Every GPU step runs under its own time limit and the script stops
# at the first failure (no retries). Bench arguments inside a step are comma-separated.
#   tests[:<pytest args>]   the GPU suite (default: tests -m gpu), one process
#   smoke                   __graft_entry__.smoke()
#   bench:<args>            one bench.py line (e.g. bench:--batch,64,--steps,50)
#   ab:<args>               alternating A/B of bench.py <args> over the arms in $ARMS, $ROUNDS times;
#                           an arm is "lib=<path>" (EVT_LIB), "var=<n>" (--gemm-variant) or "base"
#                           or "env=NAME=VALUE[+NAME=VALUE...]" (environment switches)
#                           (PROBE=1: with the per-role probe; ROLES="attention qkv": print those roles)
#   kstats:<args>           rocprofv3 kernel trace + stats of bench.py <args> -> <name>_kstats.txt
#   pmc:<name>:<role>:<args>  FETCH_SIZE / WRITE_SIZE passes over real forwards -> pmc_<name>.json
#   kpmc:<kernel>:<args>    SQ / TA / TD / TCP / TCC / GRBM counter passes of one kernel
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-run}
mkdir -p $O
ROUNDS=${ROUNDS:-2}
summ() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline'] or {}; pr=r.get('per_role') or {}; print(sys.argv[2], d['config'].get('model'), 'bs', d['config'].get('per_gpu_batch'), d['value'], 'img/s', d['ms_per_step'], 'ms', 'model', d['model_roofline']['frac'], 'dom', r.get('role'), r.get('frac'), 'cpu', (d['cpu_baseline'] or {}).get('value'), ' '.join('%s=%.1f' % (k, v['us_per_launch']) for k, v in pr.items() if k in (sys.argv[3:] or ())))" "$1" "$2" ${ROLES:-}; }
name_of() { echo "$1" | tr -c 'A-Za-z0-9_\n' '_' | sed 's/__*/_/g; s/^_//; s/_$//' | cut -c1-60; }
for STEP in "$@"; do
  kind=${STEP%%:*}; rest=${STEP#*:}; [ "$rest" = "$STEP" ] && rest=""
  case $kind in
  tests)
    args=${rest:-tests -m gpu}; args=${args//,/ }
    timeout -k 10 1100 python -u -m pytest -x -q --timeout 200 --timeout-method thread $args > $O/pytest.log 2>&1
    rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
    grep -v amdgpu.ids $O/smoke.log | tail -3 ;;
  bench)
    a=${rest//,/ }; n=$(name_of "bench $a")
    timeout -k 10 400 python bench.py $a > $O/$n.jsonl 2>&1 || { tail -5 $O/$n.jsonl; exit 1; }
    summ $O/$n.jsonl "$n" ;;
  ab)
    a=${rest//,/ }; np=--no-probe; [ -n "${PROBE:-}" ] && np=""
    for i in $(seq $ROUNDS); do
      for arm in ${ARMS:-base}; do
        n=$(name_of "ab $a $arm $i"); extra=""; envl=""
        case $arm in lib=*) envl="EVT_LIB=$R/${arm#lib=}";; var=*) extra="--gemm-variant ${arm#var=}";; env=*) envl="${arm#env=}"; envl=${envl//+/ };; esac
        env $envl timeout -k 10 300 python bench.py $a $extra --cpu-seconds 0 $np > $O/$n.jsonl 2>&1 || { tail -5 $O/$n.jsonl; exit 1; }
        summ $O/$n.jsonl "$arm#$i"
      done
    done ;;
  kstats)
    a=${rest//,/ }; n=$(name_of "$a")
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run \
      -- python3 $R/bench.py $a --cpu-seconds 0 > $O/${n}_under_rocprof.jsonl 2>&1 || { tail -5 $O/${n}_under_rocprof.jsonl; exit 1; }
    f=$(find $O/prof_$n -name "*kernel_stats*" | head -1); cp "$f" $O/${n}_kernel_stats.csv
    bs=$(echo " $a " | sed -n 's/.* --batch \([0-9]*\) .*/\1/p'); bs=${bs:-512}
    python3 $R/scripts/kstats.py $O/${n}_kernel_stats.csv $bs > $O/${n}_kstats.txt; head -8 $O/${n}_kstats.txt ;;
  pmc)
    nm=${rest%%:*}; rest2=${rest#*:}; role=${rest2%%:*}; a=${rest2#*:}; a=${a//,/ }
    mkdir -p $O/$nm
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/$nm/$C -o run \
        -- python3 $R/bench.py $a --cpu-seconds 0 --no-probe --steps 3 --warmup 1 > $O/$nm/$C.log 2>&1
      rc=$?; echo "$nm $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    set -- $a
    model=deit_base; dtype=bf16; batch=512
    while [ $# -gt 0 ]; do case $1 in --model) model=$2;; --dtype) dtype=$2;; --batch) batch=$2;; esac; shift; done
    python3 $R/scripts/pmc_roles.py $O/$nm $model $dtype $batch $role > $O/pmc_$nm.json || exit 1
    grep -E '"role"|traffic_bytes' $O/pmc_$nm.json ;;
  kpmc)
    kn=${rest%%:*}; a=${rest#*:}; a=${a//,/ }
    KNAME=$kn ARGS="$a" TAG=${TAG:-run}/kpmc_$(name_of "$kn") bash $R/scripts/gpu_pmc_kernel.sh > $O/kpmc_$(name_of "$kn").log 2>&1 || { tail -5 $O/kpmc_$(name_of "$kn").log; exit 1; }
    tail -30 $O/kpmc_$(name_of "$kn").log ;;
  *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
