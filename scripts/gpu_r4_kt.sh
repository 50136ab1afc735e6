#!/bin/bash
# Per-launch durations (rocprofv3 kernel trace) of kernels matching KNAME in a bench
# configuration (ARGS), for each library in LIBS ("product" = libevt_hip.so), alternating PAIRS times.
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-kt}
mkdir -p $O
D=$R/edgevisiontransformer_amd
for i in $(seq ${PAIRS:-2}); do
  for l in ${LIBS:-product libevt_hip_lab.so}; do
    lib=$D/libevt_hip.so; [ "$l" = product ] || lib=$D/$l
    rm -rf $O/$l
    EVT_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/$l -o run \
      -- python3 $R/bench.py $ARGS --cpu-seconds 0 --no-probe --steps 3 --warmup 1 > $O/$l.log 2>&1 || exit 1
    python3 - "$O/$l" "$KNAME" "$l" <<'PY'
import csv, glob, collections, sys
O, kname, tag = sys.argv[1], sys.argv[2], sys.argv[3]
by = collections.defaultdict(list)
for f in glob.glob(f"{O}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            by[r.get("Grid_Size_X", "?")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(tag, "  ".join(f"grid {g}: n {len(v)} med {sorted(v)[len(v)//2]:.1f}" for g, v in sorted(by.items())))
PY
  done
done
