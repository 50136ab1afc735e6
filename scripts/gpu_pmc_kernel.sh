#!/bin/bash
# SQ / TA / TD / TCP / TCC counters of one kernel (KNAME substring) inside real forwards of a bench
# configuration (ARGS), one rocprofv3 --pmc pass per counter group (slot limits: 8 SQ, 4 TCC,
# 4 TCP, 2 TA, 2 TD, 2 GRBM), kernel-trace only; per-launch averages (counters summed over each
# dispatch's rows, FETCH_SIZE doubled per the gfx950 note in MI355X_MICROARCH.md).
set -u
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_${TAG:-kernel}
mkdir -p $O
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $GROUP --output-format csv -d $O/p$i -o run \
    -- python3 $R/bench.py $ARGS --cpu-seconds 0 --no-probe --steps 2 --warmup 1 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'G'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU
GRBM_GUI_ACTIVE GRBM_COUNT TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
FETCH_SIZE
WRITE_SIZE
G
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run \
  -- python3 $R/bench.py $ARGS --cpu-seconds 0 --no-probe --steps 2 --warmup 1 > $O/kt.log 2>&1 || exit 1
python3 - "$O" "$KNAME" <<'PY'
import csv, glob, collections, sys
O, kname = sys.argv[1], sys.argv[2]
by = collections.defaultdict(list)  # per-dispatch durations by grid size (one group per stage)
for f in glob.glob(f"{O}/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            by[r.get("Grid_Size_X", r.get("Grid_Size", "?"))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for g, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print(f"grid {g}: {len(v)} launches, median {v[len(v)//2]:.1f} us, min {v[0]:.1f}")
PY
python3 - "$O" "$KNAME" <<'PY'
import csv, glob, collections, json, sys
O, kname = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(f"{O}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
c = {k: agg[k] / len(n[k]) for k in agg}
if "FETCH_SIZE" in c: c["FETCH_BYTES_corrected"] = 2 * 1024 * c["FETCH_SIZE"]
if "WRITE_SIZE" in c: c["WRITE_BYTES"] = 1024 * c["WRITE_SIZE"]
print(json.dumps({"kernel": kname, "launches": max(len(v) for v in n.values()) if n else 0,
                  "per_launch": {k: f"{v:.4e}" for k, v in sorted(c.items())}}, indent=1))
PY
