"""Round-6 probe: kernel concurrency in a rocprofv3 kernel trace (run_kernel_trace.csv): the
fraction of the busy time with two or more kernels in flight, per queue / stream id, over the
last `--tail` seconds of the trace (the timed steps).
    python scripts/probe/overlap_trace.py <kernel_trace.csv> [tail_ms]"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
tail = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""), r.get("Stream_Id", ""))
      for r in rows]
t_end = max(e for _, e, _, _ in ev)
t0 = t_end - int(tail * 1e6)
ev = [x for x in ev if x[1] > t0]
pts = sorted([(s, 1) for s, _, _, _ in ev] + [(e, -1) for _, e, _, _ in ev])
busy = multi = 0
cur, last = 0, None
for t, d in pts:
    if last is not None and cur > 0:
        busy += t - last
        if cur > 1:
            multi += t - last
    cur += d
    last = t
print(f"kernels {len(ev)}  busy {busy / 1e6:.2f} ms  >=2 in flight {multi / 1e6:.2f} ms "
      f"({100.0 * multi / max(busy, 1):.1f} %)")
print("queues:", Counter(q for _, _, q, _ in ev).most_common(6))
print("streams:", Counter(s for _, _, _, s in ev).most_common(6))
