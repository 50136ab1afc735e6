"""Scratch (spill) instructions of one kernel in a hipcc -S output, by barrier segment, with the
MFMA / ds_read / LDS-DMA counts of each segment that has any: where a kernel's spills sit relative
to its main loop.   python scripts/spills.py file.s kernel_substring"""
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2]
i = next(m.start() for m in re.finditer(r"^(\S+):", s, re.M) if want in m.group(1))
j = s.index(".Lfunc_end", i)
seg, cur = [], {"mfma": 0, "ds": 0, "glds": 0, "scratch": []}
for l in s[i:j].split("\n"):
    t = l.strip()
    if t.startswith("s_barrier"):
        seg.append(cur)
        cur = {"mfma": 0, "ds": 0, "glds": 0, "scratch": []}
        continue
    if t.startswith("v_mfma"):
        cur["mfma"] += 1
    elif t.startswith("ds_read"):
        cur["ds"] += 1
    elif "_lds" in t.split(" ")[0] or (t.startswith("buffer_load") and " lds" in t):
        cur["glds"] += 1
    elif t.startswith("scratch_"):
        cur["scratch"].append(t.split(";")[0].strip())
seg.append(cur)
tot = 0
for k, c in enumerate(seg):
    if c["scratch"]:
        tot += len(c["scratch"])
        print(k, f"mfma {c['mfma']} ds {c['ds']} glds {c['glds']}", c["scratch"][:6],
              "..." if len(c["scratch"]) > 6 else "")
print("segments", len(seg), "scratch ops", tot)
