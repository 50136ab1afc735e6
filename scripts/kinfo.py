"""Register / scratch / LDS summary of every kernel in a hipcc -S output (.amdhsa_kernel blocks).
    python scripts/kinfo.py file.s [substring]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
    name, body = m.group(1), m.group(2)
    if flt not in name:
        continue
    f = lambda k: (re.search(rf"\.amdhsa_{k} (\d+)", body) or [None, "?"])[1]  # noqa: E731
    print(f"{name[-60:]:60s} vgpr {f('next_free_vgpr'):>4s} agpr_off {f('accum_offset'):>4s} "
          f"scratch {f('private_segment_fixed_size'):>4s} lds {f('group_segment_fixed_size'):>6s}")
