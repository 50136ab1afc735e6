"""Per-launch sequence of the last Swin forward in a rocprofv3 kernel trace (stage / op table)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if 'evt' in r['Kernel_Name'] and not any(x in r['Kernel_Name'] for x in ('pack', 'fold', 'rpb'))]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'swin_patch' in r['Kernel_Name']]
f = rows[idx[-1]:]
tot = 0
out = []
for r in f:
    n = r['Kernel_Name']
    m = re.search(r'gemm_pers_kernel<(\d+)|gemm_nt_kernel\w*Li(\d+)|gemm_big_kernel<(\d+)|(window_attn|ln_rows|merge|swin_patch|ln_pool)', n)
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += d
    out.append(f"{(m.group(0) if m else n)[:24]}:{d:.0f}")
print(" ".join(out))
print("total", round(tot, 1))
