"""Compare the instruction streams of every kernel in two hipcc -S outputs (device code): labels
renumbered, comments / directives dropped. Used to check that a source clean-up leaves the product
kernels' code unchanged.   python scripts/probe/isa_diff.py before.s after.s"""
import re
import sys


def kernels(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
        name, body = m.group(1), m.group(2)
        lines, labels = [], {}
        for ln in body.splitlines():
            ln = ln.split(";")[0].strip()
            if not ln or ln.startswith("."):
                if ln.startswith(".LBB"):
                    labels.setdefault(ln.rstrip(":"), f"L{len(labels)}")
                continue
            lines.append(ln)
        norm = [re.sub(r"\.LBB\d+_\d+", lambda x: labels.setdefault(x.group(0), f"L{len(labels)}"), l)
                for l in lines]
        out[name] = norm
    return out


a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
same = diff = 0
for k in sorted(set(a) & set(b)):
    if a[k] == b[k]:
        same += 1
    else:
        diff += 1
        print("DIFF", k[:110], len(a[k]), len(b[k]))
print("only before:", len(set(a) - set(b)), " only after:", len(set(b) - set(a)))
for k in sorted(set(b) - set(a)):
    print("  new", k[:110])
print(f"identical {same}, different {diff}")
