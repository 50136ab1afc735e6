"""Scan gfx950 assembly for the wide-store data hazard: a vector-memory or LDS store of more than
64 bits whose data VGPRs are overwritten by the very next vector instruction (no wait state in
between). Found as the cause of rare wrong output elements in the persistent GEMM epilogue
(buffer_store_dwordx4 v[2:5] followed by v_and_b32 v3, ...). Usage:
  python scripts/probe/store_hazard.py [--lds] file [...]   (hipcc --cuda-device-only -S output, or
  llvm-objdump -d of the gfx950 code object: tests/test_isa_hazards.py extracts it from build_obj/)
--lds also lists LDS stores (ds_write_b128 ...), where no corruption has been observed."""
import re
import sys

VMEM = r"buffer_store_dwordx[34]|global_store_dwordx[34]|flat_store_dwordx[34]|scratch_store_dwordx[34]"
LDS = r"|ds_write_b96|ds_write_b128|ds_write2_b64"
STORE = re.compile(r"^\s*(" + VMEM + (LDS if "--lds" in sys.argv else "") + r")\s+(.*)$")
VREG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok):
    out = set()
    for m in VREG.finditer(tok):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def data_regs(op, args):
    parts = [a.strip() for a in args.split(",")]
    if op.startswith("ds_write2"):
        return regs(parts[1]) | regs(parts[2])
    if op.startswith("ds_"):
        return regs(parts[1])
    if op.startswith(("buffer_", "scratch_")):
        return regs(parts[0])
    return regs(parts[1])  # global/flat: vaddr, vdata


def scan(path):
    """path: hipcc -S output, or llvm-objdump -d text of a gfx950 code object"""
    lines = [l.split("//")[0].rstrip() for l in open(path).read().split("\n")]
    fn, hits = None, []
    for i, l in enumerate(lines):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", l)
        if m:
            fn = m.group(1)
        elif re.match(r"^[_A-Za-z][\w.$]*:", l) and not l.startswith(".L"):
            fn = l.split(":")[0]
        m = STORE.match(l)
        if not m:
            continue
        d = data_regs(m.group(1), m.group(2))
        # next real instruction
        j = i + 1
        while j < len(lines) and (not lines[j].strip() or lines[j].strip().startswith((";", "."))):
            j += 1
        if j >= len(lines):
            continue
        nxt = lines[j].strip()
        op = nxt.split()[0] if nxt else ""
        if not op.startswith("v_") or op.startswith("v_mfma") or op.startswith("v_readlane") \
                or op.startswith("v_cmp"):
            continue
        dst = nxt.split(None, 1)[1].split(",")[0] if " " in nxt else ""
        if regs(dst) & d:
            hits.append((fn, i + 1, l.strip(), nxt))
    return hits


if __name__ == "__main__":
    total = 0
    for p in [a for a in sys.argv[1:] if not a.startswith("--")]:
        for fn, ln, a, b in scan(p):
            total += 1
            print(f"{p}:{ln} {fn[:90]}\n    {a}\n    {b}")
    print(f"{total} hazard(s)")
    sys.exit(1 if total else 0)
