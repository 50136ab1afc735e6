"""Scan gfx950 assembly for the wide-store data hazard: a vector-memory store of more than 64 bits
reads its data VGPRs after issue, so a VALU instruction that overwrites them fewer than
WAIT_STATES wait states later can land first. Found as the cause of rare wrong output elements in
the persistent GEMM epilogue (buffer_store_dwordx4 v[2:5] followed by v_and_b32 v3, ...).

Wait states are counted the way the hardware (and LLVM's GCNHazardRecognizer) counts them: every
issued instruction after the store is one wait state, `s_nop N` is N + 1. gfx940-family parts
(gfx950 included) need 2 (LLVM: `VALUWaitStates = hasGFX940Insts() ? 2 : 1`), so the window is
the next two wait states: any vector instruction writing one of the store's data VGPRs inside it
is a hit. (LLVM skips MUBUF stores whose soffset is an SGPR; the measured failure was exactly
such a store, so this scan does not.)

Usage:
  python scripts/probe/store_hazard.py [--lds] file [...]   (hipcc --cuda-device-only -S output, or
  llvm-objdump -d of the gfx950 code object: tests/test_isa_hazards.py extracts it from build_obj/)
--lds also lists LDS stores (ds_write_b128 ...), where no corruption has been observed.
--strict lists every wide buffer store without the library's fence (s_nop 1 or longer) before
the next vector instruction, hazard or not."""
import re
import sys

WAIT_STATES = 2
VMEM = r"buffer_store_dwordx[34]|global_store_dwordx[34]|flat_store_dwordx[34]|scratch_store_dwordx[34]" \
       r"|buffer_store_b(?:96|128)|global_store_b(?:96|128)|flat_store_b(?:96|128)"
LDS = r"|ds_write_b96|ds_write_b128|ds_write2_b64"
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _store_re(lds):
    return re.compile(r"^\s*(" + VMEM + (LDS if lds else "") + r")\s+(.*)$")


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


def _instr(line):
    """opcode and operand text of an assembly / objdump line, or None for labels, directives,
    comments and blank lines"""
    t = line.strip()
    if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
        return None
    m = re.match(r"^[0-9a-f]+ <.+>:$", t)
    if m:
        return None
    op, _, rest = t.partition(" ")
    if not re.match(r"^[a-z_][a-z0-9_]*$", op):
        return None
    return op, rest.strip()


def wait_states(op, rest):
    if op == "s_nop":
        try:
            return int(rest.split()[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def vgpr_dst(op, rest):
    """VGPRs a vector instruction writes (its first operand), empty for non-VALU / SGPR dsts"""
    if not op.startswith("v_") or op.startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_cmpx")):
        return set()
    dst = rest.split(",")[0] if rest else ""
    return regs(dst)


def scan_lines(lines, lds=False):
    store = _store_re(lds)
    fn, hits = None, []
    body = [l.split("//")[0].rstrip() for l in lines]
    for i, l in enumerate(body):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", l)
        if m:
            fn = m.group(1)
        elif re.match(r"^[_A-Za-z][\w.$]*:", l) and not l.startswith(".L"):
            fn = l.split(":")[0]
        m = store.match(l)
        if not m:
            continue
        d = data_regs(m.group(1), m.group(2))
        states, j = 0, i + 1
        while j < len(body) and states < WAIT_STATES:
            ins = _instr(body[j])
            if ins is not None:
                op, rest = ins
                if op == "s_endpgm":
                    break
                if vgpr_dst(op, rest) & d:
                    hits.append((fn, i + 1, l.strip(), body[j].strip()))
                    break
                states += wait_states(op, rest)
            j += 1
    return hits


BUFFER_WIDE = re.compile(r"^\s*(buffer_store_dwordx[34]|buffer_store_b(?:96|128))\s+(.*)$")


def unfenced(lines):
    """wide BUFFER stores without the library's fence (csrc/common.h wide_store_fence: s_nop 1)
    before the next vector instruction. LLVM's hazard recognizer does not cover buffer stores
    with an SGPR soffset (the measured failure), so every one must come from the store helpers.
    Global / flat / scratch stores (incl. compiler-merged and spill stores) are covered by LLVM;
    scan() checks them anyway."""
    fn, out = None, []
    body = [l.split("//")[0].rstrip() for l in lines]
    for i, l in enumerate(body):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", l)
        if m:
            fn = m.group(1)
        if not BUFFER_WIDE.match(l):
            continue
        ok, j, seen = False, i + 1, 0
        while j < len(body) and seen < 8:
            ins = _instr(body[j])
            j += 1
            if ins is None:
                continue
            seen += 1
            if ins[0] == "s_nop" and wait_states(*ins) >= WAIT_STATES:
                ok = True
                break
            # conditional branches (waterfall loops over a divergent resource) fall through
            if ins[0].startswith("v_") or ins[0] in ("s_endpgm", "s_branch"):
                break
        if not ok:
            out.append((fn, i + 1, l.strip(), body[j - 1].strip() if j <= len(body) else ""))
    return out


def scan(path, lds=False):
    """path: hipcc -S output, or llvm-objdump -d text of a gfx950 code object"""
    return scan_lines(open(path).read().split("\n"), lds)


if __name__ == "__main__":
    total = 0
    lds = "--lds" in sys.argv
    strict = "--strict" in sys.argv
    for p in [a for a in sys.argv[1:] if not a.startswith("--")]:
        found = unfenced(open(p).read().split("\n")) if strict else scan(p, lds)
        for fn, ln, a, b in found:
            total += 1
            print(f"{p}:{ln} {fn[:90]}\n    {a}\n    {b}")
    print(f"{total} hazard(s)")
    sys.exit(1 if total else 0)
