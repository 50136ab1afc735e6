"""The wide-store data hazard (csrc/common.h wide_store_fence, scripts/probe/store_hazard.py).

A vector-memory store of more than 64 bits reads its data VGPRs after issue; a VALU write to them
within 2 wait states (gfx940 family, gfx950 included) can land first. hipcc inserts no wait state
after BUFFER stores with an SGPR soffset, and in the persistent GEMM epilogue that stored zeros into
about 1 launch in 12. Guarded three ways, all on the CPU:
  * source: every explicit >64-bit global / buffer store goes through the common.h helpers
    (store_b128 / store_b128_nt / buffer_store_b128 / store_f32x4 / store_bf16x8);
  * code objects (built here when missing, never skipped): no vector write to a wide store's data
    VGPRs inside 2 wait states, in any kernel, including compiler-merged and spill stores; every
    wide buffer store is fenced (s_nop 1) before the next vector instruction;
  * the scanner itself, on synthetic assembly (it must flag `store; s_nop 0; v_and vdata`).
"""
import glob
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "edgevisiontransformer_amd", "csrc")
OBJ = os.path.join(ROOT, "edgevisiontransformer_amd", "build_obj")
LLVM = "/opt/rocm/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "scripts", "probe"))
import store_hazard  # noqa: E402

sys.path.insert(0, ROOT)
from edgevisiontransformer_amd.build import SOURCES  # noqa: E402

HIP_SOURCES = [s for s in SOURCES if s.endswith(".hip")]


@pytest.fixture(scope="module")
def objects():
    missing = [s for s in HIP_SOURCES if not os.path.exists(os.path.join(OBJ, s + ".o"))]
    if missing:  # a fresh checkout: build (hipcc cross-compiles for gfx950 without a GPU)
        from edgevisiontransformer_amd.build import build
        build()
    return {s: os.path.join(OBJ, s + ".o") for s in HIP_SOURCES}


def _disassemble(obj, tmp_path):
    fb, co, dis = tmp_path / "fb.bin", tmp_path / "co.o", tmp_path / "co.dis"
    run = lambda *a: subprocess.run(a, check=True, capture_output=True, timeout=300)  # noqa: E731
    run(f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, str(tmp_path / "host.o"))
    run(f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}")
    with open(dis, "w") as f:
        subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                       stdout=f, timeout=300)
    return open(dis).read().split("\n")


@pytest.mark.parametrize("src", HIP_SOURCES)
def test_code_object_has_no_wide_store_hazard(objects, tmp_path, src):
    lines = _disassemble(objects[src], tmp_path)
    assert sum(1 for l in lines if store_hazard._store_re(False).match(l.split("//")[0])) > 0 or \
        src in ("norm.hip",), f"{src}: no wide stores found (disassembly parse broken?)"
    hits = store_hazard.scan_lines(lines)
    assert not hits, "\n".join(f"{fn[:80]}: {a} -> {b}" for fn, _, a, b in hits[:10])
    unf = store_hazard.unfenced(lines)
    assert not unf, "unfenced buffer stores:\n" + "\n".join(f"{fn[:80]}: {a} -> {b}"
                                                            for fn, _, a, b in unf[:10])


STORE = "buffer_store_dwordx4 v[2:5], v46, s[28:31], s0 offen nt"


@pytest.mark.parametrize("between,flag", [
    ([], True),                                       # the round-2 failure: next slot
    (["s_nop 0"], True),                              # one wait state: not enough on gfx950
    (["s_nop 1"], False),                             # the fence
    (["v_add_u32_e32 v9, 1, v9"], True),              # one unrelated VALU = one wait state
    (["v_add_u32_e32 v9, 1, v9", "s_nop 0"], False),  # two wait states
    (["s_mov_b32 s1, 0", "s_mov_b32 s2, 0"], False),
])
def test_scanner_wait_state_window(between, flag):
    asm = ["0000000000001000 <kern>:", "\t" + STORE + "  // 000000001000: E07E1000",
           *["\t" + b for b in between], "\tv_and_b32_e32 v3, 64, v224"]
    assert bool(store_hazard.scan_lines(asm)) == flag
    # writes to other registers are never hits; a read of the data registers is not a write
    assert not store_hazard.scan_lines(asm[:2] + ["\tv_and_b32_e32 v6, 64, v3"])


@pytest.mark.parametrize("nxt,fenced", [("s_nop 0", False), ("s_nop 1", True), ("s_nop 4", True),
                                        ("v_mov_b32_e32 v9, 0", False)])
def test_scanner_fence_check(nxt, fenced):
    asm = ["0000000000001000 <kern>:", "\t" + STORE, "\t" + nxt, "\tv_mov_b32_e32 v3, 0"]
    assert (not store_hazard.unfenced(asm)) == fenced
    # global stores are LLVM's to fence: only the hazard window applies
    g = ["0000000000001000 <kern>:", "\tglobal_store_dwordx4 v[0:1], v[2:5], off", "\t" + nxt]
    assert not store_hazard.unfenced(g)


RAW = re.compile(r"__builtin_nontemporal_store|__builtin_amdgcn_raw_buffer_store|"
                 r"\*\s*\(\s*(u32x4|f32x4|bf16x8|i32x4|u32x3|float4|uint4)\s*\*\s*\)[^;=]*=[^=]")


@pytest.mark.parametrize("src", HIP_SOURCES)
def test_sources_store_wide_only_through_helpers(src):
    bad = []
    for i, line in enumerate(open(os.path.join(CSRC, src)), 1):
        code = line.split("//")[0]
        if RAW.search(code) and "// LDS" not in line and "EVT_LDS" not in code:
            bad.append(f"{src}:{i}: {line.strip()}")
    assert not bad, "wide stores outside the common.h helpers:\n" + "\n".join(bad)


# ---- M0 integrity around the inline-asm LDS-DMA (csrc/common.h glds16s / glds16s_pair) ----------
# The inline asm writes M0 (the LDS destination of global_load_lds) and lists it as clobbered, but
# hipcc documents that it may not preserve reserved registers across asm. Every LDS DMA hipcc emits
# itself (the 64-bit-vaddr form, "v[..], off") must therefore see an M0 write of its own after the
# last inline-asm DMA block (the saddr form, "vN, s[..]") that precedes it; and M0 must have no
# other reader (s_movrel / v_movrel / ds_gws / s_sendmsg) in the kernels that use the asm form.
_M0_WRITE = re.compile(r"^\s*s_\w+\s+m0\b")
_GLDS_VADDR = re.compile(r"global_load_lds_dword\w*\s+v\[\d+:\d+\],\s*off")
_GLDS_SADDR = re.compile(r"global_load_lds_dword\w*\s+v\d+,\s*s\[\d+:\d+\]")
_M0_READERS = re.compile(r"\b(s_movrel\w*|v_movrel\w*|ds_gws\w*|s_sendmsg\w*)\b")


def m0_problems(lines):
    """Indices of hipcc LDS DMAs whose M0 may be an inline-asm block's, and of other M0 readers."""
    bad, last_write, saddr_since = [], None, False
    for i, raw in enumerate(lines):
        l = raw.split("//")[0]
        if re.match(r"^[0-9a-f]+ <.*>:", raw.strip()):  # a new function (disassembly label)
            last_write, saddr_since = None, False
        if _M0_WRITE.match(l):
            last_write, saddr_since = i, False
        elif _GLDS_SADDR.search(l):
            saddr_since = True
        elif _GLDS_VADDR.search(l) and (last_write is None or saddr_since):
            bad.append(i)
        if _M0_READERS.search(l):
            bad.append(i)
    return bad


def test_m0_scanner_flags_a_stale_m0():
    asm = ["s_mov_b32 m0, s4", "s_nop 0", "global_load_lds_dwordx4 v1, s[2:3]",
           "global_load_lds_dwordx4 v[4:5], off"]
    assert m0_problems(asm) == [3]
    assert m0_problems(["s_mov_b32 m0, s4", "global_load_lds_dwordx4 v1, s[2:3]",
                        "s_add_i32 m0, s5, 0x400", "global_load_lds_dwordx4 v[4:5], off"]) == []


def test_gemm_m0_integrity(objects, tmp_path):
    lines = _disassemble(objects["gemm.hip"], tmp_path)
    assert sum(1 for l in lines if _GLDS_SADDR.search(l)) > 0, "no inline-asm LDS DMA found"
    bad = m0_problems(lines)
    assert not bad, "\n".join(lines[max(0, i - 6): i + 1][-7:][0] + " ... " + lines[i] for i in bad[:5])
