"""Build libevt_hip.so (gfx950) in-tree with hipcc; no torch extension machinery involved.

`python -m edgevisiontransformer_amd.build` or `__graft_entry__.build()`. Objects are compiled in
parallel; the link is skipped when every source is older than the library.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# EVT_LAB=1: the diagnostic build (GEMM ablation / timeline variants, qkv_attn ablations) into
# libevt_hip_lab.so (load it with EVT_LIB=<path>); the product library never contains them
LAB = os.environ.get("EVT_LAB", "") not in ("", "0")
LIB = os.path.join(HERE, "libevt_hip_lab.so" if LAB else "libevt_hip.so")
OBJ = os.path.join(HERE, "build_obj_lab" if LAB else "build_obj")
SOURCES = ["gemm.hip", "attention.hip", "norm.hip", "t2t.hip", "swin.hip", "mx8.hip", "capi.cpp"]
HEADERS = ["common.h", "evt_internal.h", os.path.join("..", "..", "include", "evt.h")]
ARCH = os.environ.get("EVT_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-ffp-contract=on"]  # contraction only within one source expression: same result on
#                                every code path (interior / edge tiles) -> batch-independent bits
if LAB:
    FLAGS += ["-DEVT_GEMM_LAB"] + ([f"-DEVT_QA_DBG={os.environ['EVT_QA_DBG']}"]
                                   if os.environ.get("EVT_QA_DBG") else [])
    FLAGS += os.environ.get("EVT_LAB_DEFS", "").split()  # e.g. -DEVT_MFMA_PRIO=0 (lab A/B)


# MFMA results straight into VGPRs: with the default AGPR form the compiler parks the small
# attention / window-attention / performer accumulators in AGPRs and copies every element back
# (v_accvgpr_read) before the softmax / GELU VALU work (96 copies per window-attention wave).
PER_FILE_FLAGS = {s: ["-mllvm", "-amdgpu-mfma-vgpr-form=true"]
                  for s in ("attention.hip", "swin.hip", "t2t.hip")}
# attention.hip: no NaN operands either (scores of finite bf16 / fp32 q, k; masked keys are -inf):
# the softmax max runs on the raw MFMA results without a canonicalising v_max per element
PER_FILE_FLAGS["attention.hip"] = PER_FILE_FLAGS["attention.hip"] + ["-fno-honor-nans"]
# swin.hip: the same for the window-attention softmax (finite scores, -inf masks; 32 canonicalising
# v_max per wave before, round-4 counters)
PER_FILE_FLAGS["swin.hip"] = PER_FILE_FLAGS["swin.hip"] + ["-fno-honor-nans"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def _mtime(p: str) -> float:
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    # a change of compile flags (EVT_LAB_DEFS, EVT_ARCH, ...) rebuilds every object
    stamp = os.path.join(OBJ, "flags.txt")
    want = repr((FLAGS, PER_FILE_FLAGS))
    if not os.path.exists(stamp) or open(stamp).read() != want:
        force = True
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    jobs = []
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        objs.append(o)
        if force or _mtime(o) < max(_mtime(s), hdr_t):
            cmd = [_hipcc(), *FLAGS, *PER_FILE_FLAGS.get(src, []), "-c", s, "-o", o]
            if src.endswith(".cpp"):
                cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-c", s, "-o", o]
            jobs.append(cmd)

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(" ".join(cmd))
        return r

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _mtime(LIB) < max(_mtime(o) for o in objs):
        run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB])
    with open(stamp, "w") as f:
        f.write(want)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
