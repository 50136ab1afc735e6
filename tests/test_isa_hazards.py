"""The wide-store data hazard (scripts/probe/store_hazard.py): no vector-memory store of more than
64 bits may be followed directly by a vector instruction that overwrites its data VGPRs. hipcc
inserts no wait state for it on gfx950, and in the persistent GEMM epilogue it stored zeros into
about 1 launch in 12 (gemm.hip wide_store_fence). Checks the gfx950 code objects of the built
library's objects (edgevisiontransformer_amd/build_obj), disassembled on the CPU."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "edgevisiontransformer_amd", "build_obj")
LLVM = "/opt/rocm/llvm/bin"
sys.path.insert(0, os.path.join(ROOT, "scripts", "probe"))

OBJS = sorted(glob.glob(os.path.join(OBJ, "*.hip.o")))


@pytest.mark.skipif(not OBJS or not os.path.exists(os.path.join(LLVM, "llvm-objdump")),
                    reason="library objects or ROCm llvm tools not present")
@pytest.mark.parametrize("obj", [os.path.basename(o) for o in OBJS])
def test_no_wide_store_data_hazard(tmp_path, obj):
    import store_hazard
    fb, co, dis = tmp_path / "fb.bin", tmp_path / "co.o", tmp_path / "co.dis"
    run = lambda *a: subprocess.run(a, check=True, capture_output=True, timeout=300)  # noqa: E731
    run(f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", os.path.join(OBJ, obj),
        str(tmp_path / "host.o"))
    run(f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}")
    with open(dis, "w") as f:
        subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                       stdout=f, timeout=300)
    hits = store_hazard.scan(str(dis))
    assert not hits, "\n".join(f"{fn}: {a} -> {b}" for fn, _, a, b in hits[:10])
