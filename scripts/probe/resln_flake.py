"""Wrong-result check, one launch at a time (found an intermittent 160-element mismatch between the stream-K (variant 16) and persistent (default)
kernels at 22100 x 768 x 768 with the residual-LayerNorm epilogue under two rejected main-loop
changes): run each kernel N times against one fp32 reference, report which launches differ and
where. Usage: python scripts/probe/resln_flake.py [reps]"""
import math
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402
from tests import _ops  # noqa: E402
from tests.test_gpu_streamk import _randn, _stats, _ln  # noqa: E402

EPI = _lib
M, K, D = 22100, 768, 768
A = _randn((M, K), 11).bfloat16()
W, b = _randn((K, D), 12, 1 / math.sqrt(K)), _randn((D,), 13, 0.1)
x = (_randn((M, D), 14, 1.1) - 0.2).bfloat16()
g, be = 1.0 + _randn((D,), 15, 0.1), _randn((D,), 16, 0.1)
wp, kpad, npad = _ops.pack(W, "bf16")
bias = torch.zeros(npad, device=A.device)
bias[:D] = b
S = 2 * ((D + 255) // 256)
rst = _stats(x)
ref = A.float() @ W.bfloat16().float() + b + _ln(x.float(), g, be)
lib = _lib.load_library()
flags = EPI.EPI_BIAS | EPI.EPI_RESID | EPI.EPI_RESLN | EPI.EPI_STATS
def launch(variant, tag):
    lib.evt_set_gemm_variant(variant)
    so = torch.full((M, S, 2), float("nan"), device=A.device)
    C = torch.zeros((M, D), device=A.device).bfloat16()
    C = _ops.dense("bf16", flags, A, wp, kpad, npad, M, D, bias=bias, resid=x, rstats=rst,
                   rgamma=g, rbeta=be, stats_out=so, ln_width=D, C=C)
    torch.cuda.synchronize()
    bad = ~torch.isclose(C.float(), ref, rtol=2e-2, atol=2e-2)
    n = int(bad.sum())
    if n:
        idx = bad.nonzero()
        rows = sorted(set(idx[:, 0].tolist()))
        cols = sorted(set(idx[:, 1].tolist()))
        print(f"{tag}: {n} bad rows {rows[:8]} ({len(rows)}) cols {cols[:8]} ({len(cols)}) "
              f"zero {int((C.float()[bad] == 0).sum())}", flush=True)
    return n


# the GPU test's order (stream-K twice, then the persistent kernel), repeated
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
tot = {16: 0, 0: 0}
for r in range(reps):
    for v, tag in ((16, "sk"), (16, "sk2"), (0, "pers")):
        tot[v] += launch(v, f"rep {r} {tag}") > 0
print("launches with errors: stream-K", tot[16], "of", 2 * reps, "; persistent", tot[0], "of", reps)
lib.evt_set_gemm_variant(0)
