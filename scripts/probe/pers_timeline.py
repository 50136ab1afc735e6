"""Timeline probe of the persistent GEMM kernel (variant 13): per block and tile, s_memtime at
tile start / after the main loop / after coefficients + next-prologue issue / after the epilogue.
Prints median cycle counts of each segment (100 MHz-ish s_memtime units are core clocks on gfx9)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
_lib.ensure_device(0)
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
M = 100864
TV = int(os.environ.get("TV", "13"))
g = torch.Generator(device="cuda").manual_seed(0)
for spec in os.environ.get("GS", "768x3072@35,768x2304@33,768x768@197,3072x768@197").split(","):
    kn, _, fl = spec.partition("@")
    K, N = (int(v) for v in kn.split("x"))
    fl = int(fl)
    A = torch.randn((M, K), generator=g, device="cuda").bfloat16()
    W = torch.randn((K, N), generator=g, device="cuda") / K ** 0.5
    npad = (N + 255) // 256 * 256
    wp = torch.empty((npad, K), dtype=torch.bfloat16, device="cuda")
    _lib.check(lib.evt_pack_weight(1, P(W), ctypes.c_void_p(0), K, N, P(wp), K, npad, S()))
    bias = torch.randn(npad, generator=g, device="cuda") * 0.1
    R = torch.randn((M, N), generator=g, device="cuda").bfloat16()
    nsl = 2 * ((K + 255) // 256)
    stats = torch.zeros((M, nsl, 2), device="cuda")
    stats[:, 0, 1] = float(K)
    colsum = torch.randn(npad, generator=g, device="cuda")
    nso = 2 * ((N + 255) // 256)
    rst = torch.zeros((M, nso, 2), device="cuda")
    rst[:, 0, 1] = float(N)
    rg, rb = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
    sto = torch.zeros((M, nso, 2), device="cuda")
    C = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    dbg = torch.zeros(256 * 16 * 8, dtype=torch.int64, device="cuda")
    a = _lib.evt_dense_args()
    a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = fl, A.data_ptr(), K, wp.data_ptr(), K, npad
    a.C, a.ldc, a.M, a.N, a.bias = C.data_ptr(), N, M, N, bias.data_ptr()
    a.pos = dbg.data_ptr()
    if fl & 4:
        a.resid, a.ldr = R.data_ptr(), N
    if fl & 64:
        a.rstats, a.rgamma, a.rbeta, a.ln_width, a.ln_eps = rst.data_ptr(), rg.data_ptr(), rb.data_ptr(), N, 1e-5
    if fl & 128:
        a.stats_out = sto.data_ptr()
    if fl & 32:
        a.colsum, a.stats_in, a.ln_width, a.ln_eps = colsum.data_ptr(), stats.data_ptr(), K, 1e-5
    for v in (9, TV, TV):
        _lib.check(lib.evt_set_gemm_variant(v))
        _lib.check(lib.evt_dense(1, ctypes.byref(a), S()))
        torch.cuda.synchronize()
    lib.evt_set_gemm_variant(0)
    t = dbg.cpu().numpy().reshape(256, 16, 8).astype(np.float64)
    valid = t[:, :, 0] > 0
    seg = {"main": t[:, :, 1] - t[:, :, 0], "coef+issue": t[:, :, 2] - t[:, :, 1],
           "epi:fold/gelu": t[:, :, 3] - t[:, :, 2], "epi:swap/resid/stats": t[:, :, 4] - t[:, :, 3],
           "epi:stores": t[:, :, 5] - t[:, :, 4], "epi:statx": t[:, :, 7] - t[:, :, 5],
           "epilogue": t[:, :, 7] - t[:, :, 2]}
    nxt = t[:, 1:, 0] - t[:, :-1, 7]
    out = {k: (np.median(v[valid]), np.percentile(v[valid], 90)) for k, v in seg.items()}
    out["gap"] = (np.median(nxt[valid[:, 1:]]), 0)
    # per-iteration medians of main loop (first tiles are special)
    per_it = [float(np.median(seg["main"][:, i][valid[:, i]])) for i in range(6) if valid[:, i].any()]
    print(spec, {k: (round(a_), round(b_)) for k, (a_, b_) in out.items()}, "main per iter", [round(x) for x in per_it],
          flush=True)
