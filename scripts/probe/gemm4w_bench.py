"""Round-6 probe driver: the 4-wave software-pipelined main loop (scripts/probe/gemm4w.hip) against
the product persistent GEMM (evt_dense, flags 0 = plain bf16 stores; lab variant 17 = no epilogue
when EVT_LIB points at a lab build) on the same operands, HIP events, median of 5 x 10 launches.
    python scripts/probe/gemm4w_bench.py [MxKxN ...]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
probe = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemm4w.so"))
probe.gemm4w_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
shapes = sys.argv[1:] or ["100864x3072x768", "100864x768x3072", "100864x768x2304", "8192x8192x8192"]


def timeit(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    return sorted(ts)[2]


g = torch.Generator(device="cuda").manual_seed(0)
for sh in shapes:
    M, K, N = map(int, sh.split("x"))
    A = torch.randn((M, K), generator=g, device="cuda").bfloat16()
    W = torch.randn((N, K), generator=g, device="cuda").bfloat16()
    C = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    Cp = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    fl = 2.0 * M * N * K
    out = {"shape": sh}
    for var in (0, 1):
        assert probe.gemm4w_launch(P(A), P(W), P(C), M, N, K, var, 1, S()) == 0
        torch.cuda.synchronize()
        if var == 1:  # correctness on a row sample
            rows = torch.arange(0, M, max(1, M // 64), device="cuda")
            ref = (A[rows].float() @ W.float().t())
            out["maxdiff_vs_fp32"] = float((C[rows].float() - ref).abs().max())
            out["ref_absmax"] = float(ref.abs().max())
        for store in (1, 0):
            ms = timeit(lambda: probe.gemm4w_launch(P(A), P(W), P(C), M, N, K, var, store, S()))
            out[f"probe_v{var}_store{store}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    # the product persistent kernel (W packed [Npad][Kpad] = W itself here: N % 256 == 0)
    for v in [0] + ([17] if os.environ.get("EVT_LIB") else []):
        if lib.evt_set_gemm_variant(v) != 0:
            continue
        a = _lib.evt_dense_args()
        a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = 0, A.data_ptr(), K, W.data_ptr(), K, N
        a.C, a.ldc, a.M, a.N = Cp.data_ptr(), N, M, N
        ms = timeit(lambda: _lib.check(lib.evt_dense(1, ctypes.byref(a), S())))
        out[f"product_v{v}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
        if v == 0:
            torch.cuda.synchronize()
            out["probe_vs_product_maxdiff"] = float((C.float() - Cp.float()).abs().max())
    lib.evt_set_gemm_variant(0)
    print(json.dumps(out), flush=True)
    del A, W, C, Cp
    torch.cuda.empty_cache()
