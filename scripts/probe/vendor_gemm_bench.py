"""Round-6 reference point: the product persistent GEMM (evt_dense, flags 0 = plain bf16 stores)
against the vendor libraries torch.matmul dispatches to on ROCm (hipBLASLt, and rocBLAS where
torch can select it) on the same operands: C[M][N] = A[M][K] . W[N][K]^T, bf16 in / bf16 out,
fp32 accumulation. HIP events on torch's current stream, median of 5 x 10 launches.
    python scripts/probe/vendor_gemm_bench.py [MxKxN ...]"""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
# DeiT-base at 512 images (M = 512 x 197 = 100864): FC1, FC2, QKV, out-proj; at 64 images
# (M = 12608): the same four; and a square reference shape
shapes = sys.argv[1:] or ["100864x768x3072", "100864x3072x768", "100864x768x2304",
                          "100864x768x768", "12608x768x3072", "12608x3072x768",
                          "12608x768x2304", "12608x768x768", "8192x8192x8192"]


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


def blas_backends():
    out = []
    for name in ("hipblaslt", "rocblas"):
        try:
            torch.backends.cuda.preferred_blas_library(name)
            out.append(name)
        except Exception:  # noqa: BLE001 - a backend this torch build cannot select
            pass
    return out


backends = blas_backends()
g = torch.Generator(device="cuda").manual_seed(0)
for sh in shapes:
    M, K, N = map(int, sh.split("x"))
    A = torch.randn((M, K), generator=g, device="cuda").bfloat16()
    W = torch.randn((N, K), generator=g, device="cuda").bfloat16()
    Cp = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    Cv = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    fl = 2.0 * M * N * K
    out = {"shape": f"M{M} K{K} N{N}"}
    a = _lib.evt_dense_args()
    a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = 0, A.data_ptr(), K, W.data_ptr(), K, N
    a.C, a.ldc, a.M, a.N = Cp.data_ptr(), N, M, N
    ms = timeit(lambda: _lib.check(lib.evt_dense(1, ctypes.byref(a), S())))
    out["product"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    Wt = W.t()
    for be in backends:
        torch.backends.cuda.preferred_blas_library(be)
        ms = timeit(lambda: torch.matmul(A, Wt, out=Cv))
        torch.cuda.synchronize()
        d = float((Cv.float() - Cp.float()).abs().max())
        out[be] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1), "maxdiff_vs_product": d}
    print(json.dumps(out), flush=True)
    del A, W, Cp, Cv
    torch.cuda.empty_cache()
