"""GEMM microbenchmark on the GPU: model-shaped bf16 GEMMs, 128x128 vs 256x256 tile kernels,
interleaved rounds in one process (HIP events), plus a cross-check of the two variants.
Ablation / A-B variants (10, 11, 13, 15, 17-25, 106, 108) exist only in the lab build:
  EVT_LAB=1 python -m edgevisiontransformer_amd.build && EVT_LIB=edgevisiontransformer_amd/libevt_hip_lab.so python scripts/gemm_bench.py ..."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
_lib.ensure_device(0)
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
M = int(sys.argv[1]) if len(sys.argv) > 1 else 512 * 197
VARS = [int(v) for v in sys.argv[2].split(',')] if len(sys.argv) > 2 else [1, 2, 3]
shapes = {"qkv": (768, 2304, 0), "out": (768, 768, 21), "fc1": (768, 3072, 3), "fc2": (3072, 768, 21),
          "nt3072": (3072, 768, 0), "nt768x3072": (768, 3072, 0)}
import os
sel = os.environ.get("GS", "qkv,out,fc1,fc2").split(",")
# custom shapes: "KxN" or "KxN@flags" (e.g. 4096x4096@0)
for it in sel:
    if "x" in it and it not in shapes:
        kn, _, fl = it.partition("@")
        k, n = kn.split("x")
        shapes[it] = (int(k), int(n), int(fl or 0))
shapes = {k: v for k, v in shapes.items() if k in sel}
LDC_PAD = int(os.environ.get("LDC_PAD", "0"))  # extra output row pitch (elements)
res = {}
g = torch.Generator(device="cuda").manual_seed(0)
for name, (K, N, fl) in shapes.items():
    A = torch.randn((M, K), generator=g, device="cuda").bfloat16()
    W = torch.randn((K, N), generator=g, device="cuda") / K ** 0.5
    npad = (N + 255) // 256 * 256
    wp = torch.empty((npad, K), dtype=torch.bfloat16, device="cuda")
    _lib.check(lib.evt_pack_weight(1, P(W), ctypes.c_void_p(0), K, N, P(wp), K, npad, S()))
    bias = torch.randn(npad, generator=g, device="cuda") * 0.1
    R = torch.randn((M, N), generator=g, device="cuda").bfloat16()
    nsl = 2 * ((K + 255) // 256)
    stats = torch.zeros((M, nsl, 2), device="cuda")   # include/evt.h slot layout
    Af = A.float()
    stats[:, 0, 0], stats[:, 0, 1] = Af.sum(1), (Af * Af).sum(1)
    del Af
    colsum = torch.randn(npad, generator=g, device="cuda")
    nso = 2 * ((N + 255) // 256)
    rst = torch.zeros((M, nso, 2), device="cuda")
    Rf = R.float()
    rst[:, 0, 0], rst[:, 0, 1] = Rf.sum(1), (Rf * Rf).sum(1)
    del Rf
    rg, rb = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
    sto = torch.zeros((M, nso, 2), device="cuda")
    outs = {}
    for v in VARS:
        outs[v] = torch.empty((M, N + LDC_PAD), dtype=torch.float32 if fl & 16 else torch.bfloat16,
                              device="cuda")
    def run(v):
        _lib.check(lib.evt_set_gemm_variant(v))
        a = _lib.evt_dense_args()
        a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = fl, A.data_ptr(), K, wp.data_ptr(), K, npad
        a.C, a.ldc, a.M, a.N, a.bias = outs[v].data_ptr(), N + LDC_PAD, M, N, bias.data_ptr()
        if fl & 4:
            a.resid, a.ldr = R.data_ptr(), N
        if fl & 64:
            a.rstats, a.rgamma, a.rbeta, a.ln_width = rst.data_ptr(), rg.data_ptr(), rb.data_ptr(), N
            a.ln_eps = 1e-5
        if fl & 128:
            a.stats_out = sto.data_ptr()
        if fl & 32:
            a.colsum, a.stats_in, a.ln_width, a.ln_eps = colsum.data_ptr(), stats.data_ptr(), K, 1e-5
        _lib.check(lib.evt_dense(1, ctypes.byref(a), S()))
    times = {v: [] for v in VARS}
    for v in VARS:
        run(v)
    torch.cuda.synchronize()
    diff = max((outs[VARS[0]][:, :N].float() - outs[v][:, :N].float()).abs().max().item() for v in VARS)
    for rnd in range(5):
        for v in VARS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    if os.environ.get("TORCHMM") == "1":  # vendor GEMM (hipBLASLt via torch) on the same operands
        Wt = W.bfloat16().contiguous()
        Ct = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        for _ in range(3):
            torch.matmul(A, Wt, out=Ct)
        tt = []
        for rnd in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                torch.matmul(A, Wt, out=Ct)
            e1.record()
            torch.cuda.synchronize()
            tt.append(e0.elapsed_time(e1) / 10)
        times["torch"] = tt
    fl_ = 2.0 * M * N * K
    res[name] = {(f"v{v}" if v != "torch" else v): {"ms": round(sorted(t)[2], 4), "tflops": round(fl_ / (sorted(t)[2] / 1e3) / 1e12, 1)}
                 for v, t in times.items()}
    res[name]["maxdiff_vs_v1"] = diff
    print(name, json.dumps(res[name]), flush=True)
lib.evt_set_gemm_variant(0)
