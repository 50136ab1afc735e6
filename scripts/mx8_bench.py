"""Time the MXFP8 GEMM against the bf16 GEMM on the DeiT-base bs512 encoder shapes (1 GPU).

python scripts/mx8_bench.py [--reps 20]  -> one JSON line per shape (us per launch, TFLOP/s)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from edgevisiontransformer_amd import _lib  # noqa: E402
from tests import _ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=512 * 197)
    ap.add_argument("--only", default="", help="comma list of gemm names (qkv,proj,fc1,fc2)")
    ap.add_argument("--no-bf16", action="store_true")
    a = ap.parse_args()
    _lib.ensure_device(0)
    dev = torch.device("cuda", 0)
    M = a.rows
    shapes = [("qkv", 768, 2304, 1, 1), ("proj", 768, 768, 5, 1), ("fc1", 768, 3072, 515, 3),
              ("fc2", 3072, 768, 5, 1)]
    if a.only:
        shapes = [x for x in shapes if x[0] in a.only.split(",")]
    for name, K, N, fmx, fbf in shapes:
        g = torch.Generator(device=dev).manual_seed(K + N)
        x = torch.randn((M, K), device=dev, generator=g)
        W = torch.randn((K, N), device=dev, generator=g) * K ** -0.5
        bias = torch.randn(N, device=dev, generator=g) * 0.1
        resid = torch.randn((M, N), device=dev, generator=g).to(torch.bfloat16)
        Aq, As = _ops.mx8_quantize(x)
        wq, ws, kpad, npad = _ops.mx8_pack(W)
        t_mx = timeit(lambda: _ops.dense_mx8(fmx, Aq, As, wq, ws, kpad, npad, M, N, bias=bias,
                                             resid=resid if fmx & 4 else None), a.reps)
        xb = x.to(torch.bfloat16)
        wp, kp, np_ = _ops.pack(W, "bf16")
        C = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
        t_bf = 1e30 if a.no_bf16 else timeit(lambda: _ops.dense("bf16", fbf, xb, wp, kp, np_, M, N, bias=bias,
                                         resid=resid if fbf & 4 else None, C=C), a.reps)
        t_q = timeit(lambda: _ops.mx8_quantize(x.to(torch.bfloat16) if False else xb), a.reps)
        fl = 2.0 * M * K * N
        print(json.dumps({"gemm": name, "M": M, "K": K, "N": N, "mx8_flags": fmx,
                          "mx8_us": round(t_mx, 1), "mx8_tflops": round(fl / t_mx / 1e6, 1),
                          "bf16_us": round(t_bf, 1), "bf16_tflops": round(fl / t_bf / 1e6, 1),
                          "quantize_bf16_us(incl alloc)": round(t_q, 1)}), flush=True)


if __name__ == "__main__":
    main()
