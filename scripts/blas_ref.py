"""Reference point for the GEMM main loop: hipBLASLt (torch.matmul, bf16) on the DeiT-base encoder
shapes (M = batch * 197), no epilogue fusion, timed with HIP events (median of 20).
    python scripts/blas_ref.py [batch ...]      (default 512 64)"""
import json
import sys

import torch

for B in [int(a) for a in sys.argv[1:]] or [512, 64]:
    M = B * 197
    shapes = {"qkv": (M, 768, 2304), "out_proj": (M, 768, 768), "fc1": (M, 768, 3072),
              "fc2": (M, 3072, 768)}
    out = {"batch": B}
    for name, (m, k, n) in shapes.items():
        a = torch.randn((m, k), device="cuda", dtype=torch.bfloat16)
        w = torch.randn((n, k), device="cuda", dtype=torch.bfloat16)
        for _ in range(5):
            c = a @ w.t()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); c = a @ w.t(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        t = sorted(ts)[len(ts) // 2]
        out[name] = {"us": round(t, 1), "tflops": round(2 * m * k * n / t / 1e6, 1)}
    print(json.dumps(out), flush=True)
