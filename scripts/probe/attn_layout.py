"""Does the attention kernel's HBM rate depend on the qkv layout? Same bytes, same arithmetic:
  token-major  qkv [B*N][3*H*64] (the QKV GEMM's output today: a head's K rows are 128-B pieces at a
               4,608-B stride at DeiT-base),
  head-major   qkv [B*H*N][3*64] (every (image, head) slice one contiguous 75 KB run: evt_attention
               with B' = B*H images of one head),
timed back to back with HIP events on the launching stream (DeiT-base bs512 shape by default).
    python scripts/probe/attn_layout.py"""
import os

import torch

from tests import _ops

B = int(os.environ.get("BATCH", "512"))
N, H = 197, 12
qa = torch.randn((B * N, 3 * H * 64), device="cuda").to(torch.bfloat16)
oa = torch.empty((B * N, H * 64), device="cuda", dtype=torch.bfloat16)
qb = torch.randn((B * H * N, 3 * 64), device="cuda").to(torch.bfloat16)
ob = torch.empty((B * H * N, 64), device="cuda", dtype=torch.bfloat16)
s = torch.cuda.current_stream()


def run(f, n=30):
    for _ in range(5):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        f()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


byt = (qa.numel() + oa.numel()) * 2
for rnd in range(3):
    ta = run(lambda: _ops.attention("bf16", qa, B, N, H, out=oa))
    tb = run(lambda: _ops.attention("bf16", qb, B * H, N, 1, out=ob))
    print(f"round {rnd}: token-major {ta:7.1f} us ({byt / ta / 1e6:5.2f} TB/s)   "
          f"head-major {tb:7.1f} us ({byt / tb / 1e6:5.2f} TB/s)", flush=True)
