"""Attention microbenchmark (DeiT-base shape): evt_attention bf16 B=512 N=197 H=12 timed with
HIP events, against a device-to-device copy of the same bytes (HBM reference)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
_lib.ensure_device(0)
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
B, N, H = int(os.environ.get("B", 512)), 197, int(os.environ.get("H", 12))
qkv = torch.randn((B * N, 3 * H * 64), device="cuda").bfloat16()
out = torch.empty((B * N, H * 64), device="cuda", dtype=torch.bfloat16)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(ts)[2]


run = lambda: _lib.check(lib.evt_attention(1, ctypes.c_void_p(qkv.data_ptr()), 3 * H * 64,  # noqa: E731
                                           ctypes.c_void_p(out.data_ptr()), H * 64, B, N, H,
                                           ctypes.c_float(0.125), S()))
t = timeit(run)
nbytes = qkv.numel() * 2 + out.numel() * 2
dst = torch.empty_like(qkv)
tc = timeit(lambda: dst.copy_(qkv))
print(json.dumps({"var": os.environ.get("EVT_ATTN_VAR", "0"), "attn_us": round(t, 1),
                  "attn_TBps": round(nbytes / t / 1e6, 2), "copy_us": round(tc, 1),
                  "copy_TBps": round(2 * qkv.numel() * 2 / tc / 1e6, 2)}), flush=True)
