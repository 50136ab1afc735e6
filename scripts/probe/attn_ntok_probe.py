"""Round-6 probe: does the 13th query tile of N = 197 (wave 0 of each (image, head) workgroup takes
tiles 0, 4, 8, 12; waves 1-3 take three) cost a full extra tile-time? evt_attention (bf16,
token-major qkv, 512 images x 12 heads) at N = 192 (12 x 12 tiles, 3 per wave), 197 and 208 (13 x 13),
HIP events, median of 5 x 10 launches. Work-proportional timing predicts t192 / t197 = 144 / 169 =
0.85; timing set by the busiest wave predicts 36 / 52 = 0.69. (qkv carries 16 spare rows: round 6
also ran it on a lab build whose K/V staging read rows past N unclamped; r06_attn_ntok_probe.txt.)
    python scripts/probe/attn_ntok_probe.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402

lib = _lib.load_library()
S = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731


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
B, H, DH = 512, 12, 64
res = {}
for N in (192, 197, 208):
    qkv = torch.randn((B * N + 16, 3 * H * DH), generator=g, device="cuda").bfloat16()
    out = torch.empty((B * N, H * DH), dtype=torch.bfloat16, device="cuda")
    ms = timeit(lambda: _lib.check(lib.evt_attention(1, ctypes.c_void_p(qkv.data_ptr()), 3 * H * DH,
                                                     ctypes.c_void_p(out.data_ptr()), H * DH, B, N,
                                                     H, ctypes.c_float(DH ** -0.5), S())))
    res[N] = round(ms * 1e3, 1)
    del qkv, out
res["lib"] = os.environ.get("EVT_LIB", "product")
res["t192/t197"] = round(res[192] / res[197], 3)
res["t208/t197"] = round(res[208] / res[197], 3)
print(json.dumps(res), flush=True)
