"""Round-6 reference point: the product attention core (evt_attention, bf16, token-major qkv
[B*N][3*H*64] -> out [B*N][H*64], attention.py:20-34) against torch's scaled_dot_product_attention
backends on ROCm (flash / memory-efficient / math) given contiguous q, k, v [B][H][N][64] (their
best case; the layout transform is not timed). DeiT-base shapes: N = 197, H = 12, B = 512 and 64.
HIP events on torch's current stream, median of 5 x 10 launches.
    python scripts/probe/vendor_attn_bench.py"""
import ctypes
import json
import sys

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

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
H, N, DH = 12, 197, 64
for B in (512, 64):
    qkv = torch.randn((B * N, 3 * H * DH), generator=g, device="cuda").bfloat16()
    out = torch.empty((B * N, H * DH), dtype=torch.bfloat16, device="cuda")
    scale = DH ** -0.5
    # algorithmic bytes: q, k, v read once, o written once
    nbytes = 4 * B * H * N * DH * 2
    flops = 4.0 * B * H * N * N * DH
    res = {"B": B, "N": N, "H": H}
    ms = timeit(lambda: _lib.check(lib.evt_attention(1, ctypes.c_void_p(qkv.data_ptr()), 3 * H * DH,
                                                     ctypes.c_void_p(out.data_ptr()), H * DH, B, N,
                                                     H, ctypes.c_float(scale), S())))
    res["product"] = {"us": round(ms * 1e3, 1), "TB/s": round(nbytes / ms / 1e9, 2),
                      "TFLOP/s": round(flops / ms / 1e9, 1)}
    q, k, v = (qkv.view(B, N, 3, H, DH)[:, :, i].permute(0, 2, 1, 3).contiguous() for i in range(3))
    torch.cuda.synchronize()
    ref = out.view(B, N, H, DH).permute(0, 2, 1, 3).float()
    for name, be in (("flash", SDPBackend.FLASH_ATTENTION), ("efficient", SDPBackend.EFFICIENT_ATTENTION),
                     ("math", SDPBackend.MATH)):
        try:
            with sdpa_kernel([be]):
                o = F.scaled_dot_product_attention(q, k, v, scale=scale)
                torch.cuda.synchronize()
                ms = timeit(lambda: F.scaled_dot_product_attention(q, k, v, scale=scale))
            res[name] = {"us": round(ms * 1e3, 1), "TB/s": round(nbytes / ms / 1e9, 2),
                         "TFLOP/s": round(flops / ms / 1e9, 1),
                         "maxdiff_vs_product": float((o.float() - ref).abs().max())}
        except Exception as e:  # noqa: BLE001 - a backend this build / shape does not support
            res[name] = {"error": str(e).splitlines()[0][:160]}
    print(json.dumps(res), flush=True)
    del qkv, out, q, k, v
    torch.cuda.empty_cache()
