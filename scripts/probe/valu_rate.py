"""Driver of valu_rate.hip: cycles per wave-instruction per SIMD for the epilogue's VALU ops at
1, 2 and 4 waves per SIMD (every CU busy).   python scripts/probe/valu_rate.py"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(HERE, "valu_rate.so"))
OPS = ["v_fma_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_pk_fma_f16", "v_exp_f32",
       "v_exp_f16", "v_rcp_f32", "v_mul_f32", "v_med3_f32", "v_pk_mul_f16", "v_rcp_f16",
       "v_cvt_pk_bf16_f32", "v_add_f32"]
out = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
ms = ctypes.c_float()
iters = 2000
for k, name in enumerate(OPS):
    row = []
    for w in (1, 2, 4):
        lib.valu_run(k, w, 200, ctypes.c_void_p(out.data_ptr()), ctypes.byref(ms))  # warm
        rc = lib.valu_run(k, w, iters, ctypes.c_void_p(out.data_ptr()), ctypes.byref(ms))
        torch.cuda.synchronize()
        assert rc == 0, rc
        cyc = out.view(256, 16)[:, :4 * w].float().median().item()
        row.append(f"{w}/SIMD {cyc * w / (iters * 8):5.2f} cyc ({ms.value * 1e3:7.1f} us)")
    print(f"{name:18s}", "  ".join(row), flush=True)
