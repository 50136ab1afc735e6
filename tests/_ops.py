"""Thin test helpers that call the op-level C ABI (include/evt.h) on torch device tensors."""
from __future__ import annotations

import ctypes

import torch

from edgevisiontransformer_amd import _lib

TDT = {"f32": torch.float32, "bf16": torch.bfloat16}


def _p(t):
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def round_up(x, m):
    return (x + m - 1) // m * m


def pack(W: torch.Tensor, dtype: str, row_scale: torch.Tensor = None) -> tuple:
    """Keras [K, N] fp32 (device) -> packed [Npad][Kpad] (optionally rows scaled by gamma)."""
    K, N = W.shape
    kpad, npad = round_up(K, 64), round_up(N, 256)
    wp = torch.empty((npad, kpad), dtype=TDT[dtype], device=W.device)
    _lib.check(_lib.load_library().evt_pack_weight(_lib.DTYPE[dtype], _p(W.contiguous()),
                                                    _p(row_scale), K, N, _p(wp), kpad, npad, _s()))
    return wp, kpad, npad


def ln_fold(dtype, wp, kpad, npad, W, beta, bias=None):
    K, N = W.shape
    colsum = torch.empty(npad, device=W.device)
    cvec = torch.empty(npad, device=W.device)
    _lib.check(_lib.load_library().evt_ln_fold(_lib.DTYPE[dtype], _p(wp), kpad, npad,
                                                _p(W.contiguous()), _p(beta), _p(bias), K, N,
                                                _p(colsum), _p(cvec), _s()))
    return colsum, cvec


def dense(dtype, flags, A, wp, kpad, npad, M, N, ldc=None, bias=None, resid=None, pos=None, P=0,
          C=None, colsum=None, stats_in=None, rstats=None, rgamma=None, rbeta=None,
          stats_out=None, ln_width=0, ln_eps=1e-5):
    out_f32 = bool(flags & _lib.EPI_OUT_F32)
    ldc = ldc or N
    if C is None:
        rows = M if not (flags & _lib.EPI_POS) else (M // P) * (P + 1)
        C = torch.zeros((rows, ldc), dtype=torch.float32 if out_f32 else TDT[dtype], device=A.device)
    a = _lib.evt_dense_args()
    a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = flags, A.data_ptr(), A.stride(0), wp.data_ptr(), kpad, npad
    a.C, a.ldc, a.M, a.N = C.data_ptr(), ldc, M, N
    for name, t in (("bias", bias), ("resid", resid), ("pos", pos), ("colsum", colsum),
                    ("stats_in", stats_in), ("rstats", rstats), ("rgamma", rgamma),
                    ("rbeta", rbeta), ("stats_out", stats_out)):
        setattr(a, name, t.data_ptr() if t is not None else None)
    a.ldr = resid.stride(0) if resid is not None else 0
    a.ldp = pos.stride(0) if pos is not None else 0
    a.P, a.ln_width, a.ln_eps = P, ln_width, ln_eps
    _lib.check(_lib.load_library().evt_dense(_lib.DTYPE[dtype], ctypes.byref(a), _s()))
    return C


def dense_splitk(dtype, flags, A, wp, kpad, npad, M, N, splits, bias=None, C=None):
    """evt_dense_splitk: the classifier head's K-split Dense (fp32 partials, fixed-order reduce)."""
    out_f32 = bool(flags & _lib.EPI_OUT_F32)
    if C is None:
        C = torch.zeros((M, N), dtype=torch.float32 if out_f32 else TDT[dtype], device=A.device)
    part = torch.full((splits, M, npad), float("nan"), device=A.device)
    a = _lib.evt_dense_args()
    a.flags, a.A, a.lda, a.Wp, a.Kpad, a.Npad = flags, A.data_ptr(), A.stride(0), wp.data_ptr(), kpad, npad
    a.C, a.ldc, a.M, a.N = C.data_ptr(), C.stride(0), M, N
    a.bias = bias.data_ptr() if bias is not None else None
    _lib.check(_lib.load_library().evt_dense_splitk(_lib.DTYPE[dtype], ctypes.byref(a), splits,
                                                     _p(part), _s()))
    return C


def attention(dtype, qkv, B, N, H, scale=0.125, out=None):
    if out is None:
        out = torch.zeros((B * N, H * 64), dtype=TDT[dtype], device=qkv.device)
    _lib.check(_lib.load_library().evt_attention(_lib.DTYPE[dtype], _p(qkv), qkv.stride(0), _p(out),
                                                 out.stride(0), B, N, H, scale, _s()))
    return out


def attention_hd(dtype, qkv, B, N, H, hd, scale=None, out=None):
    """evt_attention_hd: any head size hd (attention.py:6-12); scale defaults to hd^-0.5."""
    if out is None:
        out = torch.zeros((B * N, H * hd), dtype=TDT[dtype], device=qkv.device)
    if scale is None:
        scale = hd ** -0.5
    _lib.check(_lib.load_library().evt_attention_hd(_lib.DTYPE[dtype], _p(qkv), qkv.stride(0),
                                                    _p(out), out.stride(0), B, N, H, hd, scale,
                                                    _s()))
    return out


def layernorm(dtype, x, gamma, beta, eps=1e-5):
    rows, D = x.shape
    y = torch.empty((rows, D), dtype=TDT[dtype], device=x.device)
    _lib.check(_lib.load_library().evt_layernorm(_lib.DTYPE[dtype], _p(x), x.stride(0), _p(y),
                                                 y.stride(0), _p(gamma), _p(beta), rows, D, eps,
                                                 _s()))
    return y


def patchify(dtype, img, ps, cls, pos, D, channel_major=False):
    """evt_patchify ((p1 p2 c) vectors) or, channel_major, evt_patchify_cm ((c p1 p2))."""
    B, C, HW, _ = img.shape
    P = (HW // ps) ** 2
    out = torch.empty((B * P, ps * ps * C), dtype=TDT[dtype], device=img.device)
    x = torch.zeros((B * (P + 1), D), dtype=TDT[dtype], device=img.device)
    stats = torch.full((B * (P + 1), 2 * ((D + 255) // 256), 2), -1.0, device=img.device)
    lib = _lib.load_library()
    fn = lib.evt_patchify_cm if channel_major else lib.evt_patchify
    _lib.check(fn(_lib.DTYPE[dtype], _p(img), B, C, HW, ps, _p(out), _p(x), _p(cls), _p(pos), D,
                  _p(stats), _s()))
    return out, x, stats


# ---- MXFP8 (evt_mx8_*) ----
def mx8_quantize(x: torch.Tensor, Kpad: int = None, ld_s: int = None):
    """rows x K (bf16 / f32 device tensor) -> (q uint8 [rows, Kpad], scale dwords [Kpad/128, ld_s])."""
    rows, K = x.shape
    Kpad = Kpad or round_up(K, 128)
    ld_s = ld_s or rows
    q = torch.full((rows, Kpad), 0x7F, dtype=torch.uint8, device=x.device)  # NaN fill: all written
    s = torch.full((Kpad // 128, ld_s), 0x7F7F7F7F, dtype=torch.int32, device=x.device)
    dt = 1 if x.dtype == torch.bfloat16 else 0
    _lib.check(_lib.load_library().evt_mx8_quantize(dt, _p(x), x.stride(0), rows, K, Kpad, _p(q),
                                                    q.stride(0), _p(s), ld_s, _s()))
    return q, s


def mx8_pack(W: torch.Tensor, row_scale: torch.Tensor = None):
    K, N = W.shape
    kpad, npad = round_up(K, 128), round_up(N, 128)
    wq = torch.full((npad, kpad), 0x7F, dtype=torch.uint8, device=W.device)
    s = torch.full((kpad // 128, npad), 0x7F7F7F7F, dtype=torch.int32, device=W.device)
    _lib.check(_lib.load_library().evt_mx8_pack_weight(_p(W.contiguous()), _p(row_scale), K, N,
                                                       _p(wq), kpad, npad, _p(s), _s()))
    return wq, s, kpad, npad


def mx8_layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, Kpad: int,
                  eps: float = 1e-5):
    """bf16 rows [rows, D] -> (q uint8 [rows, Kpad], scale dwords [Kpad/128, rows],
    (mu, rstd) fp32 [rows, 2]) through evt_mx8_layernorm."""
    rows, D = x.shape
    q = torch.full((rows, Kpad), 0x7F, dtype=torch.uint8, device=x.device)  # NaN fill: all written
    s = torch.full((Kpad // 128, rows), 0x7F7F7F7F, dtype=torch.int32, device=x.device)
    st = torch.full((rows, 2), float("nan"), dtype=torch.float32, device=x.device)
    _lib.check(_lib.load_library().evt_mx8_layernorm(_p(x), rows, D, Kpad, _p(gamma), _p(beta), eps,
                                                     _p(st), _p(q), _p(s), _s()))
    return q, s, st


def attention_mx8(qkv: torch.Tensor, B: int, N: int, H: int, scale: float = 0.125):
    """bf16 qkv [B*N, 3*H*64] -> MX8 O (q uint8 [B*N, ldq8], scale dwords [ldq8/128, B*N])."""
    ldq8 = round_up(H * 64, 128)
    q = torch.full((B * N, ldq8), 0x7F, dtype=torch.uint8, device=qkv.device)
    s = torch.full((ldq8 // 128, B * N), 0x7F7F7F7F, dtype=torch.int32, device=qkv.device)
    _lib.check(_lib.load_library().evt_attention_mx8(_p(qkv), qkv.stride(0), _p(q), ldq8, _p(s),
                                                     B * N, B, N, H, scale, _s()))
    return q, s


def dense_mx8(flags, Aq, As, wq, ws, kpad, npad, M, N, bias=None, resid=None, rstats=None,
              rgamma=None, rbeta=None):
    a = _lib.evt_dense_mx8_args()
    a.flags, a.A, a.lda, a.a_scales, a.ld_as = flags, Aq.data_ptr(), Aq.stride(0), As.data_ptr(), As.shape[1]
    a.Wq, a.Kpad, a.Npad, a.w_scales = wq.data_ptr(), kpad, npad, ws.data_ptr()
    a.M, a.N = M, N
    Cs = None
    if flags & _lib.EPI_OUT_MX8:
        C = torch.full((M, N), 0x7F, dtype=torch.uint8, device=Aq.device)
        Cs = torch.full((N // 128 if N % 128 == 0 else N // 128 + 1, M), 0x7F7F7F7F,
                        dtype=torch.int32, device=Aq.device)
        a.c_scales, a.ld_cs = Cs.data_ptr(), M
    else:
        C = torch.zeros((M, N), dtype=torch.float32 if flags & _lib.EPI_OUT_F32 else torch.bfloat16,
                        device=Aq.device)
    a.C, a.ldc = C.data_ptr(), C.stride(0)
    a.bias = bias.data_ptr() if bias is not None else None
    a.resid = resid.data_ptr() if resid is not None else None
    a.ldr = resid.stride(0) if resid is not None else 0
    a.rstats, a.rgamma, a.rbeta = (t.data_ptr() if t is not None else None
                                   for t in (rstats, rgamma, rbeta))
    _lib.check(_lib.load_library().evt_dense_mx8(ctypes.byref(a), _s()))
    return (C, Cs) if Cs is not None else C


