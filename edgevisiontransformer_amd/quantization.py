"""MXFP8 quantized Dense layers on the MI355X block-scaled matrix cores.

The reference's reduced-precision axis is post-training quantization of the Keras model through
the TFLite converter (`utils.py:242-294` tf2tflite(quantization='float16' | 'dynamic' | 'int8'),
driven by `tools.py:458-498,826-844`): weights (and for 'int8' activations) stored in 8 bits,
computed by phone-CPU kernels. On MI355X the 8-bit format the matrix cores consume natively is
OCP MX FP8 (e4m3 elements + one power-of-two scale per 32 values, include/evt.h): weights are
quantized once at construction ('dynamic' analogue), activations per call by a HIP kernel (the
'int8' analogue, with per-block instead of calibrated per-tensor scales, so no representative
dataset is needed), and the product runs on v_mfma_scale_f32_16x16x128_f8f6f4 with fp32
accumulation and the bias / GELU / residual epilogue fused.

    dense = MX8Dense(W, bias, activation="gelu")   # W: Keras kernel [in, out]
    y = dense(x)                                    # x: [rows, in] bf16/fp32 -> [rows, out] bf16

No CPU fallback: every call goes through libevt_hip.so (fails loudly without it).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

_ACT = {None: 0, "linear": 0, "gelu": _lib.EPI_GELU, "gelu_erf": _lib.EPI_GELU_ERF}


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def _aligned_rows(t: torch.Tensor) -> torch.Tensor:
    """The kernels read rows with 16-B vector loads: rows must be contiguous, 16-B aligned and a
    multiple of 16 B apart. A view that is not (e.g. a column slice) is copied."""
    esz = t.element_size()
    if t.stride(-1) != 1 or t.data_ptr() % 16 or (t.dim() == 2 and (t.stride(0) * esz) % 16):
        t = t.contiguous()
        if t.data_ptr() % 16 or (t.dim() == 2 and (t.stride(0) * esz) % 16):
            raise ValueError("MX8: rows must be 16-B aligned (row width a multiple of 16 bytes)")
    return t


class MX8Tensor:
    """An MX8 matrix on the device: e4m3 bytes q [rows, Kpad] and scale dwords [Kpad/128, rows]."""

    def __init__(self, q: torch.Tensor, scales: torch.Tensor, cols: int):
        self.q, self.scales, self.cols = q, scales, cols

    @property
    def rows(self) -> int:
        return self.q.shape[0]


def quantize_mx8(x: torch.Tensor) -> MX8Tensor:
    """[rows, K] bf16 / fp32 device tensor (K % 8 == 0, rows 16-B aligned) -> MX8Tensor."""
    if x.dim() != 2 or not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float32):
        raise ValueError("quantize_mx8: expects a 2-D bf16 / fp32 device tensor")
    rows, K = x.shape
    if K % 8:
        raise ValueError("quantize_mx8: K must be a multiple of 8")
    x = _aligned_rows(x)
    _lib.ensure_device(x.device.index or 0)
    kpad = _round_up(K, 128)
    q = torch.empty((rows, kpad), dtype=torch.uint8, device=x.device)
    s = torch.empty((kpad // 128, max(rows, 1)), dtype=torch.int32, device=x.device)
    dt = _lib.DTYPE["bf16"] if x.dtype == torch.bfloat16 else _lib.DTYPE["f32"]
    _lib.check(_lib.load_library().evt_mx8_quantize(
        dt, _ptr(x), x.stride(0), rows, K, kpad, _ptr(q), q.stride(0), _ptr(s), s.shape[1],
        ctypes.c_void_p(_lib.stream_ptr(x.device))))
    return MX8Tensor(q, s, K)


class MX8Dense:
    """tf.keras.layers.Dense(units, activation) with MXFP8 weights and activations.

    W: Keras kernel [in, out] (fp32, any device: copied to `device`), bias [out] or None.
    activation: None / 'linear', 'gelu' (tanh form, reference activation.py:13-15) or 'gelu_erf'.
    __call__(x, residual=None, out_dtype=torch.bfloat16): x is [rows, in] bf16/fp32 or an
    MX8Tensor; residual [rows, out] bf16 is added after the activation (residual.py:9).
    """

    def __init__(self, W: torch.Tensor, bias: Optional[torch.Tensor] = None,
                 activation: Optional[str] = None, device=None):
        if W.dim() != 2:
            raise ValueError("MX8Dense: W must be [in, out]")
        if activation not in _ACT:
            raise ValueError(f"MX8Dense: unsupported activation {activation!r}")
        self.K, self.N = int(W.shape[0]), int(W.shape[1])
        if self.N % 8:
            raise ValueError("MX8Dense: units must be a multiple of 8")
        if bias is None:  # every instantiated epilogue with an activation / residual has a bias
            bias = torch.zeros(self.N)
        self.device = torch.device(device) if device is not None else torch.device("cuda", 0)
        _lib.ensure_device(self.device.index or 0)
        self.activation = activation
        self.kpad, self.npad = _round_up(self.K, 128), _round_up(self.N, 128)
        w = W.detach().to(self.device, torch.float32).contiguous()
        self.wq = torch.empty((self.npad, self.kpad), dtype=torch.uint8, device=self.device)
        self.ws = torch.empty((self.kpad // 128, self.npad), dtype=torch.int32, device=self.device)
        _lib.check(_lib.load_library().evt_mx8_pack_weight(
            _ptr(w), None, self.K, self.N, _ptr(self.wq), self.kpad, self.npad, _ptr(self.ws),
            ctypes.c_void_p(_lib.stream_ptr(self.device))))
        self.bias = bias.detach().to(self.device, torch.float32).contiguous()

    def __call__(self, x, residual: Optional[torch.Tensor] = None,
                 out_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
        xq = x if isinstance(x, MX8Tensor) else quantize_mx8(x)
        if xq.cols != self.K:
            raise ValueError(f"MX8Dense: input has {xq.cols} features, expected {self.K}")
        M = xq.rows
        flags = _ACT[self.activation] | (_lib.EPI_BIAS if self.bias is not None else 0)
        if residual is not None:
            if residual.shape != (M, self.N) or residual.dtype != torch.bfloat16:
                raise ValueError("MX8Dense: residual must be [rows, units] bf16")
            if flags & (_lib.EPI_GELU | _lib.EPI_GELU_ERF) or out_dtype != torch.bfloat16:
                raise ValueError("MX8Dense: residual fuses with a linear bf16-output layer only")
            residual = _aligned_rows(residual)
            flags |= _lib.EPI_RESID
        if out_dtype == torch.float32:
            flags |= _lib.EPI_OUT_F32
        elif out_dtype != torch.bfloat16:
            raise ValueError("MX8Dense: out_dtype is bf16 or fp32")
        C = torch.empty((M, self.N), dtype=out_dtype, device=self.device)
        a = _lib.evt_dense_mx8_args()
        a.flags, a.A, a.lda = flags, xq.q.data_ptr(), xq.q.stride(0)
        a.a_scales, a.ld_as = xq.scales.data_ptr(), xq.scales.shape[1]
        a.Wq, a.Kpad, a.Npad, a.w_scales = self.wq.data_ptr(), self.kpad, self.npad, self.ws.data_ptr()
        a.C, a.ldc, a.M, a.N = C.data_ptr(), C.stride(0), M, self.N
        a.bias = self.bias.data_ptr() if self.bias is not None else None
        a.resid = residual.data_ptr() if residual is not None else None
        a.ldr = residual.stride(0) if residual is not None else 0
        _lib.check(_lib.load_library().evt_dense_mx8(ctypes.byref(a),
                                                     ctypes.c_void_p(_lib.stream_ptr(self.device))))
        return C

    def quantized_output(self, x) -> MX8Tensor:
        """Same layer with the result re-quantized to MX8 in the epilogue (feeds the next MX8Dense,
        e.g. FC1 -> FC2 of the FeedForward, ffn.py:8-9). Requires units % 32 == 0."""
        if self.N % 32:
            raise ValueError("MX8Dense: MX8 output needs units % 32 == 0")
        xq = x if isinstance(x, MX8Tensor) else quantize_mx8(x)
        M = xq.rows
        flags = _ACT[self.activation] | _lib.EPI_OUT_MX8 | (_lib.EPI_BIAS if self.bias is not None else 0)
        # K-padded to 128 like every MX8Tensor; padding columns stay zero with scale byte 0
        q = torch.zeros((M, self.npad), dtype=torch.uint8, device=self.device)
        s = torch.zeros((self.npad // 128, max(M, 1)), dtype=torch.int32, device=self.device)
        a = _lib.evt_dense_mx8_args()
        a.flags, a.A, a.lda = flags, xq.q.data_ptr(), xq.q.stride(0)
        a.a_scales, a.ld_as = xq.scales.data_ptr(), xq.scales.shape[1]
        a.Wq, a.Kpad, a.Npad, a.w_scales = self.wq.data_ptr(), self.kpad, self.npad, self.ws.data_ptr()
        a.C, a.ldc, a.c_scales, a.ld_cs = q.data_ptr(), q.stride(0), s.data_ptr(), s.shape[1]
        a.M, a.N = M, self.N
        a.bias = self.bias.data_ptr() if self.bias is not None else None
        _lib.check(_lib.load_library().evt_dense_mx8(ctypes.byref(a),
                                                     ctypes.c_void_p(_lib.stream_ptr(self.device))))
        return MX8Tensor(q, s, self.N)
