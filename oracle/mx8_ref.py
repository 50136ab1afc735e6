"""CPU restatement (numpy) of the MXFP8 format and the MX8 Dense layer.

TEST INFRASTRUCTURE ONLY: imported by `tests/` alone, never by the product path.

The reference's reduced-precision axis is TFLite post-training quantization (`utils.py:242-294`
tf2tflite with quantization 'float16' / 'dynamic' / 'int8', `tools.py:458-498,826-844`), which
needs TensorFlow (not installed) and targets phone CPUs; the MI355X counterpart is the matrix
cores' block-scaled OCP MX format, so there is no reference output to pin against (parity
unpinned with respect to the reference). What is pinned: the e4m3fn element rounding against
torch's independent `float8_e4m3fn` cast (tests/test_mx8_oracle.py), and the block rule below,
which restates the OCP Microscaling Formats (MX) v1.0 specification:

  * a block is 32 consecutive elements along K of one row;
  * shared scale X = 2^(floor(log2(amax)) - emax_elem), emax_elem = 8 for e4m3
    (largest normal 448 = 1.75 * 2^8), stored as an e8m0 byte 127 + exponent, clamped at 0
    (an all-zero block gets byte 0);
  * elements = e4m3fn(v / X), round-to-nearest-even, saturated to +-448 (|v / X| < 512, so
    saturation only trims (448, 512)).

Storage (include/evt.h): elements q[rows][ldq] bytes; scales k-step-major dwords
S[K / 128][ld_s], byte j of S[ks][r] = block 4 ks + j of row r.
"""
from __future__ import annotations

import numpy as np

E4M3_MAX = 448.0


def e4m3_round(v: np.ndarray) -> np.ndarray:
    """RNE to the e4m3fn grid (values already within +-448), returned as float32."""
    v = np.asarray(v, dtype=np.float32)
    a = np.abs(v).astype(np.float64)
    # exponent of each value (frexp: exact); subnormal range (< 2^-6) has the fixed step 2^-9
    e = np.frexp(np.where(a > 0, a, 1.0))[1] - 1.0
    e = np.maximum(e, -6.0)
    step = np.exp2(e - 3.0)
    q = np.rint(a / step) * step  # np.rint: half to even
    return (np.sign(v) * q).astype(np.float32)


def e4m3_encode(v: np.ndarray) -> np.ndarray:
    """float32 values on the e4m3fn grid -> bytes (sign from the sign bit, so -0 -> 0x80)."""
    v = np.asarray(v, dtype=np.float32)
    sign = (np.signbit(v)).astype(np.uint8) << 7
    a = np.abs(v).astype(np.float64)
    normal = a >= 2.0 ** -6
    e = np.frexp(np.where(normal, a, 1.0))[1] - 1.0
    exp_field = np.where(normal, e + 7, 0).astype(np.int64)
    mant = np.where(normal, a / np.exp2(e) - 1.0, a / 2.0 ** -9)
    mant = np.where(normal, mant * 8.0, mant)
    m = np.rint(mant).astype(np.int64)
    assert np.all(np.abs(mant - m) < 1e-9), "value not on the e4m3 grid"
    return (sign | (exp_field << 3).astype(np.uint8) | m.astype(np.uint8)).astype(np.uint8)


def e4m3_decode(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, dtype=np.uint8).astype(np.int64)
    s = np.where(b & 0x80, -1.0, 1.0)
    ef = (b >> 3) & 0xF
    m = b & 0x7
    val = np.where(ef == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * np.exp2(ef - 7.0))
    val = np.where((ef == 15) & (m == 7), np.nan, val)
    return (s * val).astype(np.float32)


def scale_bytes(amax: np.ndarray) -> np.ndarray:
    """e8m0 scale byte of blocks with absolute maximum amax (float32)."""
    bits = np.asarray(amax, dtype=np.float32).view(np.uint32)
    E = ((bits >> 23) & 0xFF).astype(np.int64)
    return np.maximum(E - 8, 0).astype(np.uint8)


def quantize(x: np.ndarray, Kpad: int | None = None):
    """fp32 rows [R, K] -> (q bytes [R, Kpad], scale bytes [R, Kpad / 32]) per the OCP MX rule,
    the fp32 arithmetic of the device (v * 2^(127 - s), exact power-of-two scaling)."""
    x = np.asarray(x, dtype=np.float32)
    R, K = x.shape
    Kpad = Kpad or K
    xp = np.zeros((R, Kpad), np.float32)
    xp[:, :K] = x
    blocks = xp.reshape(R, Kpad // 32, 32)
    sb = scale_bytes(np.abs(blocks).max(-1))
    inv = np.exp2(127.0 - sb.astype(np.float64)).astype(np.float32)
    v = np.clip(blocks * inv[..., None], -E4M3_MAX, E4M3_MAX)
    q = e4m3_encode(e4m3_round(v)).reshape(R, Kpad)
    return q, sb


def dequantize(q: np.ndarray, sb: np.ndarray) -> np.ndarray:
    R, K = q.shape
    v = e4m3_decode(q).astype(np.float64).reshape(R, K // 32, 32)
    return (v * np.exp2(sb.astype(np.float64) - 127.0)[..., None]).reshape(R, K)


def scales_to_dwords(sb: np.ndarray, ld: int | None = None) -> np.ndarray:
    """scale bytes [R, K / 32] -> the k-step-major dword layout [K / 128, ld] (uint32)."""
    R, nb = sb.shape
    ld = ld or R
    out = np.zeros((nb // 4, ld, 4), np.uint8)
    out[:, :R, :] = sb.reshape(R, nb // 4, 4).transpose(1, 0, 2)
    return out.reshape(nb // 4, ld * 4).view(np.uint32).reshape(nb // 4, ld)


def dwords_to_scales(s: np.ndarray, rows: int) -> np.ndarray:
    """Inverse of scales_to_dwords: [K / 128, ld] dwords -> bytes [rows, K / 32]."""
    nks, ld = s.shape
    b = np.ascontiguousarray(s).view(np.uint8).reshape(nks, ld, 4)[:, :rows, :]
    return b.transpose(1, 0, 2).reshape(rows, nks * 4)


def pack_weight(W: np.ndarray, Kpad: int, Npad: int, row_scale=None):
    """Keras W[K][N] -> (Wq bytes [Npad, Kpad], scale bytes [Npad, Kpad / 32])."""
    K, N = W.shape
    Wt = np.zeros((Npad, Kpad), np.float32)
    w = np.asarray(W, np.float32)
    if row_scale is not None:
        w = (w * np.asarray(row_scale, np.float32)[:, None]).astype(np.float32)
    Wt[:N, :K] = w.T
    return quantize(Wt)


def gelu_tanh(x):
    return 0.5 * x * (1.0 + np.tanh(np.sqrt(2.0 / np.pi) * (x + 0.044715 * x ** 3)))


def gelu_erf(x):
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))


def dense_mx8(Aq, As, Wq, Ws, N, flags, bias=None, resid=None):
    """fp64 epi(dequant(A) . dequant(W)^T) for the evt_dense_mx8 flag sets (output before any
    MX8 re-quantization)."""
    A = dequantize(Aq, As)
    W = dequantize(Wq, Ws)[:N]
    y = A @ W.T
    if flags & 1:
        y = y + np.asarray(bias, np.float64)[:N]
    if flags & 2:
        y = gelu_tanh(y)
    if flags & 256:
        y = gelu_erf(y)
    if flags & 4:
        y = y + np.asarray(resid, np.float64)[:, :N]
    return y
