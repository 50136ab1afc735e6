"""MXFP8 kernels on the GPU vs the numpy restatement (oracle/mx8_ref.py).

Quantizer and weight packer: bit-exact (bytes and scale dwords). GEMM: against the fp64 product
of the dequantized operands the fp32 output is within 3e-5 x sum|a||w| (the block-scaled MFMA
does not sum its 128 exact fp8 x fp8 x 2^k products in full fp32: measured on the device
|err| <= 1.9e-5 x sum|a||w|, about 2^-16 of one instruction's magnitude, independent of K) and
the bf16 output within bf16 rounding (2^-8 relative) of that; the MX8 output is checked bit-exactly against the quantizer run on the same kernel's fp32
output (same accumulators), and within half an e4m3 ulp of its block (2^-3 amax with the OCP
saturation) of the fp64 result.
"""
import numpy as np
import pytest
import torch

from edgevisiontransformer_amd import _lib
from oracle import mx8_ref
from tests import _ops

pytestmark = pytest.mark.gpu


def _rand(shape, seed, spread=0):
    g = np.random.default_rng(seed)
    x = g.standard_normal(shape)
    if spread:  # per-row dynamic range across 2^-spread .. 2^spread
        x = x * np.exp2(g.integers(-spread, spread + 1, (shape[0], 1)))
    return x.astype(np.float32)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("rows,K,Kpad", [(1, 128, 128), (197, 768, 768), (300, 200, 256),
                                         (1000, 3072, 3072), (64, 40, 128)])
def test_quantize_bit_exact(gpu, dt, rows, K, Kpad):
    x = _rand((rows, K), seed=rows + K, spread=12)
    x[rows // 2, :min(K, 32)] = 0.0                      # an all-zero block
    x[0, :8] = [448.0, 449.0, -511.0, 1e-30, -1e-30, 2.0 ** -140, 0.0, -0.0]  # saturation, denormals
    xt = torch.from_numpy(x).to(gpu).to(_ops.TDT[dt])
    q, s = _ops.mx8_quantize(xt, Kpad=Kpad, ld_s=rows + 3)
    torch.cuda.synchronize()
    xin = xt.float().cpu().numpy()
    qr, sbr = mx8_ref.quantize(xin, Kpad)
    sb = mx8_ref.dwords_to_scales(s.cpu().numpy().view(np.uint32), rows)
    assert np.array_equal(sb, sbr)
    qg = q.cpu().numpy()
    # compare values (bytes up to the sign of zero)
    dq = mx8_ref.e4m3_decode(qr)
    assert np.array_equal(mx8_ref.e4m3_decode(qg), dq)
    assert np.array_equal(qg[dq != 0], qr[dq != 0])


@pytest.mark.parametrize("K,N", [(768, 2304), (200, 136), (3072, 768), (64, 1000)])
def test_pack_weight_bit_exact(gpu, K, N):
    W = _rand((K, N), seed=K * 7 + N) * 0.05
    gamma = 1.0 + 0.1 * _rand((K,), seed=5)
    wq, s, kpad, npad = _ops.mx8_pack(torch.from_numpy(W).to(gpu), torch.from_numpy(gamma).to(gpu))
    torch.cuda.synchronize()
    qr, sbr = mx8_ref.pack_weight(W, kpad, npad, row_scale=gamma)
    sb = mx8_ref.dwords_to_scales(s.cpu().numpy().view(np.uint32), npad)
    assert np.array_equal(sb, sbr)
    qg = wq.cpu().numpy()
    assert np.array_equal(mx8_ref.e4m3_decode(qg), mx8_ref.e4m3_decode(qr))


def _operands(gpu, M, K, N, seed):
    A = _rand((M, K), seed=seed, spread=4)
    W = (_rand((K, N), seed=seed + 1) / np.float32(np.sqrt(K))).astype(np.float32)
    At = torch.from_numpy(A).to(gpu)
    Aq, As = _ops.mx8_quantize(At)
    wq, ws, kpad, npad = _ops.mx8_pack(torch.from_numpy(W).to(gpu))
    torch.cuda.synchronize()
    aq = Aq.cpu().numpy()
    asb = mx8_ref.dwords_to_scales(As.cpu().numpy().view(np.uint32), M)
    wqn = wq.cpu().numpy()
    wsb = mx8_ref.dwords_to_scales(ws.cpu().numpy().view(np.uint32), npad)
    mag = np.abs(mx8_ref.dequantize(aq, asb)) @ np.abs(mx8_ref.dequantize(wqn, wsb)[:N]).T
    return (Aq, As, wq, ws, kpad, npad), (aq, asb, wqn, wsb), mag


SHAPES = [(197, 768, 2304), (300, 256, 136), (128, 128, 128), (1000, 3072, 768), (77, 384, 40),
          (2048, 768, 1024)]


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("flags", [0, 1, 3, 257, 5, 16, 17])
def test_dense_mx8(gpu, M, K, N, flags):
    dev, host, mag = _operands(gpu, M, K, N, seed=M + K + N)
    bias = _rand((N,), seed=3) * 0.1
    resid = _rand((M, N), seed=4)
    resid_t = torch.from_numpy(resid).to(gpu).to(torch.bfloat16)
    out = _ops.dense_mx8(flags, *dev, M, N, bias=torch.from_numpy(bias).to(gpu),
                         resid=resid_t if flags & 4 else None)
    torch.cuda.synchronize()
    ref = mx8_ref.dense_mx8(*host, N, flags, bias=bias,
                            resid=resid_t.float().cpu().numpy() if flags & 4 else None)
    got = out.float().cpu().numpy()
    assert np.all(np.isfinite(got))
    tol = 3e-5 * mag + 1e-30
    if flags & 16:
        assert np.all(np.abs(got - ref) <= tol + 1e-6 * np.abs(ref))
    else:  # bf16 rounding of the output (+ the fp32 GELU / bias arithmetic)
        assert np.all(np.abs(got - ref) <= tol + 2.0 ** -8 * np.abs(ref) + 1e-4)


@pytest.mark.parametrize("M,K,N", [(197, 768, 2304), (1000, 3072, 768), (77, 384, 160)])
@pytest.mark.parametrize("flags", [512, 513, 515, 769])
def test_dense_mx8_out(gpu, M, K, N, flags):
    dev, host, mag = _operands(gpu, M, K, N, seed=2 * M + K + N)
    bias = torch.from_numpy(_rand((N,), seed=6) * 0.1).to(gpu)
    C, Cs = _ops.dense_mx8(flags, *dev, M, N, bias=bias)
    f32 = _ops.dense_mx8((flags & ~_lib.EPI_OUT_MX8) | _lib.EPI_OUT_F32, *dev, M, N, bias=bias)
    q2, s2 = _ops.mx8_quantize(f32)
    torch.cuda.synchronize()
    # the fused epilogue quantizer == the standalone quantizer on the same accumulators
    nb = N // 32
    sg = mx8_ref.dwords_to_scales(Cs.cpu().numpy().view(np.uint32), M)[:, :nb]
    assert np.array_equal(sg, mx8_ref.dwords_to_scales(s2.cpu().numpy().view(np.uint32), M)[:, :nb])
    cg = C.cpu().numpy()
    assert np.array_equal(mx8_ref.e4m3_decode(cg), mx8_ref.e4m3_decode(q2[:, :N].cpu().numpy()))
    # and the dequantized output is within the block quantization error of the fp64 product
    ref = mx8_ref.dense_mx8(*host, N, flags & ~_lib.EPI_OUT_MX8, bias=bias.cpu().numpy())
    deq = mx8_ref.dequantize(cg, sg)
    amax = np.abs(ref).reshape(M, N // 32, 32).max(-1)
    err = np.abs(deq - ref).reshape(M, N // 32, 32).max(-1)
    assert np.all(err <= amax * 2.0 ** -3 + 1e-5)


def test_dense_mx8_rejects(gpu):
    dev, _, _ = _operands(gpu, 64, 128, 128, seed=9)
    with pytest.raises(RuntimeError):
        _ops.dense_mx8(2, *dev, 64, 128)  # GELU without bias: not an instantiated flag set
    with pytest.raises(RuntimeError):
        _ops.dense_mx8(0, *dev, 64, 124)  # N % 8


# ---- kernel-level checks of the MX8 model's fused kernels (LayerNorm quantizer, LN-residual
# epilogue, attention MX8 output). Quantization is a step function, so the device's fp32 values
# and the fp64 restatement can land on different sides of a rounding midpoint (or of a power of
# two for a block's scale); such elements / blocks are identified from the fp64 value and excluded
# from the bit-exact comparison (their fraction is bounded), every other byte must match.
def _near_midpoint(v, dv):
    """v (already divided by the block scale) within +-dv of an e4m3 rounding midpoint."""
    lo = mx8_ref.e4m3_round(np.clip(v - dv, -448, 448).astype(np.float32))
    hi = mx8_ref.e4m3_round(np.clip(v + dv, -448, 448).astype(np.float32))
    return lo != hi


def _check_mx8_against(q, sb, y, dy, max_amb=2e-3):
    """q bytes [R, K] / scale bytes [R, K/32] from the device vs the fp64 values y [R, K], whose
    device-side (fp32 / bf16) counterparts differ from y by at most dy (array or scalar)."""
    R, K = y.shape
    dy = np.broadcast_to(np.asarray(dy, np.float64), y.shape)
    blocks = np.abs(y).reshape(R, K // 32, 32).max(-1)
    dblk = dy.reshape(R, K // 32, 32).max(-1)
    sb_ref = mx8_ref.scale_bytes(blocks.astype(np.float32))
    amb_blk = (mx8_ref.scale_bytes(np.maximum(blocks - dblk, 0).astype(np.float32)) !=
               mx8_ref.scale_bytes((blocks + dblk).astype(np.float32)))
    assert np.array_equal(sb[~amb_blk], sb_ref[~amb_blk])
    inv = np.exp2(127.0 - sb_ref.astype(np.float64))
    v = (y.reshape(R, K // 32, 32) * inv[..., None]).reshape(R, K)
    dv = (dy.reshape(R, K // 32, 32) * inv[..., None]).reshape(R, K)
    qr = mx8_ref.e4m3_encode(mx8_ref.e4m3_round(np.clip(v, -448, 448).astype(np.float32)))
    amb = _near_midpoint(v, dv) | np.repeat(amb_blk, 32, axis=1)
    dg, dr = mx8_ref.e4m3_decode(q), mx8_ref.e4m3_decode(qr)
    assert np.array_equal(dg[~amb], dr[~amb])
    assert amb.mean() <= max_amb, amb.mean()
    # every element (ambiguous ones included) within one e4m3 step of its block
    err = np.abs(mx8_ref.dequantize(q, sb) - y).reshape(R, K // 32, 32).max(-1)
    assert np.all(err <= blocks * 2.0 ** -3 + 1e-30)


@pytest.mark.parametrize("rows,D,Kpad", [(2 * 197 + 3, 192, 256), (301, 320, 384), (999, 768, 768),
                                         (1003, 1024, 1024), (5, 64, 128)])
def test_mx8_layernorm_kernel(gpu, rows, D, Kpad):
    g = np.random.default_rng(rows + D)
    x = (g.standard_normal((rows, D)) * np.exp2(g.integers(-3, 4, (rows, 1)))
         + g.standard_normal((rows, 1))).astype(np.float32)
    x[1, :] = 7.0  # constant row: variance 0 -> rstd = 1/sqrt(eps), LN(x) = beta
    xt = torch.from_numpy(x).to(gpu).to(torch.bfloat16)
    gamma = (1.0 + 0.2 * g.standard_normal(D)).astype(np.float32)
    beta = (0.1 * g.standard_normal(D)).astype(np.float32)
    q, s, st = _ops.mx8_layernorm(xt, torch.from_numpy(gamma).to(gpu),
                                  torch.from_numpy(beta).to(gpu), Kpad)
    torch.cuda.synchronize()
    xb = xt.float().cpu().numpy().astype(np.float64)
    mu = xb.mean(1)
    rstd = 1.0 / np.sqrt(((xb - mu[:, None]) ** 2).mean(1) + 1e-5)
    stg = st.cpu().numpy().astype(np.float64)
    assert np.all(np.abs(stg[:, 0] - mu) <= 1e-6 * (np.abs(mu) + 1.0 / rstd))
    assert np.all(np.abs(stg[:, 1] / rstd - 1.0) <= 1e-5)
    y = np.zeros((rows, Kpad))
    t = (xb - mu[:, None]) * rstd[:, None] * gamma
    y[:, :D] = t + beta
    # fp32 evaluation error of the device's (x - mu) * rstd * gamma + beta (incl. mu's rounding)
    dy = np.zeros((rows, Kpad))
    mu_err = np.where(xb.std(1) > 0, 5e-7 * np.abs(mu), 0.0)  # a constant row's mean is exact
    dy[:, :D] = 2e-6 * (np.abs(t) + np.abs(beta)) + (mu_err * rstd)[:, None] * np.abs(gamma)
    sb = mx8_ref.dwords_to_scales(s.cpu().numpy().view(np.uint32), rows)
    qg = q.cpu().numpy()
    assert np.all(qg[:, D:] & 0x7F == 0) and np.all(sb[:, (D + 31) // 32:] == 0)  # padding = zeros
    _check_mx8_against(qg, sb, y, dy, max_amb=0.01)


def test_mx8_layernorm_rejects(gpu):
    x = torch.zeros((4, 100), dtype=torch.bfloat16, device=gpu)
    gb = torch.ones(128, device=gpu)
    with pytest.raises(RuntimeError):
        _ops.mx8_layernorm(x, gb, gb, 128)  # D % 8
    with pytest.raises(RuntimeError):
        _ops.mx8_layernorm(torch.zeros((4, 256), dtype=torch.bfloat16, device=gpu), gb, gb, 128)


@pytest.mark.parametrize("M,K,N", [(197, 768, 768), (1003, 3072, 768), (77, 384, 192)])
def test_dense_mx8_resln(gpu, M, K, N):
    """Flag set 69 (bias + residual LN(resid) from (mu, rstd)): the MX8 out-proj / FC2 epilogue."""
    dev, host, mag = _operands(gpu, M, K, N, seed=3 * M + K + N)
    g = np.random.default_rng(M)
    bias = (0.1 * g.standard_normal(N)).astype(np.float32)
    resid = (g.standard_normal((M, N)) * 2.0 + 0.5).astype(np.float32)
    rt = torch.from_numpy(resid).to(gpu).to(torch.bfloat16)
    rb = rt.float().cpu().numpy().astype(np.float64)
    mu = rb.mean(1)
    rstd = 1.0 / np.sqrt(((rb - mu[:, None]) ** 2).mean(1) + 1e-5)
    rst = torch.from_numpy(np.stack([mu, rstd], 1).astype(np.float32)).to(gpu)
    gam = (1.0 + 0.2 * g.standard_normal(N)).astype(np.float32)
    bet = (0.1 * g.standard_normal(N)).astype(np.float32)
    out = _ops.dense_mx8(69, *dev, M, N, bias=torch.from_numpy(bias).to(gpu), resid=rt,
                         rstats=rst, rgamma=torch.from_numpy(gam).to(gpu),
                         rbeta=torch.from_numpy(bet).to(gpu))
    torch.cuda.synchronize()
    mu32, r32 = rst.cpu().numpy()[:, 0].astype(np.float64), rst.cpu().numpy()[:, 1].astype(np.float64)
    lnr = (rb - mu32[:, None]) * r32[:, None] * gam + bet
    ref = mx8_ref.dense_mx8(*host, N, 1, bias=bias) + lnr
    got = out.float().cpu().numpy()
    tol = 3e-5 * mag + 2.0 ** -8 * np.abs(ref) + 1e-4 + 1e-5 * np.abs(lnr)
    assert np.all(np.abs(got - ref) <= tol)
    with pytest.raises(RuntimeError):  # RESLN without its statistics
        _ops.dense_mx8(69, *dev, M, N, bias=torch.from_numpy(bias).to(gpu), resid=rt)


def _attn64(qkv, B, N, H, scale=0.125):
    q, k, v = (qkv.reshape(B, N, 3, H, 64)[:, :, i].transpose(0, 2, 1, 3) for i in range(3))
    s = np.einsum("bhid,bhjd->bhij", q, k) * scale
    p = np.exp(s - s.max(-1, keepdims=True))
    p /= p.sum(-1, keepdims=True)
    return np.einsum("bhij,bhjd->bhid", p, v).transpose(0, 2, 1, 3).reshape(B * N, H * 64)


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (3, 197, 3), (1, 50, 6), (2, 129, 2)])
def test_attention_mx8_kernel(gpu, B, N, H):
    g = np.random.default_rng(B * N + H)
    qkv = torch.from_numpy((1.5 * g.standard_normal((B * N, 3 * H * 64))).astype(np.float32))
    qkv = qkv.to(gpu).to(torch.bfloat16)
    q, s = _ops.attention_mx8(qkv, B, N, H)
    o16 = _ops.attention("bf16", qkv, B, N, H)  # same kernel, bf16 output
    torch.cuda.synchronize()
    K = q.shape[1]
    sb = mx8_ref.dwords_to_scales(s.cpu().numpy().view(np.uint32), B * N)[:, :H * 2]
    qg = q.cpu().numpy()[:, :H * 64]
    # layout / scale placement: the MX8 output equals the quantization of the same kernel's bf16
    # output up to that output's own rounding (bf16: <= 2^-9 relative)
    y16 = o16.float().cpu().numpy().astype(np.float64)
    _check_mx8_against(qg, sb, y16, 1.01 * 2.0 ** -9 * np.abs(y16), max_amb=0.1)
    # and both against the fp64 restatement (bf16 P in the PV product: 2e-2 as test_attention)
    ref = _attn64(qkv.float().cpu().numpy().astype(np.float64), B, N, H)
    blocks = np.abs(ref).reshape(B * N, H * 2, 32).max(-1)
    err = np.abs(mx8_ref.dequantize(qg, sb) - ref).reshape(B * N, H * 2, 32).max(-1)
    assert np.all(err <= blocks * 2.0 ** -3 + 2e-2)
    assert K % 128 == 0
