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
