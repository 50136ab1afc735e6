"""Stream-K persistent GEMM (gemm.hip, gemm_sk_kernel): the four encoder GEMM shapes with their
fused epilogues, at token counts large enough (>= #CUs 256x256 tiles) for the K-iteration split
to cut tiles in two. Checked three ways: against a plain PyTorch fp32 reference of the same op
(bf16 tolerance), against the tile-persistent kernel (variant 9; only the split tiles may differ,
by fp32 reassociation before the bf16 rounding), and run twice for bitwise-identical output (the
hand-off flags are left at zero by every launch)."""
import math

import pytest
import torch

from edgevisiontransformer_amd import _lib
from tests import _ops

pytestmark = pytest.mark.gpu

EPI = _lib


def _randn(shape, seed, scale=1.0, dev="cuda"):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randn(shape, generator=g, device=dev) * scale


def _stats(xq):
    S = 2 * ((xq.shape[-1] + 255) // 256)
    st = torch.zeros((xq.shape[0], S, 2), dtype=torch.float32, device=xq.device)
    xf = xq.float()
    st[:, 0, 0], st[:, 0, 1] = xf.sum(-1), (xf * xf).sum(-1)
    return st


def _ln(x, g, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) * torch.rsqrt(var + eps) * g + b


def _gelu(x):
    return x * 0.5 * (1.0 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x ** 3)))


def _run(variant, fn):
    lib = _lib.load_library()
    lib.evt_set_gemm_variant(variant)
    try:
        out = fn()
        torch.cuda.synchronize()
    finally:
        lib.evt_set_gemm_variant(0)
    return out


# (M, K, N): 22100 token rows = 87 M tiles (ragged last tile) -> 261 .. 1044 tiles of 256x256
@pytest.mark.parametrize("M,D,N,gelu", [(22100, 768, 2304, False), (22100, 768, 3072, True),
                                        (30000, 384, 1536, True)])
def test_streamk_layernorm_folded_input(gpu, M, D, N, gelu):
    """QKV / FC1 shape: LN1/LN2 folded (raw stream in, per-row statistics in the epilogue)."""
    x = (_randn((M, D), 1, 1.3) + 0.3).bfloat16()
    g, be = 1.0 + _randn((D,), 2, 0.1), _randn((D,), 3, 0.1)
    W, bias = _randn((D, N), 4, 1 / math.sqrt(D)), _randn((N,), 5, 0.05)
    wp, kpad, npad = _ops.pack(W, "bf16", row_scale=g)
    colsum, cvec = _ops.ln_fold("bf16", wp, kpad, npad, W, be, bias)
    flags = EPI.EPI_LNIN | EPI.EPI_BIAS | (EPI.EPI_GELU if gelu else 0)
    st = _stats(x)

    def call():
        return _ops.dense("bf16", flags, x, wp, kpad, npad, M, N, bias=cvec, colsum=colsum,
                          stats_in=st, ln_width=D)

    sk = _run(16, call)
    sk2 = _run(16, call)
    pers = _run(9, call)
    assert torch.equal(sk, sk2), "stream-K output must be reproducible launch to launch"
    torch.testing.assert_close(sk.float(), pers.float(), rtol=8e-3, atol=8e-3)
    ref = _ln(x.float(), g, be) @ W + bias
    if gelu:
        ref = _gelu(ref)
    torch.testing.assert_close(sk.float(), ref, rtol=2.5e-2, atol=2.5e-2)
    del ref


@pytest.mark.parametrize("M,K,D", [(22100, 768, 768), (22100, 3072, 768), (33000, 1536, 384)])
def test_streamk_layernorm_residual_and_stats(gpu, M, K, D):
    """out-proj / FC2 shape: + bias + LN(resid) residual, new stream + its row statistics."""
    A = _randn((M, K), 11).bfloat16()
    W, b = _randn((K, D), 12, 1 / math.sqrt(K)), _randn((D,), 13, 0.1)
    x = (_randn((M, D), 14, 1.1) - 0.2).bfloat16()
    g, be = 1.0 + _randn((D,), 15, 0.1), _randn((D,), 16, 0.1)
    wp, kpad, npad = _ops.pack(W, "bf16")
    bias = torch.zeros(npad, device=A.device)
    bias[:D] = b
    S = 2 * ((D + 255) // 256)
    rst = _stats(x)
    outs = {}

    def call(tag):
        def f():
            so = torch.full((M, S, 2), float("nan"), device=A.device)
            C = _ops.dense("bf16", EPI.EPI_BIAS | EPI.EPI_RESID | EPI.EPI_RESLN | EPI.EPI_STATS, A,
                           wp, kpad, npad, M, D, bias=bias, resid=x, rstats=rst, rgamma=g,
                           rbeta=be, stats_out=so, ln_width=D)
            outs[tag] = so
            return C
        return f

    sk = _run(16, call("sk"))
    sk2 = _run(16, call("sk2"))
    pers = _run(9, call("pers"))
    assert torch.equal(sk, sk2) and torch.equal(outs["sk"], outs["sk2"])
    torch.testing.assert_close(sk.float(), pers.float(), rtol=8e-3, atol=8e-3)
    ref = A.float() @ W.bfloat16().float() + b + _ln(x.float(), g, be)
    torch.testing.assert_close(sk.float(), ref, rtol=2e-2, atol=2e-2)
    # statistics are of the values as stored, every slot written (no NaN left)
    got = sk.float()
    so = outs["sk"]
    assert not torch.isnan(so).any()
    torch.testing.assert_close(so.sum(1)[:, 0], got.sum(-1), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(so.sum(1)[:, 1], (got * got).sum(-1), rtol=1e-4, atol=1e-2)
