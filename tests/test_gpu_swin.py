"""GPU parity of the Swin path: the whole forward against the HF-produced fp64 goldens
(tests/golden/make_golden_swin.py, pinned by the numpy oracle), and the window-attention and
patch-merge kernels against the oracle on identical rounded inputs.

Tolerances: f32 path max-abs <= 1e-3 on logits; bf16 path max-abs <= 3e-2 and per-row cosine
>= 0.9995 (as for DeiT). Kernel tests: f32 within 2e-5, bf16 within 3e-2 (bf16
output rounding of O ~ 4e-3 relative plus bf16 P) of the fp64 restatement.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from edgevisiontransformer_amd import _lib
from edgevisiontransformer_amd.modeling.models.swin import SwinTransformer
from edgevisiontransformer_amd.weights import make_images, make_swin_params, swin_config
from oracle import swin_ref
from tests._ops import TDT, _p, _s
from tests.test_swin_oracle import golden_case

pytestmark = pytest.mark.gpu


def _model(cfg, dtype, params, gpu, **kw):
    return SwinTransformer(img_size=cfg.image_size, patch_size=cfg.patch_size,
                           num_classes=cfg.num_classes, embed_dim=cfg.embed_dim,
                           depths=cfg.depths, num_heads=cfg.num_heads, dtype=dtype,
                           weights=params, device=gpu, **kw)


def _cos_rows(a, b):
    return (a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))


@pytest.mark.parametrize("name", ["swin_micro_b2", "swin_tiny_b1", "swin_base_micro_b3"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_swin_golden(gpu, name, dtype):
    z, cfg, params, img = golden_case(name)
    m = _model(cfg, dtype, params, gpu)
    out = m(torch.from_numpy(img).to(gpu)).cpu().numpy().astype(np.float64)
    err = np.abs(out - z["logits"]).max()
    if dtype == "f32":
        assert err <= 1e-3, f"{name} f32 max-abs {err:.3e}"
    else:
        assert err <= 3e-2, f"{name} bf16 max-abs {err:.3e}"
        assert _cos_rows(out, z["logits"]).min() >= 0.9995


def test_swin_batch_independence_and_graph(gpu):
    """Image i's logits do not depend on its batch neighbours (bitwise), and a HIP-graph replay
    reproduces the eager forward bitwise."""
    cfg = swin_config("tiny", image_size=56, depths=(2, 2), num_heads=(3, 6), num_classes=37)
    params = make_swin_params(cfg, seed=5)
    m = _model(cfg, "bf16", params, gpu, max_batch=20)
    img = torch.from_numpy(make_images(20, seed=6, image_size=56)).to(gpu)
    full = m(img)
    part = m(img[7:10].contiguous())
    assert torch.equal(full[7:10], part)
    logits = torch.empty_like(full)
    m.capture_graph(img, logits)
    m.replay_graph()
    torch.cuda.synchronize()
    assert torch.equal(logits, full)


def _window_case(dtype, R, H, shift, B, gpu, seed=0):
    rng = np.random.default_rng(seed)
    C = 32 * H
    ldo = (C + 63) // 64 * 64
    qkv = rng.standard_normal((B * R * R, 3 * C)).astype(np.float32)
    rpb = (rng.standard_normal((169, H)) * 0.5).astype(np.float32)
    tq = torch.from_numpy(qkv).to(gpu).to(TDT[dtype])
    out = torch.full((B * R * R, ldo), float("nan"), dtype=TDT[dtype], device=gpu)
    trpb = torch.from_numpy(rpb).to(gpu)
    _lib.check(_lib.load_library().evt_window_attention(
        _lib.DTYPE[dtype], _p(tq), 3 * C, _p(out), ldo, _p(trpb), B, R, C, H, shift, _s()))
    torch.cuda.synchronize()
    q64 = tq.float().cpu().numpy().astype(np.float64)  # the rounded inputs the kernel saw
    ref = [_oracle_core(q64[b * R * R:(b + 1) * R * R], R, H, shift, rpb.astype(np.float64))
           for b in range(B)]
    return out.float().cpu().numpy(), np.concatenate(ref), C, ldo


def _oracle_core(qkv, R, H, s, rpb):
    """swin_ref.window_attention's core on precomputed (q|k|v) rows (no Linear layers)."""
    C = qkv.shape[1] // 3
    hd = C // H
    x = qkv.reshape(R, R, 3 * C)
    if s:
        x = np.roll(x, (-s, -s), axis=(0, 1))
    nw = R // 7
    win = x.reshape(nw, 7, nw, 7, 3 * C).transpose(0, 2, 1, 3, 4).reshape(nw * nw, 49, 3, H, hd)
    q, k, v = (win[:, :, i].transpose(0, 2, 1, 3) for i in range(3))
    att = np.einsum("whid,whjd->whij", q, k) * hd ** -0.5
    bias = rpb[swin_ref.relative_position_index(7).reshape(-1)].reshape(49, 49, H)
    att = att + bias.transpose(2, 0, 1)[None]
    if s:
        att = att + swin_ref.shift_mask(R, R, 7, s)[:, None]
    o = np.einsum("whij,whjd->whid", swin_ref.softmax(att), v)
    o = o.transpose(0, 2, 1, 3).reshape(nw, nw, 7, 7, C).transpose(0, 2, 1, 3, 4).reshape(R, R, C)
    if s:
        o = np.roll(o, (s, s), axis=(0, 1))
    return o.reshape(R * R, C)


@pytest.mark.parametrize("dtype,tol", [("f32", 2e-5), ("bf16", 3e-2)])
@pytest.mark.parametrize("R,H,shift,B", [(14, 3, 0, 2), (14, 3, 3, 2), (28, 6, 3, 1),
                                         (7, 24, 0, 3), (21, 4, 3, 1)])
def test_window_attention_kernel(gpu, dtype, tol, R, H, shift, B):
    out, ref, C, ldo = _window_case(dtype, R, H, shift, B, gpu)
    assert np.abs(out[:, :C] - ref).max() <= tol
    assert (out[:, C:] == 0).all()  # pad columns zeroed for the proj GEMM's K padding


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_patch_merge_kernel(gpu, dtype):
    rng = np.random.default_rng(1)
    B, R, C, ldx = 2, 14, 96, 128
    x = torch.from_numpy(rng.standard_normal((B * R * R, ldx)).astype(np.float32)).to(gpu).to(TDT[dtype])
    out = torch.empty((B * (R // 2) ** 2, 4 * C), dtype=TDT[dtype], device=gpu)
    nslots = 2
    stats = torch.full((out.shape[0], nslots, 2), float("nan"), device=gpu)
    _lib.check(_lib.load_library().evt_patch_merge(_lib.DTYPE[dtype], _p(x), ldx, B, R, C, _p(out),
                                                   _p(stats), nslots, _s()))
    torch.cuda.synchronize()
    xs = x.float().cpu().numpy()[:, :C].reshape(B, R, R, C)
    ref = np.concatenate([xs[:, 0::2, 0::2], xs[:, 1::2, 0::2], xs[:, 0::2, 1::2],
                          xs[:, 1::2, 1::2]], -1).reshape(-1, 4 * C)
    o = out.float().cpu().numpy()
    assert np.array_equal(o, ref)  # a gather: bit-exact
    st = stats.cpu().numpy()
    assert np.allclose(st[:, 0, 0], ref.astype(np.float64).sum(1), rtol=1e-5, atol=1e-3)
    assert np.allclose(st[:, 0, 1], (ref.astype(np.float64) ** 2).sum(1), rtol=1e-5, atol=1e-3)
    assert (st[:, 1:] == 0).all()


def test_fused_stage1_mlp_matches_gemm_path(gpu):
    """The fused C = 96 MLP kernel (default) against the two-GEMM path (forced by any explicit GEMM
    variant) on the same model and images: same math, different bf16 rounding points."""
    cfg = swin_config("tiny", image_size=56, depths=(2, 2), num_heads=(3, 6), num_classes=37)
    params = make_swin_params(cfg, seed=15)
    m = _model(cfg, "bf16", params, gpu, max_batch=6)
    img = torch.from_numpy(make_images(6, seed=16, image_size=56)).to(gpu)
    lib = _lib.load_library()
    fused = m(img).cpu().numpy().astype(np.float64)
    _lib.check(lib.evt_set_gemm_variant(9))
    try:
        gemm = m(img).cpu().numpy().astype(np.float64)
    finally:
        _lib.check(lib.evt_set_gemm_variant(0))
    ref = swin_ref.swin_forward(params, cfg, make_images(6, seed=16, image_size=56))
    assert np.abs(fused - gemm).max() <= 3e-2
    assert np.abs(fused - ref).max() <= 3e-2 and _cos_rows(fused, ref).min() >= 0.9995
