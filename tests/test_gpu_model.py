"""End-to-end parity of the MI355X ViT forward against the committed golden fixtures (produced by
the reference's own torch_layers, tests/golden/make_golden.py) and the numpy oracle.

Tolerances (stated):
  * f32 path (exact fp32 MFMA): max |logits - golden| <= 1e-3.
  * bf16 path (bf16 operands, fp32 accumulate / LN / softmax / GELU): max-abs <= 3e-2 and
    per-row cosine >= 0.9995 vs the fp64 golden.
"""
import os

import numpy as np
import pytest
import torch

from edgevisiontransformer_amd.modeling.models.vit import ViT, ViT_Pruned, get_deit_tiny
from edgevisiontransformer_amd.weights import digest, make_images, make_vit_params
from oracle import vit_ref
from tests.golden.make_golden import CASES, case_config

pytestmark = pytest.mark.gpu

F32_TOL = 1e-3
BF16_ABS, BF16_COS = 3e-2, 0.9995
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _model_for(name, dtype, gpu):
    kw, enc, batch, pseed, iseed = CASES[name]
    cfg = case_config(name)
    params = make_vit_params(cfg, seed=pseed)
    common = dict(image_size=cfg.image_size, patch_size=cfg.patch_size,
                  num_classes=cfg.num_classes, dim=kw["dim"], depth=kw["depth"],
                  heads=kw["heads"], mlp_dim=kw["mlp_dim"], dtype=dtype, weights=params, device=gpu)
    if enc:
        m = ViT_Pruned(head_size=64, prune_encoding=enc, **common)
    else:
        m = ViT(**common)
    assert tuple(m.cfg.heads) == tuple(cfg.heads) and tuple(m.cfg.ffn) == tuple(cfg.ffn)
    img = make_images(batch, seed=iseed, image_size=cfg.image_size)
    return m, img


def _cos_rows(a, b):
    return (a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))


@pytest.mark.parametrize("name", list(CASES))
def test_golden_f32(gpu, name):
    m, img = _model_for(name, "f32", gpu)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    assert digest([img]) == str(z["image_digest"])
    out = m(torch.from_numpy(img).to(gpu))
    torch.cuda.synchronize()
    err = np.abs(out.cpu().numpy().astype(np.float64) - z["logits"]).max()
    assert err <= F32_TOL, f"{name}: f32 max-abs {err:.3e} > {F32_TOL}"


@pytest.mark.parametrize("name", list(CASES))
def test_golden_bf16(gpu, name):
    m, img = _model_for(name, "bf16", gpu)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    out = m(img).astype(np.float64)  # numpy in -> numpy out
    err = np.abs(out - z["logits"]).max()
    cos = _cos_rows(out, z["logits"]).min()
    assert err <= BF16_ABS and cos >= BF16_COS, f"{name}: bf16 max-abs {err:.3e}, min cos {cos:.5f}"


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_batch_independence(gpu, dtype):
    """Images are independent (reference has no cross-image op): for a fixed GEMM kernel selection a
    37-image batch equals the per-image results bit for bit (batch sizes past the first build
    re-plan), and at 37 images under the automatic selection (which may pick 256 x 256 tiles for
    the batch and 128 x 128 for one image) the rows follow their images through a roll of the
    batch bit for bit."""
    from edgevisiontransformer_amd import _lib
    m = get_deit_tiny(dtype=dtype, seed=3, device=gpu)
    img = torch.from_numpy(make_images(37, seed=9)).to(gpu)
    lib = _lib.load_library()
    lib.evt_set_gemm_variant(1)  # every GEMM on the 128 x 128 kernel, whatever the batch
    try:
        full = m(img)
        parts = torch.cat([m(img[i:i + 1]) for i in (0, 17, 36)])
        torch.cuda.synchronize()
    finally:
        lib.evt_set_gemm_variant(0)
    assert torch.equal(full[[0, 17, 36]], parts)
    auto = m(img)
    rolled = m(torch.roll(img, 11, 0))
    torch.cuda.synchronize()
    assert torch.equal(torch.roll(auto, 11, 0), rolled)


@pytest.mark.parametrize("which,batch,hm_layers", [
    ("deit_tiny", 64, 12), ("deit_base", 20, 12), ("deit_tiny", 3, 0),
    # the two 1-head layers (QKV width 192: 37 tiles of 256 x 256) keep the 128 x 128 kernel and
    # token-major qkv, the other four go head-major: mixed layouts within one forward
    ("pruned", 48, 4),
    # fewer than 128 tokens per image: the per-row image / token decode of the EPI_HM store (37
    # and 50 tokens; images straddle lanes' 16-row runs and the M edge of the last tile)
    ("tiny96", 300, 12), ("tiny112", 260, 12)])
def test_qkv_head_major_bitwise(gpu, monkeypatch, which, batch, hm_layers):
    """The head-major qkv layout (the QKV GEMM's EPI_HM store + the attention's slice strides; used
    where that GEMM runs the persistent kernel: every case here but the 3-image one) against the
    token-major layout (EVT_QKV_LAYOUT=token at model creation): the same arithmetic at other
    addresses, so the logits agree bit for bit. 'pruned': per-layer head counts 1-3 (QKV widths
    192-576, column-padded tiles). `hm_layers`: the layers whose QKV must have stored head-major
    (evt_model_qkv_layout), so a silent fallback to token-major cannot pass as equality."""
    from edgevisiontransformer_amd.modeling.models import vit

    def build():
        if which == "pruned":
            return ViT_Pruned(dim=192, depth=6, heads=3, mlp_dim=768, head_size=64,
                              prune_encoding="layerwise_h1-d0.5_h3-d1.0_h2-d0.3_h3-d0.7_h1-d1.0_h2-d0.2",
                              dtype="bf16", seed=12, device=gpu)
        if which.startswith("tiny"):
            return ViT(image_size=int(which[4:]), patch_size=16, dim=192, depth=12, heads=3,
                       mlp_dim=768, dtype="bf16", seed=12, device=gpu)
        return getattr(vit, f"get_{which}")(dtype="bf16", seed=12, device=gpu)

    size = int(which[4:]) if which.startswith("tiny") else 224
    img = torch.from_numpy(make_images(batch, seed=21, image_size=size)).to(gpu)
    monkeypatch.setenv("EVT_QKV_LAYOUT", "token")
    mt = build()
    tok = mt(img)
    torch.cuda.synchronize()
    assert mt.qkv_headmajor_layers() == 0
    monkeypatch.delenv("EVT_QKV_LAYOUT")
    mh = build()
    hm = mh(img)
    torch.cuda.synchronize()
    assert mh.qkv_headmajor_layers() == hm_layers
    assert torch.isfinite(hm).all()
    assert torch.equal(tok, hm)


@pytest.mark.parametrize("which,batch", [("deit_base", 64), ("t2t_vit_14", 128)])
def test_grid_balance_bitwise(gpu, which, batch):
    """Persistent GEMM launches of 2-4 tile rounds run on fewer blocks with equal tile counts
    (launch_pers, round 6): only the tile -> block assignment changes, so the logits equal those
    of one block per CU (evt_set_gemm_variant 36) bit for bit. DeiT-base at 64 images: FC1 600
    tiles on 200 blocks, QKV 450 on 232; T2T-ViT-14 at 128 images: QKV / FC1 495 tiles on 248."""
    from edgevisiontransformer_amd import _lib
    from edgevisiontransformer_amd.modeling.models import t2t_vit, vit
    if which == "deit_base":
        m = vit.get_deit_base(dtype="bf16", seed=3, device=gpu)
        img = torch.from_numpy(make_images(batch, seed=31)).to(gpu)
    else:
        m = t2t_vit.get_t2t_vit_14(dtype="bf16", seed=3, device=gpu)
        img = torch.from_numpy(make_images(batch, seed=31, layout="NHWC")).to(gpu)
    lib = _lib.load_library()
    auto = m(img)
    torch.cuda.synchronize()
    lib.evt_set_gemm_variant(36)
    try:
        flat = m(img)
        torch.cuda.synchronize()
    finally:
        lib.evt_set_gemm_variant(0)
    assert torch.isfinite(auto).all()
    assert torch.equal(auto, flat)


def test_deit_small_bf16_vs_oracle(gpu):
    from edgevisiontransformer_amd.modeling.models.vit import get_deit_small
    m = get_deit_small(dtype="bf16", seed=4, device=gpu)
    img = make_images(2, seed=10)
    ref = vit_ref.vit_forward(make_vit_params(m.cfg, seed=4), m.cfg, img)
    out = m(img).astype(np.float64)
    assert np.abs(out - ref).max() <= BF16_ABS and _cos_rows(out, ref).min() >= BF16_COS


@pytest.mark.parametrize("enc", ["all_head1_ffn0.1", "layerwise_" + "_".join(
    f"h{1 + i % 3}-d{0.1 * (1 + i % 9):.1f}" for i in range(12))])
def test_pruned_tiny_f32_vs_oracle(gpu, enc):
    m = ViT_Pruned(dim=192, depth=12, heads=3, mlp_dim=768, head_size=64, prune_encoding=enc,
                   dtype="f32", seed=6, device=gpu)
    img = make_images(2, seed=11)
    ref = vit_ref.vit_forward(make_vit_params(m.cfg, seed=6), m.cfg, img)
    out = m(img).astype(np.float64)
    assert np.abs(out - ref).max() <= F32_TOL


def test_errors_are_loud(gpu):
    from edgevisiontransformer_amd._lib import EvtError
    m = get_deit_tiny(dtype="bf16", seed=0, device=gpu)
    with pytest.raises(ValueError):
        m(torch.zeros((1, 3, 32, 32), device=gpu))
    with pytest.raises(ValueError):
        ViT(dim=200, heads=3)
    with pytest.raises(AssertionError):
        ViT(image_size=225, patch_size=16)
    with pytest.raises(EvtError):
        ViT(dim=100, heads=1, mlp_dim=96, depth=1, device=gpu, max_batch=1)  # dim % 8 != 0
    with pytest.raises(EvtError):
        ViT(dim=256, heads=1, mlp_dim=96, depth=1, device=gpu, max_batch=1)  # h_k 256 > 128
    with pytest.raises(EvtError):
        ViT(dim=96, heads=1, mlp_dim=96, depth=1, dtype="mx8", device=gpu, max_batch=1)  # MX8: 64


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
def test_graph_replay_matches_eager(gpu, dtype):
    """evt_graph_capture / evt_graph_launch: the replayed HIP graph gives the eager logits bit
    for bit, and follows in-place updates of the captured input buffer."""
    m = get_deit_tiny(dtype=dtype, seed=5, device=gpu, max_batch=3)
    img = torch.from_numpy(make_images(3, seed=21)).to(gpu)
    eager = m(img).clone()
    logits = torch.empty_like(eager)
    m.capture_graph(img, logits)
    m.replay_graph()
    torch.cuda.synchronize()
    assert torch.equal(logits, eager)
    img.copy_(torch.from_numpy(make_images(3, seed=22)).to(gpu))
    m.replay_graph()
    torch.cuda.synchronize()
    assert torch.equal(logits, m(img))

