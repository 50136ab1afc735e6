"""CPU: the numpy oracle (oracle/vit_ref.py) against the golden fixtures produced from the
reference's own torch_layers (tests/golden/make_golden.py), plus generator pinning."""
import os

import numpy as np
import pytest

from edgevisiontransformer_amd.weights import digest, make_images, make_vit_params
from oracle import vit_ref
from tests.golden.make_golden import CASES, case_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_matches_reference_golden(name):
    z = _load(name)
    cfg = case_config(name)
    params = make_vit_params(cfg, seed=int(z["param_seed"]))
    img = make_images(int(z["batch"]), seed=int(z["image_seed"]))
    assert digest(params) == str(z["param_digest"]), "weight generator drifted"
    assert digest([img]) == str(z["image_digest"]), "image generator drifted"
    trace = {}
    out = vit_ref.vit_forward(params, cfg, img, trace=trace)
    assert np.abs(out - z["logits"]).max() < 1e-9
    np.testing.assert_allclose(trace["l0.attn"][:, :4], z["l0_attn_row0"], atol=1e-10)
    np.testing.assert_allclose(trace["l0.ffn"][:, :4], z["l0_ffn_row0"], atol=1e-10)


def test_oracle_fp32_close_to_fp64():
    z = _load("deit_tiny_b2")
    cfg = case_config("deit_tiny_b2")
    p = make_vit_params(cfg, seed=int(z["param_seed"]))
    img = make_images(2, seed=int(z["image_seed"]))
    out = vit_ref.vit_forward(p, cfg, img, dtype=np.float32)
    assert out.dtype == np.float32 and np.abs(out - z["logits"]).max() < 1e-4


def test_patchify_matches_einops_pattern():
    einops = pytest.importorskip("einops")
    x = np.random.default_rng(0).standard_normal((2, 3, 32, 48))
    ref = einops.rearrange(x, "b c (h p1) (w p2) -> b (h w) (p1 p2 c)", p1=16, p2=16)
    np.testing.assert_array_equal(vit_ref.patchify_nchw(x, 16), ref)


def test_layernorm_quirk_residual_is_normalised_input():
    """Pre-norm sublayer returns f(LN(x)) + LN(x) (reference norm.py:11-12 + residual.py:9)."""
    cfg = case_config("vit_small2_layerwise_b3")
    p = make_vit_params(cfg, seed=5)
    x = np.random.default_rng(1).standard_normal((1, cfg.tokens, cfg.dim))
    tr = {}
    vit_ref.encoder_layer(x, p, 0, cfg.heads[0], 64, tr)
    y = vit_ref.layer_norm(x, p["l0.ln1_g"], p["l0.ln1_b"])
    a = vit_ref.attention(y, p["l0.qkv_w"], p["l0.out_w"], p["l0.out_b"], cfg.heads[0], 64)
    np.testing.assert_allclose(tr["l0.attn"], a + y)


def test_gelu_is_tanh_approximation():
    x = np.linspace(-6, 6, 101)
    ref = 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x ** 3)))
    np.testing.assert_allclose(vit_ref.gelu(x), ref)


# ---- T2T-ViT ------------------------------------------------------------------------------

from edgevisiontransformer_amd.weights import make_t2t_params, t2t_config  # noqa: E402
from oracle import t2t_ref  # noqa: E402
from tests.golden.make_golden import T2T_CASES  # noqa: E402


@pytest.mark.parametrize("name", list(T2T_CASES))
def test_t2t_oracle_matches_golden(name):
    """Encoder part pinned by the reference torch twins; the T2T stage is an independent torch
    formulation of the same reference lines (parity unpinned for that stage)."""
    args, batch, pseed, iseed = T2T_CASES[name]
    z = _load(name)
    cfg = t2t_config(*args)
    params = make_t2t_params(cfg, seed=pseed)
    img = make_images(batch, seed=iseed, image_size=cfg.image_size, layout="NHWC")
    assert digest(params) == str(z["param_digest"]), "weight generator drifted"
    assert digest([img]) == str(z["image_digest"]), "image generator drifted"
    trace = {}
    out = t2t_ref.t2t_vit_forward(params, cfg, img, trace=trace)
    assert np.abs(out - z["logits"]).max() < 1e-9
    np.testing.assert_allclose(trace["split2"][:, :4], z["split2_row0"], atol=1e-10)
    np.testing.assert_allclose(trace["l0.attn"][:, :4], z["l0_attn_row0"], atol=1e-10)


@pytest.mark.parametrize("k,s,p,c", [(7, 4, 2, 3), (3, 2, 1, 64), (3, 2, 1, 5)])
def test_unfold_vector_order_matches_torch_unfold(k, s, p, c):
    """tf_Unfold(channel_last=True) == torch unfold on NCHW with (c, kh, kw) -> (kh, kw, c)."""
    import torch
    rng = np.random.default_rng(k * 100 + c)
    x = rng.standard_normal((2, 12, 12, c))
    ours = t2t_ref.unfold_nhwc(x, k, s, p)
    cols = torch.nn.functional.unfold(torch.from_numpy(x).permute(0, 3, 1, 2), k, padding=p, stride=s)
    ref = cols.reshape(2, c, k * k, -1).permute(0, 3, 2, 1).reshape(2, -1, k * k * c).numpy()
    np.testing.assert_array_equal(ours, ref)


def test_sinusoid_table_matches_reference_formula():
    tab = t2t_ref.sinusoid_table(5, 8)
    assert tab.dtype == np.float32
    assert tab[0, 0] == 0.0 and tab[0, 1] == 1.0          # sin(0), cos(0)
    np.testing.assert_allclose(tab[3, 2], np.sin(3 / 10000 ** (2 / 8)), rtol=1e-6)
    np.testing.assert_allclose(tab[3, 3], np.cos(3 / 10000 ** (2 / 8)), rtol=1e-6)
