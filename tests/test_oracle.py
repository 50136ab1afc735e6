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
