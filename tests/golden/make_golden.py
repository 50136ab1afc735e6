"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own layer code.

Run in the build container only (it needs /root/reference, which never reaches the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case ...]

What it does
------------
The reference's TF-Keras forward (`modeling/models/vit.py`) cannot run here: TensorFlow is
not installed (ModuleNotFoundError; no permission was denied). Its PyTorch twins
`modeling/torch_layers/{attention,ffn,norm,residual,activation}.py` DO import, and
reproduce the TF encoder sublayer exactly under this weight mapping:

  to_query/to_key/to_value.weight = Wqkv[:, s*h*d:(s+1)*h*d].T, biases = 0   (TF has no QKV bias)
  to_out.weight = Wout.T, to_out.bias = bout
  FeedForward.linear1/2.weight = W1.T / W2.T, biases b1 / b2
  torch_layers.norm.LayerNorm(D, Residual(sub), is_pre=True)  -> f(LN(x)) + LN(x)

This script composes those reference modules in the order of `modeling/models/vit.py:41-55`
(einops Rearrange with the reference's own pattern string, cls concat, +pos, encoder,
token 0, Dense(M)+gelu (reference torch gelu), Dense(C)), runs it in float64 on the seeded
parameters of `edgevisiontransformer_amd.weights`, and stores inputs digests + logits +
layer-0 checkpoints. Only data is stored: no reference source text is copied.
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

import torch  # noqa: E402
from einops import rearrange  # noqa: E402

from edgevisiontransformer_amd.weights import (digest, make_images, make_t2t_params,  # noqa: E402
                                               make_vit_params, t2t_config, vit_config)
from edgevisiontransformer_amd.modeling.models.vit import decode_prune_encoding  # noqa: E402


def _ref_modules():
    sys.path.insert(0, REF)
    from modeling.torch_layers.attention import Attention
    from modeling.torch_layers.ffn import FeedForward
    from modeling.torch_layers.norm import LayerNorm
    from modeling.torch_layers.residual import Residual
    from modeling.torch_layers.activation import gelu
    return Attention, FeedForward, LayerNorm, Residual, gelu


def _t(a):
    return torch.from_numpy(np.asarray(a, dtype=np.float64))


def ref_encoder(x, params, d, heads, hks, ffns, trace=None):
    """Encoder layers composed from the reference torch twins (transformer_encoder.py:13-18)."""
    Attention, FeedForward, LayerNorm, Residual, gelu = _ref_modules()
    for i in range(len(heads)):
        h, hk = heads[i], hks[i]
        attn = Attention(d, h, hk)
        inner = h * hk
        W = _t(params[f"l{i}.qkv_w"])
        attn.to_query.weight.copy_(W[:, 0:inner].T)
        attn.to_key.weight.copy_(W[:, inner:2 * inner].T)
        attn.to_value.weight.copy_(W[:, 2 * inner:3 * inner].T)
        for lin in (attn.to_query, attn.to_key, attn.to_value):
            lin.bias.zero_()
        attn.to_out.weight.copy_(_t(params[f"l{i}.out_w"]).T)
        attn.to_out.bias.copy_(_t(params[f"l{i}.out_b"]))
        blk1 = LayerNorm(d, Residual(attn), is_pre=True)
        blk1.layer_norm.weight.copy_(_t(params[f"l{i}.ln1_g"]))
        blk1.layer_norm.bias.copy_(_t(params[f"l{i}.ln1_b"]))
        ffn = FeedForward(d, ffns[i])
        ffn.linear1.weight.copy_(_t(params[f"l{i}.fc1_w"]).T)
        ffn.linear1.bias.copy_(_t(params[f"l{i}.fc1_b"]))
        ffn.linear2.weight.copy_(_t(params[f"l{i}.fc2_w"]).T)
        ffn.linear2.bias.copy_(_t(params[f"l{i}.fc2_b"]))
        blk2 = LayerNorm(d, Residual(ffn), is_pre=True)
        blk2.layer_norm.weight.copy_(_t(params[f"l{i}.ln2_g"]))
        blk2.layer_norm.bias.copy_(_t(params[f"l{i}.ln2_b"]))
        x = blk1(x)
        if trace is not None and i == 0:
            trace["l0.attn"] = x.numpy().copy()
        x = blk2(x)
        if trace is not None and i == 0:
            trace["l0.ffn"] = x.numpy().copy()
    return x


def reference_forward(params, cfg, img, trace=None):
    gelu = _ref_modules()[4]
    torch.set_default_dtype(torch.float64)
    d = cfg.dim
    with torch.no_grad():
        x = rearrange(_t(img), "b c (h p1) (w p2) -> b (h w) (p1 p2 c)",
                      p1=cfg.patch_size, p2=cfg.patch_size)
        x = x @ _t(params["patch_w"]) + _t(params["patch_b"])
        cls = _t(params["cls"]).reshape(1, 1, d).expand(x.shape[0], 1, d)
        x = torch.cat([cls, x], dim=1) + _t(params["pos"])
        x = ref_encoder(x, params, d, cfg.heads, cfg.head_dim, cfg.ffn, trace)
        t = x[:, 0]
        hid = gelu(t @ _t(params["head1_w"]) + _t(params["head1_b"]))
        out = hid @ _t(params["head2_w"]) + _t(params["head2_b"])
    return out.numpy()


# ---- T2T-ViT ---------------------------------------------------------------------------------
# The tokens-to-token stage has no runnable reference (TF absent; no torch twin of TokenPerformer
# in the reference): it is formulated here independently in torch ops from the reference lines
# (t2t_vit.py:7-88, transformer_encoder.py:39-101) - torch.nn.functional.unfold for the soft
# split, permuted from torch's (c, kh, kw) to extract_patches' (kh, kw, c) vector order - and the
# encoder is the reference torch twins again. PARITY UNPINNED for the T2T stage.

def _t2t_unfold(x, k, s, p):
    """tf_Unfold(channel_last=True) on NHWC x via torch unfold on NCHW."""
    b, h, w, c = x.shape
    cols = torch.nn.functional.unfold(x.permute(0, 3, 1, 2), k, padding=p, stride=s)  # b, c*k*k, L
    cols = cols.reshape(b, c, k * k, -1).permute(0, 3, 2, 1)                           # b, L, kk, c
    return cols.reshape(b, -1, k * k * c)


def _t2t_performer(x, params, pre):
    gelu = _ref_modules()[4]
    P = lambda n: _t(params[pre + n])  # noqa: E731
    x = torch.nn.functional.layer_norm(x, x.shape[-1:], P("ln1_g"), P("ln1_b"), eps=1e-5)
    k, q, v = torch.chunk(x @ P("kqv_w") + P("kqv_b"), 3, dim=-1)
    w = P("w")
    m = w.shape[0]

    def prm(z):
        return torch.exp(z @ w.T - (z * z).sum(-1, keepdim=True) / 2) / m ** 0.5
    kp, qp = prm(k), prm(q)
    dd = (qp * kp.sum(1, keepdim=True)).sum(-1, keepdim=True)
    kptv = v.transpose(1, 2) @ kp                         # b, hs, m
    y = (qp @ kptv.transpose(1, 2)) / (dd + 1e-8)
    y = v + y @ P("out_w") + P("out_b")
    h = torch.nn.functional.layer_norm(y, y.shape[-1:], P("ln2_g"), P("ln2_b"), eps=1e-5)
    return y + gelu(h @ P("fc1_w") + P("fc1_b")) @ P("fc2_w") + P("fc2_b")


def t2t_reference_forward(params, cfg, img, trace=None):
    torch.set_default_dtype(torch.float64)
    d = cfg.dim
    with torch.no_grad():
        x = _t2t_unfold(_t(img), 7, 4, 2)
        x = _t2t_performer(x, params, "p1.")
        g1, g2, _ = cfg.grids
        x = _t2t_unfold(x.reshape(x.shape[0], g1, g1, -1), 3, 2, 1)
        x = _t2t_performer(x, params, "p2.")
        x = _t2t_unfold(x.reshape(x.shape[0], g2, g2, -1), 3, 2, 1)
        if trace is not None:
            trace["split2"] = x.numpy().copy()
        x = x @ _t(params["project_w"]) + _t(params["project_b"])
        cls = _t(params["cls"]).reshape(1, 1, d).expand(x.shape[0], 1, d)
        x = torch.cat([cls, x], dim=1) + _t(params["pos"])
        # TransformerEncoderBlock -> Attention(hidden_size, num_heads): h_k = dim // heads
        x = ref_encoder(x, params, d, [cfg.heads] * cfg.depth, [d // cfg.heads] * cfg.depth,
                        [cfg.mlp_dim] * cfg.depth, trace)
        t = torch.nn.functional.layer_norm(x[:, 0], (d,), _t(params["norm_g"]),
                                           _t(params["norm_b"]), eps=1e-5)
        out = t @ _t(params["head_w"]) + _t(params["head_b"])
    return out.numpy()


# name -> (t2t_config args (hidden, depth, heads, mlp_ratio), batch, param seed, image seed)
T2T_CASES = {
    "t2t_vit_7_b2": ((256, 7, 4, 2), 2, 11, 12),
    "t2t_vit_14_b1": ((384, 14, 6, 3), 1, 13, 14),
    # head size 96 (T2T_ViT(hidden_size=384, num_heads=4)): the generic attention kernels
    "t2t_384h4_d2_b1": ((384, 2, 4, 3), 1, 15, 16),
}


# name -> (config kwargs, batch, param seed, image seed)
CASES = {
    "deit_tiny_b2": (dict(dim=192, depth=12, heads=3, mlp_dim=768), None, 2, 0, 1),
    "deit_tiny_pruned_all_head2_ffn0.7_b2": (dict(dim=192, depth=12, heads=3, mlp_dim=768),
                                             "all_head2_ffn0.7", 2, 3, 4),
    "vit_small2_layerwise_b3": (dict(dim=128, depth=2, heads=2, mlp_dim=320, num_classes=37),
                                "layerwise_h1-d0.37_h3-d0.1", 3, 5, 6),
    "deit_base_b1": (dict(dim=768, depth=12, heads=12, mlp_dim=3072), None, 1, 7, 8),
    # head sizes other than 64 (attention.py:6-12, h_k = dim // heads) and widths that are not a
    # multiple of 64: Attention(96, 1), Attention(768, 8), h_k 32, and h_k 10 with D = 80
    "vit_d96_h1_b2": (dict(dim=96, depth=2, heads=1, mlp_dim=192, num_classes=10), None, 2, 17, 18),
    "vit_d768_h8_b1": (dict(dim=768, depth=2, heads=8, mlp_dim=1536), None, 1, 19, 20),
    "vit_d192_h6_b2": (dict(dim=192, depth=3, heads=6, mlp_dim=384), None, 2, 21, 22),
    "vit_d80_h8_b2": (dict(dim=80, depth=2, heads=8, mlp_dim=160, num_classes=7), None, 2, 23, 24),
}


def case_config(name):
    kw, enc, _, _, _ = CASES[name]
    kw = dict(kw)
    if enc is None:
        return vit_config(**kw)
    setting, heads, thr = decode_prune_encoding(enc)
    depth = kw["depth"]
    if setting == "all":
        hl, fl = [heads] * depth, [int(thr * kw["mlp_dim"])] * depth
    else:
        hl, fl = heads, [int(t * kw["mlp_dim"]) for t in thr]
    return vit_config(**kw, head_size=64, heads_list=hl, ffn_list=fl)


def main(only=()):
    for name, (kw, enc, batch, pseed, iseed) in CASES.items():
        if only and name not in only:
            continue
        cfg = case_config(name)
        params = make_vit_params(cfg, seed=pseed)
        img = make_images(batch, seed=iseed, image_size=cfg.image_size)
        trace = {}
        logits = reference_forward(params, cfg, img, trace)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(
            path, logits=logits, param_seed=pseed, image_seed=iseed, batch=batch,
            param_digest=digest(params), image_digest=digest([img]),
            l0_attn_row0=trace["l0.attn"][:, :4], l0_ffn_row0=trace["l0.ffn"][:, :4],
            encoding=enc or "")
        print(f"{name}: logits {logits.shape} absmax {np.abs(logits).max():.4f} -> {path}")
    for name, (args, batch, pseed, iseed) in T2T_CASES.items():
        if only and name not in only:
            continue
        cfg = t2t_config(*args)
        params = make_t2t_params(cfg, seed=pseed)
        img = make_images(batch, seed=iseed, image_size=cfg.image_size, layout="NHWC")
        trace = {}
        logits = t2t_reference_forward(params, cfg, img, trace)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(
            path, logits=logits, param_seed=pseed, image_seed=iseed, batch=batch,
            param_digest=digest(params), image_digest=digest([img]),
            split2_row0=trace["split2"][:, :4], l0_attn_row0=trace["l0.attn"][:, :4],
            l0_ffn_row0=trace["l0.ffn"][:, :4])
        print(f"{name}: logits {logits.shape} absmax {np.abs(logits).max():.4f} -> {path}")


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))  # optional case names: regenerate only those
