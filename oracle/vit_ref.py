"""CPU restatement (numpy) of the reference TF-Keras ViT / ViT_Pruned forward.

TEST INFRASTRUCTURE ONLY. This module is the parity oracle: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it. The product
path (`edgevisiontransformer_amd`) never imports or calls it and fails loudly without its
HIP library.

It follows, line by line, the reference files below (paths relative to the reference
repo root). The reference forward itself needs TensorFlow, which is not installed here
(an ordinary ModuleNotFoundError, not a denial); parity of this restatement is pinned by
`tests/golden/*.npz`, produced by `tests/golden/make_golden.py` from the reference's own
PyTorch twins `modeling/torch_layers/*.py` composed in the order of
`modeling/models/vit.py` (see SURVEY.md 8c for the weight mapping).

Semantics reproduced (parity traps):
  * pre-norm block returns f(LN(x)) + LN(x)            norm.py:11-12 + residual.py:9
  * LayerNorm eps 1e-5, population variance            norm.py:6 (Keras LayerNormalization)
  * tanh-approximate GELU                              activation.py:13-15
  * fused QKV Dense without bias, columns (qkv h d)    attention.py:17,20
  * scale = h_k ** -0.5 on q.k                         attention.py:15,30
  * patch vector order (p1 p2 c) from NCHW input       vit.py:31-32,45
  * no final LayerNorm; head = Dense(M, gelu) -> Dense(C) on token 0   vit.py:38-39,54-55
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np


def layer_norm(x: np.ndarray, gamma: np.ndarray, beta: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    """Keras LayerNormalization over the last axis (`modeling/layers/norm.py:6`)."""
    mean = x.mean(axis=-1, keepdims=True)
    var = ((x - mean) ** 2).mean(axis=-1, keepdims=True)
    return (x - mean) / np.sqrt(var + eps) * gamma + beta


def gelu(x: np.ndarray) -> np.ndarray:
    """`modeling/layers/activation.py:13-15` (tanh approximation)."""
    return x * (0.5 * (1.0 + np.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x ** 3))))


def patchify_nchw(img: np.ndarray, p: int) -> np.ndarray:
    """einops 'b c (h p1) (w p2) -> b (h w) (p1 p2 c)' (`modeling/models/vit.py:31-32`)."""
    b, c, hh, ww = img.shape
    x = img.reshape(b, c, hh // p, p, ww // p, p)          # b c h p1 w p2
    x = x.transpose(0, 2, 4, 3, 5, 1)                       # b h w p1 p2 c
    return x.reshape(b, (hh // p) * (ww // p), p * p * c)


def softmax(x: np.ndarray, axis: int = -1) -> np.ndarray:
    """tf.nn.softmax (`modeling/layers/attention.py:31`)."""
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def attention(y: np.ndarray, qkv_w: np.ndarray, out_w: np.ndarray, out_b: np.ndarray,
              heads: int, hk: int) -> np.ndarray:
    """`modeling/layers/attention.py:23-35` for y [B, N, D]."""
    b, n, _ = y.shape
    qkv = y @ qkv_w                                          # :24 (no bias)
    qkv = qkv.reshape(b, n, 3, heads, hk).transpose(2, 0, 3, 1, 4)   # :20 (qkv h d)
    q, k, v = qkv[0], qkv[1], qkv[2]                         # [B, h, N, d]
    dots = np.einsum("bhid,bhjd->bhij", q, k) * (hk ** -0.5)  # :30
    attn = softmax(dots, axis=-1)                            # :31
    out = np.einsum("bhij,bhjd->bhid", attn, v)              # :33
    out = out.transpose(0, 2, 1, 3).reshape(b, n, heads * hk)  # :34 'b h n d -> b n (h d)'
    return out @ out_w + out_b                               # :35


def feed_forward(y: np.ndarray, fc1_w, fc1_b, fc2_w, fc2_b) -> np.ndarray:
    """`modeling/layers/ffn.py:8-12`."""
    return gelu(y @ fc1_w + fc1_b) @ fc2_w + fc2_b


def encoder_layer(x: np.ndarray, P: Dict[str, np.ndarray], i: int, heads: int, hk: int,
                  trace: Optional[dict] = None) -> np.ndarray:
    """Two `LayerNorm(Residual(.), pre=True)` sublayers (`transformer_encoder.py:13-18,26-34`)."""
    y = layer_norm(x, P[f"l{i}.ln1_g"], P[f"l{i}.ln1_b"])
    a = attention(y, P[f"l{i}.qkv_w"], P[f"l{i}.out_w"], P[f"l{i}.out_b"], heads, hk)
    x = a + y                                                # residual.py:9 on LN(x)
    if trace is not None:
        trace[f"l{i}.ln1"] = y
        trace[f"l{i}.attn"] = x
    y = layer_norm(x, P[f"l{i}.ln2_g"], P[f"l{i}.ln2_b"])
    f = feed_forward(y, P[f"l{i}.fc1_w"], P[f"l{i}.fc1_b"], P[f"l{i}.fc2_w"], P[f"l{i}.fc2_b"])
    x = f + y
    if trace is not None:
        trace[f"l{i}.ln2"] = y
        trace[f"l{i}.ffn"] = x
    return x


def vit_forward(params: Dict[str, np.ndarray], cfg, img: np.ndarray,
                dtype=np.float64, trace: Optional[dict] = None) -> np.ndarray:
    """`ViT.call` (`modeling/models/vit.py:41-55`); also `ViT_Pruned` via cfg.heads/cfg.ffn.

    img: NCHW [B, C, H, W]. Returns logits [B, num_classes] in `dtype`.
    """
    P = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    x = patchify_nchw(np.asarray(img, dtype=dtype), cfg.patch_size)   # :45
    x = x @ P["patch_w"] + P["patch_b"]                                # :46
    b = x.shape[0]
    cls = np.broadcast_to(P["cls"].reshape(1, 1, -1), (b, 1, cfg.dim))  # :48-49
    x = np.concatenate([cls, x], axis=1)                               # :50
    x = x + P["pos"]                                                   # :51
    if trace is not None:
        trace["embed"] = x
    for i in range(cfg.depth):                                         # :52
        x = encoder_layer(x, P, i, cfg.heads[i], cfg.head_dim[i], trace)
    t = x[:, 0]                                                        # :54
    h = gelu(t @ P["head1_w"] + P["head1_b"])                          # :55 mlp_head[0]
    return h @ P["head2_w"] + P["head2_b"]                             # :55 mlp_head[1]


def std_vit_forward(params: Dict[str, np.ndarray], cfg, img: np.ndarray, eps: float = 1e-6,
                    dtype=np.float64) -> np.ndarray:
    """The STANDARD DeiT / ViT forward (EVT_VIT_STANDARD; timm VisionTransformer, HF
    ViTForImageClassification): x + attn(LN1 x), x + mlp(LN2 x) with QKV bias and exact GELU,
    final LayerNorm, Linear head on token 0. Patch vectors in this build's (p1 p2 c) order.
    Pinned by tests/golden/std_*.npz (HF transformers, fp64). TEST INFRASTRUCTURE ONLY."""
    from scipy.special import erf
    P = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    x = patchify_nchw(np.asarray(img, dtype=dtype), cfg.patch_size) @ P["patch_w"] + P["patch_b"]
    b = x.shape[0]
    x = np.concatenate([np.broadcast_to(P["cls"], (b, 1, cfg.dim)), x], axis=1) + P["pos"]
    for i in range(cfg.depth):
        h, hk = cfg.heads[i], cfg.head_dim[i]
        y = layer_norm(x, P[f"l{i}.ln1_g"], P[f"l{i}.ln1_b"], eps)
        n = y.shape[1]
        qkv = (y @ P[f"l{i}.qkv_w"] + P[f"l{i}.qkv_b"]).reshape(b, n, 3, h, hk).transpose(2, 0, 3, 1, 4)
        att = softmax(np.einsum("bhid,bhjd->bhij", qkv[0], qkv[1]) * hk ** -0.5)
        o = np.einsum("bhij,bhjd->bhid", att, qkv[2]).transpose(0, 2, 1, 3).reshape(b, n, h * hk)
        x = x + o @ P[f"l{i}.out_w"] + P[f"l{i}.out_b"]
        y = layer_norm(x, P[f"l{i}.ln2_g"], P[f"l{i}.ln2_b"], eps)
        z = y @ P[f"l{i}.fc1_w"] + P[f"l{i}.fc1_b"]
        z = 0.5 * z * (1.0 + erf(z / math.sqrt(2.0)))
        x = x + z @ P[f"l{i}.fc2_w"] + P[f"l{i}.fc2_b"]
    x = layer_norm(x[:, 0], P["norm_g"], P["norm_b"], eps)
    return x @ P["head_w"] + P["head_b"]
