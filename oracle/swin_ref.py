"""CPU restatement (numpy) of the Swin Transformer forward the reference benchmarks.

TEST INFRASTRUCTURE ONLY. Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module; the product path never calls it.

The reference does not contain Swin's code: `utils.py:14-47` (`get_swin`) imports
`SwinTransformer` from an external checkout of microsoft/Swin-Transformer (unpinned, not
vendored; `tools.py:272-282` benchmarks `swin_tiny_patch4_window7_224` NCHW [B,3,224,224]).
This restatement follows the published algorithm of that model, as also implemented by the
third-party HuggingFace `transformers` 5.15.0 `models/swin/modeling_swin.py` (importable in the
build container, never on the GPU box), whose outputs pin it: `tests/golden/make_golden_swin.py`
runs `SwinForImageClassification` in float64 on the same seeded weights and stores the logits
(parity of the reference's own Swin is therefore "pinned by a third-party restatement", see
DESIGN.md). Line references are to that HF file:

  * patch embed: Conv2d(k=s=patch) (:264) -> flatten (h w) (:283-284) -> LayerNorm (SwinEmbeddings)
  * block: x + proj(WMSA(LN1(x))); x + fc2(gelu(fc1(LN2(x))))   (:542-574), pre-norm, erf GELU
  * cyclic shift torch.roll(-s) before / (+s) after the window attention (:616-626)
  * window partition / reverse 7x7 windows, row-major inside a window (:486-505)
  * relative position bias table[(dh+w-1)*(2w-1) + (dw+w-1)] (:350-371), scale hd^-0.5 (:408)
  * SW-MSA mask: 3x3 regions, -100 where the region ids differ (:584-607)
  * patch merging: cat(x[0::2,0::2], x[1::2,0::2], x[0::2,1::2], x[1::2,1::2]) -> LN(4C) ->
    Linear(4C, 2C, bias=False) (:309-326)
  * head: LN -> mean over tokens -> Linear (SwinModel :876-880, classifier)
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

try:  # scipy is in the image; fall back to math.erf if not
    from scipy.special import erf as _erf
except ImportError:  # pragma: no cover
    _erf = np.vectorize(math.erf)


def layer_norm(x, g, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * g + b


def gelu_erf(x):
    """nn.GELU() (exact erf form; HF ACT2FN['gelu'])."""
    return 0.5 * x * (1.0 + _erf(x / math.sqrt(2.0)))


def softmax(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def patch_embed(img, w, b, p):
    """Conv2d(in, E, k=p, s=p) as a matmul over (c, kh, kw) patch vectors -> [B, T, E]."""
    bsz, c, hh, ww = img.shape
    x = img.reshape(bsz, c, hh // p, p, ww // p, p).transpose(0, 2, 4, 1, 3, 5)
    x = x.reshape(bsz, (hh // p) * (ww // p), c * p * p)
    return x @ w + b


def relative_position_index(w):
    """Index into the [(2w-1)^2, heads] table for each (query, key) of a w*w window."""
    ys, xs = np.meshgrid(np.arange(w), np.arange(w), indexing="ij")
    cy, cx = ys.reshape(-1), xs.reshape(-1)
    dy = cy[:, None] - cy[None, :] + (w - 1)
    dx = cx[:, None] - cx[None, :] + (w - 1)
    return dy * (2 * w - 1) + dx


def shift_mask(h, wd, w, s):
    """[nW, w*w, w*w] additive mask of the shifted-window attention (0 / -100)."""
    hr = (np.arange(h) >= h - w).astype(np.int64) + (np.arange(h) >= h - s)
    wr = (np.arange(wd) >= wd - w).astype(np.int64) + (np.arange(wd) >= wd - s)
    reg = hr[:, None] * 3 + wr[None, :]
    win = reg.reshape(h // w, w, wd // w, w).transpose(0, 2, 1, 3).reshape(-1, w * w)
    return np.where(win[:, None, :] != win[:, :, None], -100.0, 0.0)


def window_attention(y, res, heads, w, s, qkv_w, qkv_b, rpb, proj_w, proj_b):
    """Shifted-window MSA on normalised tokens y [B, res*res, C] -> [B, res*res, C]."""
    bsz, n, c = y.shape
    hd = c // heads
    x = y.reshape(bsz, res, res, c)
    if s:
        x = np.roll(x, (-s, -s), axis=(1, 2))
    nw = res // w
    win = x.reshape(bsz, nw, w, nw, w, c).transpose(0, 1, 3, 2, 4, 5).reshape(bsz, nw * nw, w * w, c)
    qkv = (win @ qkv_w + qkv_b).reshape(bsz, nw * nw, w * w, 3, heads, hd)
    q, k, v = (qkv[..., i, :, :].transpose(0, 1, 3, 2, 4) for i in range(3))  # [B, nW, h, N, hd]
    att = np.einsum("bwhid,bwhjd->bwhij", q, k) * hd ** -0.5
    bias = rpb[relative_position_index(w).reshape(-1)].reshape(w * w, w * w, heads)
    att = att + bias.transpose(2, 0, 1)[None, None]
    if s:
        att = att + shift_mask(res, res, w, s)[None, :, None]
    o = np.einsum("bwhij,bwhjd->bwhid", softmax(att), v)
    o = o.transpose(0, 1, 3, 2, 4).reshape(bsz, nw, nw, w, w, c).transpose(0, 1, 3, 2, 4, 5)
    o = o.reshape(bsz, res, res, c)
    if s:
        o = np.roll(o, (s, s), axis=(1, 2))
    return o.reshape(bsz, n, c) @ proj_w + proj_b


def patch_merge(x, res, g, b, w):
    bsz, _, c = x.shape
    x = x.reshape(bsz, res, res, c)
    x = np.concatenate([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
    x = x.reshape(bsz, -1, 4 * c)
    return layer_norm(x, g, b) @ w


def swin_forward(params: Dict[str, np.ndarray], cfg, img: np.ndarray, dtype=np.float64,
                 trace: dict | None = None) -> np.ndarray:
    """NCHW fp32 images [B, C, S, S] -> logits [B, num_classes] (float64)."""
    P = {k: np.asarray(v, dtype=dtype) for k, v in params.items()}
    x = patch_embed(np.asarray(img, dtype=dtype), P["patch_w"], P["patch_b"], cfg.patch_size)
    x = layer_norm(x, P["pnorm_g"], P["pnorm_b"])
    if trace is not None:
        trace["embed"] = x
    for i in range(cfg.num_stages):
        res = cfg.res(i)
        if i > 0:
            x = patch_merge(x, cfg.res(i - 1), P[f"s{i}.merge_g"], P[f"s{i}.merge_b"],
                            P[f"s{i}.merge_w"])
        for j in range(cfg.depths[i]):
            pre = f"s{i}.b{j}."
            y = layer_norm(x, P[pre + "ln1_g"], P[pre + "ln1_b"])
            x = x + window_attention(y, res, cfg.num_heads[i], cfg.window(i), cfg.shift(i, j),
                                     P[pre + "qkv_w"], P[pre + "qkv_b"], P[pre + "rpb"],
                                     P[pre + "proj_w"], P[pre + "proj_b"])
            y = layer_norm(x, P[pre + "ln2_g"], P[pre + "ln2_b"])
            x = x + gelu_erf(y @ P[pre + "fc1_w"] + P[pre + "fc1_b"]) @ P[pre + "fc2_w"] + P[pre + "fc2_b"]
            if trace is not None:
                trace[f"s{i}.b{j}"] = x
    x = layer_norm(x, P["norm_g"], P["norm_b"]).mean(axis=1)
    return x @ P["head_w"] + P["head_b"]
