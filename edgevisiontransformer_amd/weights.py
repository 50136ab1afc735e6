"""Deterministic parameter and input generation for the ViT family.

The reference never loads trained weights for its `modeling.models` forward: every
parameter is random-initialised by Keras (`modeling/models/vit.py:18-29`,
`modeling/models/t2t_vit.py:116-118` "not needed when only measuring inference latency").
This module is the MI355X build's equivalent: a seeded, platform-independent generator
(numpy PCG64) so the GPU box, the oracle and the golden fixtures all see bit-identical
fp32 parameters without shipping megabytes of weights.

Parameter layout is the Keras one (`Dense.kernel` is ``[in, out]``, ``y = x @ W + b``),
named after the reference attributes:

==========================  =========================  ==========================================
name                        shape                      reference
==========================  =========================  ==========================================
``patch_w`` / ``patch_b``   ``[p*p*c, D]`` / ``[D]``   ``patch_to_embedding`` vit.py:23
``cls``                     ``[D]``                    ``cls_token [1,1,D]`` vit.py:24-29
``pos``                     ``[P+1, D]``               ``pos_embedding`` vit.py:18-22
``l{i}.ln1_g/ln1_b``        ``[D]``                    attention-side ``LayerNorm`` norm.py:6
``l{i}.qkv_w``              ``[D, 3*h*hk]``            ``Attention.to_qkv`` (no bias) attention.py:17
``l{i}.out_w/out_b``        ``[h*hk, D]`` / ``[D]``    ``Attention.to_out`` attention.py:18
``l{i}.ln2_g/ln2_b``        ``[D]``                    FFN-side ``LayerNorm`` norm.py:6
``l{i}.fc1_w/fc1_b``        ``[D, F]`` / ``[F]``       ``FeedForward`` Dense 1 ffn.py:8
``l{i}.fc2_w/fc2_b``        ``[F, D]`` / ``[D]``       ``FeedForward`` Dense 2 ffn.py:9
``head1_w/head1_b``         ``[D, M]`` / ``[M]``       ``mlp_head[0]`` vit.py:38
``head2_w/head2_b``         ``[M, C]`` / ``[C]``       ``mlp_head[1]`` vit.py:39
==========================  =========================  ==========================================

Initialisers (Keras-like, with non-zero biases on purpose so every bias path is exercised):
glorot-uniform kernels, biases ~ N(0, 0.02), gamma = 1 + N(0, 0.02), beta ~ N(0, 0.02),
cls / pos ~ N(0, 0.05) (the Keras ``RandomNormal`` default, vit.py:21,28).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import numpy as np


@dataclass(frozen=True)
class ViTConfig:
    """Static shape of a `ViT` / `ViT_Pruned` (reference `modeling/models/vit.py:11-75`)."""

    image_size: int = 224
    patch_size: int = 16
    in_chans: int = 3
    num_classes: int = 1000
    dim: int = 768
    depth: int = 12
    mlp_dim: int = 3072           # head MLP width; also the unpruned FFN width
    heads: Sequence[int] = field(default_factory=lambda: (12,) * 12)   # per layer
    head_dim: Sequence[int] = field(default_factory=lambda: (64,) * 12)  # per layer h_k
    ffn: Sequence[int] = field(default_factory=lambda: (3072,) * 12)    # per layer width

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def tokens(self) -> int:
        return self.num_patches + 1

    @property
    def patch_dim(self) -> int:
        return self.patch_size * self.patch_size * self.in_chans

    def gflop_per_image(self) -> float:
        """Matmul FLOPs (2*MAC) of one image's forward; the roofline's algorithmic work."""
        n, p, d = self.tokens, self.num_patches, self.dim
        f = 2.0 * p * self.patch_dim * d
        for i in range(self.depth):
            inner = self.heads[i] * self.head_dim[i]
            f += 2.0 * n * d * 3 * inner              # QKV
            f += 2.0 * 2 * n * n * inner              # QK^T and P.V
            f += 2.0 * n * inner * d                  # out-proj
            f += 2.0 * 2 * n * d * self.ffn[i]        # FC1 + FC2
        f += 2.0 * d * self.mlp_dim + 2.0 * self.mlp_dim * self.num_classes
        return f / 1e9


def vit_config(dim: int, depth: int, heads: int, mlp_dim: int, *, image_size=224, patch_size=16,
               num_classes=1000, head_size: int | None = None,
               heads_list: Sequence[int] | None = None,
               ffn_list: Sequence[int] | None = None) -> ViTConfig:
    hk = head_size if head_size is not None else dim // heads
    hl = tuple(heads_list) if heads_list is not None else (heads,) * depth
    fl = tuple(ffn_list) if ffn_list is not None else (mlp_dim,) * depth
    return ViTConfig(image_size=image_size, patch_size=patch_size, num_classes=num_classes,
                     dim=dim, depth=depth, mlp_dim=mlp_dim, heads=hl,
                     head_dim=(hk,) * depth, ffn=fl)


def _glorot(rng: np.random.Generator, fan_in: int, fan_out: int) -> np.ndarray:
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out))


def vit_param_shapes(cfg: ViTConfig) -> List[tuple]:
    """Ordered (name, shape) list; this order is also the C-ABI weight-pointer order."""
    d = cfg.dim
    out = [("patch_w", (cfg.patch_dim, d)), ("patch_b", (d,)), ("cls", (d,)),
           ("pos", (cfg.tokens, d))]
    for i in range(cfg.depth):
        inner = cfg.heads[i] * cfg.head_dim[i]
        f = cfg.ffn[i]
        out += [(f"l{i}.ln1_g", (d,)), (f"l{i}.ln1_b", (d,)),
                (f"l{i}.qkv_w", (d, 3 * inner)),
                (f"l{i}.out_w", (inner, d)), (f"l{i}.out_b", (d,)),
                (f"l{i}.ln2_g", (d,)), (f"l{i}.ln2_b", (d,)),
                (f"l{i}.fc1_w", (d, f)), (f"l{i}.fc1_b", (f,)),
                (f"l{i}.fc2_w", (f, d)), (f"l{i}.fc2_b", (d,))]
    out += [("head1_w", (d, cfg.mlp_dim)), ("head1_b", (cfg.mlp_dim,)),
            ("head2_w", (cfg.mlp_dim, cfg.num_classes)), ("head2_b", (cfg.num_classes,))]
    return out


def make_vit_params(cfg: ViTConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded fp32 parameters for `cfg` (same values on every platform)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    params: Dict[str, np.ndarray] = {}
    for name, shape in vit_param_shapes(cfg):
        leaf = name.split(".")[-1]
        if leaf.endswith("_w"):
            v = _glorot(rng, shape[0], shape[1])
        elif leaf.endswith("_g"):
            v = 1.0 + rng.normal(0.0, 0.02, size=shape)
        elif leaf in ("cls", "pos"):
            v = rng.normal(0.0, 0.05, size=shape)
        else:  # biases, LN beta
            v = rng.normal(0.0, 0.02, size=shape)
        params[name] = np.ascontiguousarray(v, dtype=np.float32)
    return params


def std_vit_param_shapes(cfg: ViTConfig) -> List[tuple]:
    """(name, shape) list of the STANDARD-semantics ViT (timm / HF DeiT; EVT_VIT_STANDARD in
    include/evt.h): the reference order plus a qkv bias per layer, and a final LayerNorm + one
    Linear head instead of the two-layer mlp_head."""
    d = cfg.dim
    out = [("patch_w", (cfg.patch_dim, d)), ("patch_b", (d,)), ("cls", (d,)),
           ("pos", (cfg.tokens, d))]
    for i in range(cfg.depth):
        inner = cfg.heads[i] * cfg.head_dim[i]
        f = cfg.ffn[i]
        out += [(f"l{i}.ln1_g", (d,)), (f"l{i}.ln1_b", (d,)),
                (f"l{i}.qkv_w", (d, 3 * inner)), (f"l{i}.qkv_b", (3 * inner,)),
                (f"l{i}.out_w", (inner, d)), (f"l{i}.out_b", (d,)),
                (f"l{i}.ln2_g", (d,)), (f"l{i}.ln2_b", (d,)),
                (f"l{i}.fc1_w", (d, f)), (f"l{i}.fc1_b", (f,)),
                (f"l{i}.fc2_w", (f, d)), (f"l{i}.fc2_b", (d,))]
    out += [("norm_g", (d,)), ("norm_b", (d,)), ("head_w", (d, cfg.num_classes)),
            ("head_b", (cfg.num_classes,))]
    return out


def make_std_vit_params(cfg: ViTConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded fp32 parameters of a standard ViT (same init families as make_vit_params)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    params: Dict[str, np.ndarray] = {}
    for name, shape in std_vit_param_shapes(cfg):
        leaf = name.split(".")[-1]
        if leaf.endswith("_w"):
            v = _glorot(rng, shape[0], shape[1])
        elif leaf.endswith("_g"):
            v = 1.0 + rng.normal(0.0, 0.02, size=shape)
        elif leaf in ("cls", "pos"):
            v = rng.normal(0.0, 0.05, size=shape)
        else:
            v = rng.normal(0.0, 0.02, size=shape)
        params[name] = np.ascontiguousarray(v, dtype=np.float32)
    return params


@dataclass(frozen=True)
class T2TConfig:
    """Static shape of a `T2T_ViT` (reference `modeling/models/t2t_vit.py:91-114`).

    Tokens-to-token geometry (t2t_vit.py:50-52,61): soft_split0 k7 s4 p2, soft_split1/2 k3 s2 p1
    -> S/4, S/8, S/16 token grids; TokenPerformer head size `token_size`, m = token_size / 2
    random features (kernel_ratio 0.5, transformer_encoder.py:59).
    """

    image_size: int = 224
    in_chans: int = 3
    num_classes: int = 1000
    dim: int = 384                # hidden_size
    depth: int = 14
    heads: int = 6                # num_heads (head size h_k = dim // heads)
    mlp_dim: int = 1152           # int(mlp_ratio * hidden_size) (t2t_vit.py:110)
    token_size: int = 64

    @property
    def grids(self) -> tuple:
        s = self.image_size
        return (s // 4, s // 8, s // 16)

    @property
    def num_patches(self) -> int:
        return (self.image_size // 16) ** 2   # t2t_vit.py:61

    @property
    def tokens(self) -> int:
        return self.num_patches + 1

    @property
    def m(self) -> int:
        return int(self.token_size * 0.5)

    @property
    def split_dims(self) -> tuple:
        """Unfolded vector widths feeding performer1, performer2 and project."""
        return (49 * self.in_chans, 9 * self.token_size, 9 * self.token_size)

    def gflop_per_image(self) -> float:
        """Matmul FLOPs (2*MAC) per image: T2T stage + encoder + head."""
        hs, m = self.token_size, self.m
        g1, g2, g3 = self.grids
        f = 0.0
        for t, din in ((g1 * g1, self.split_dims[0]), (g2 * g2, self.split_dims[1])):
            f += 2.0 * t * din * 3 * hs                  # kqv
            f += 2.0 * 2 * t * hs * m                     # prm_exp(k), prm_exp(q)
            f += 2.0 * 2 * t * hs * m                     # kptv, qp . kptv
            f += 2.0 * 3 * t * hs * hs                    # attn_output, FFN x2
        f += 2.0 * g3 * g3 * self.split_dims[2] * self.dim   # project
        n, d = self.tokens, self.dim
        f += self.depth * (2.0 * n * d * 3 * d + 2.0 * 2 * n * n * d + 2.0 * n * d * d
                           + 2.0 * 2 * n * d * self.mlp_dim)
        f += 2.0 * d * self.num_classes
        return f / 1e9


def t2t_config(hidden_size: int, depth: int, num_heads: int, mlp_ratio: float, *,
               image_size: int = 224, num_classes: int = 1000, token_size: int = 64,
               in_channels: int = 3) -> T2TConfig:
    return T2TConfig(image_size=image_size, in_chans=in_channels, num_classes=num_classes,
                     dim=hidden_size, depth=depth, heads=num_heads,
                     mlp_dim=int(mlp_ratio * hidden_size), token_size=token_size)


def t2t_param_shapes(cfg: T2TConfig) -> List[tuple]:
    """Ordered (name, shape) list = the C-ABI weight order of evt_t2t_create (include/evt.h)."""
    hs, m, d = cfg.token_size, cfg.m, cfg.dim
    out = []
    for pre, din in (("p1.", cfg.split_dims[0]), ("p2.", cfg.split_dims[1])):
        out += [(pre + "ln1_g", (din,)), (pre + "ln1_b", (din,)),
                (pre + "kqv_w", (din, 3 * hs)), (pre + "kqv_b", (3 * hs,)),
                (pre + "w", (m, hs)),
                (pre + "out_w", (hs, hs)), (pre + "out_b", (hs,)),
                (pre + "ln2_g", (hs,)), (pre + "ln2_b", (hs,)),
                (pre + "fc1_w", (hs, hs)), (pre + "fc1_b", (hs,)),
                (pre + "fc2_w", (hs, hs)), (pre + "fc2_b", (hs,))]
    out += [("project_w", (cfg.split_dims[2], d)), ("project_b", (d,)), ("cls", (d,)),
            ("pos", (cfg.tokens, d))]
    for i in range(cfg.depth):
        inner = cfg.heads * (d // cfg.heads)  # Attention(hidden_size, num_heads): h_k = d // heads
        out += [(f"l{i}.ln1_g", (d,)), (f"l{i}.ln1_b", (d,)),
                (f"l{i}.qkv_w", (d, 3 * inner)),
                (f"l{i}.out_w", (inner, d)), (f"l{i}.out_b", (d,)),
                (f"l{i}.ln2_g", (d,)), (f"l{i}.ln2_b", (d,)),
                (f"l{i}.fc1_w", (d, cfg.mlp_dim)), (f"l{i}.fc1_b", (cfg.mlp_dim,)),
                (f"l{i}.fc2_w", (cfg.mlp_dim, d)), (f"l{i}.fc2_b", (d,))]
    out += [("norm_g", (d,)), ("norm_b", (d,)), ("head_w", (d, cfg.num_classes)),
            ("head_b", (cfg.num_classes,))]
    return out


def _orthogonal(rng: np.random.Generator, rows: int, cols: int) -> np.ndarray:
    """Keras `Orthogonal()` (gain 1) for a [rows, cols] kernel: QR of a Gaussian, sign-fixed."""
    a = rng.standard_normal((max(rows, cols), min(rows, cols)))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    return q.T if rows < cols else q


def make_t2t_params(cfg: T2TConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded fp32 parameters for a T2T-ViT (same families as make_vit_params; the performer
    feature matrix is Orthogonal * sqrt(m) (transformer_encoder.py:60-65) and the position table
    is the fixed sinusoid (t2t_vit.py:106-107))."""
    from math import sqrt
    rng = np.random.Generator(np.random.PCG64(seed))
    params: Dict[str, np.ndarray] = {}
    for name, shape in t2t_param_shapes(cfg):
        leaf = name.split(".")[-1]
        if leaf == "w":
            v = _orthogonal(rng, shape[0], shape[1]) * sqrt(shape[0])
        elif name == "pos":
            v = _sinusoid(shape[0], shape[1])
        elif leaf.endswith("_w"):
            v = _glorot(rng, shape[0], shape[1])
        elif leaf.endswith("_g"):
            v = 1.0 + rng.normal(0.0, 0.02, size=shape)
        elif leaf == "cls":
            v = rng.normal(0.0, 0.05, size=shape)
        else:  # biases, LN beta
            v = rng.normal(0.0, 0.02, size=shape)
        params[name] = np.ascontiguousarray(v, dtype=np.float32)
    return params


def _sinusoid(n_position: int, d_hid: int) -> np.ndarray:
    """Fixed sinusoid position table of reference `modeling/layers/embedding.py:4-15`."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)
    table = pos / np.power(10000.0, 2 * (j // 2) / d_hid)
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    return table.astype(np.float32)


def make_images(batch: int, seed: int = 1, image_size: int = 224, chans: int = 3,
                layout: str = "NCHW") -> np.ndarray:
    """Seeded N(0,1) fp32 images, the distribution of `tools.py:204` / `utils.py:482`."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.standard_normal((batch, chans, image_size, image_size), dtype=np.float32)
    if layout == "NHWC":
        x = np.ascontiguousarray(x.transpose(0, 2, 3, 1))
    return x


def digest(arrays: Dict[str, np.ndarray] | Sequence[np.ndarray]) -> str:
    """SHA-256 over the raw bytes (in order) - pins generator output in fixtures."""
    h = hashlib.sha256()
    items = arrays.items() if isinstance(arrays, dict) else enumerate(arrays)
    for k, v in items:
        h.update(str(k).encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()


@dataclass(frozen=True)
class SwinConfig:
    """Static shape of a Swin Transformer, the model the reference builds with `get_swin`
    (`utils.py:14-47`, config `swin_tiny_patch4_window7_224`, `tools.py:282`) from the external
    microsoft/Swin-Transformer repo (not vendored in the reference). Stage i has embed_dim * 2^i
    channels, num_heads[i] heads of size 32, depths[i] blocks alternating W-MSA / SW-MSA
    (shift window_size // 2), and a PatchMerging in front of every stage but the first.
    """

    image_size: int = 224
    patch_size: int = 4
    in_chans: int = 3
    num_classes: int = 1000
    embed_dim: int = 96
    depths: Sequence[int] = (2, 2, 6, 2)
    num_heads: Sequence[int] = (3, 6, 12, 24)
    window_size: int = 7
    mlp_ratio: float = 4.0

    @property
    def num_stages(self) -> int:
        return len(self.depths)

    def dim(self, i: int) -> int:
        return self.embed_dim * (1 << i)

    def res(self, i: int) -> int:
        return self.image_size // self.patch_size // (1 << i)

    def window(self, i: int) -> int:
        """Window of stage i: clamped to the resolution when that is not larger (the reference
        Swin's `min(input_resolution) <= window_size` rule: no shift then)."""
        return min(self.window_size, self.res(i))

    def shift(self, i: int, j: int) -> int:
        return 0 if (j % 2 == 0 or self.res(i) <= self.window_size) else self.window_size // 2

    def mlp(self, i: int) -> int:
        return int(self.dim(i) * self.mlp_ratio)

    @property
    def num_features(self) -> int:
        return self.dim(self.num_stages - 1)

    def gflop_per_image(self) -> float:
        """Matmul FLOPs (2*MAC) per image: patch embed, QKV / window attention / proj / MLP,
        patch merging, head (the MAC terms of the reference's `SwinFlops`,
        flops_calculation.py:313-386)."""
        f = 2.0 * self.res(0) ** 2 * self.in_chans * self.patch_size ** 2 * self.embed_dim
        for i in range(self.num_stages):
            n, c, w = self.res(i) ** 2, self.dim(i), self.window(i)
            per = 2.0 * n * c * 3 * c + 2.0 * 2 * n * w * w * c + 2.0 * n * c * c \
                + 2.0 * 2 * n * c * self.mlp(i)
            f += self.depths[i] * per
            if i + 1 < self.num_stages:
                f += 2.0 * (n // 4) * 4 * c * 2 * c
        f += 2.0 * self.num_features * self.num_classes
        return f / 1e9


SWIN_VARIANTS = {  # microsoft/Swin-Transformer configs/swin_{tiny,small,base}_patch4_window7_224.yaml
    "tiny": dict(embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24)),
    "small": dict(embed_dim=96, depths=(2, 2, 18, 2), num_heads=(3, 6, 12, 24)),
    "base": dict(embed_dim=128, depths=(2, 2, 18, 2), num_heads=(4, 8, 16, 32)),
}


def swin_config(variant: str = "tiny", **kw) -> SwinConfig:
    args = dict(SWIN_VARIANTS[variant])
    args.update(kw)
    args["depths"] = tuple(args["depths"])
    args["num_heads"] = tuple(args["num_heads"])
    return SwinConfig(**args)


def swin_param_shapes(cfg: SwinConfig) -> List[tuple]:
    """Ordered (name, shape) list = the C-ABI weight order of evt_swin_create (include/evt.h).
    Dense kernels are [in, out]; `patch_w` is the Conv2d(k=s=patch) kernel flattened to rows
    (c, kh, kw); `rpb` is the relative-position-bias table [(2w-1)^2, heads]."""
    e, p = cfg.embed_dim, cfg.patch_size
    out = [("patch_w", (cfg.in_chans * p * p, e)), ("patch_b", (e,)),
           ("pnorm_g", (e,)), ("pnorm_b", (e,))]
    for i in range(cfg.num_stages):
        c, h, w = cfg.dim(i), cfg.num_heads[i], cfg.window(i)
        if i > 0:
            cp = cfg.dim(i - 1)
            out += [(f"s{i}.merge_g", (4 * cp,)), (f"s{i}.merge_b", (4 * cp,)),
                    (f"s{i}.merge_w", (4 * cp, c))]
        for j in range(cfg.depths[i]):
            pre = f"s{i}.b{j}."
            out += [(pre + "ln1_g", (c,)), (pre + "ln1_b", (c,)),
                    (pre + "qkv_w", (c, 3 * c)), (pre + "qkv_b", (3 * c,)),
                    (pre + "rpb", ((2 * w - 1) ** 2, h)),
                    (pre + "proj_w", (c, c)), (pre + "proj_b", (c,)),
                    (pre + "ln2_g", (c,)), (pre + "ln2_b", (c,)),
                    (pre + "fc1_w", (c, cfg.mlp(i))), (pre + "fc1_b", (cfg.mlp(i),)),
                    (pre + "fc2_w", (cfg.mlp(i), c)), (pre + "fc2_b", (c,))]
    nf = cfg.num_features
    out += [("norm_g", (nf,)), ("norm_b", (nf,)), ("head_w", (nf, cfg.num_classes)),
            ("head_b", (cfg.num_classes,))]
    return out


def make_swin_params(cfg: SwinConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    """Seeded fp32 Swin parameters (families as make_vit_params; the relative-position-bias
    tables ~ N(0, 0.5), wider than the reference's trunc_normal(0.02) so that a wrong bias index
    shows in the logits)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    params: Dict[str, np.ndarray] = {}
    for name, shape in swin_param_shapes(cfg):
        leaf = name.split(".")[-1]
        if leaf == "rpb":
            v = rng.normal(0.0, 0.5, size=shape)
        elif leaf.endswith("_w"):
            v = _glorot(rng, shape[0], shape[1])
        elif leaf.endswith("_g"):
            v = 1.0 + rng.normal(0.0, 0.02, size=shape)
        else:  # biases, LN beta
            v = rng.normal(0.0, 0.02, size=shape)
        params[name] = np.ascontiguousarray(v, dtype=np.float32)
    return params
