"""Reference-side weight glue: a built reference Keras ViT's variables in the C-ABI weight order.

The C ABI (`evt_vit_create`, include/evt.h) takes the weights as an ordered pointer list
(`weights.vit_param_shapes`: patch Dense, cls, pos, then per block LN1, to_qkv, to_out, LN2, the
FeedForward Dense pair, then the two mlp_head Dense layers). A maintainer who keeps the
reference's own `modeling` package and swaps only the compute needs
that list from the Keras model. Two forms, neither importing TensorFlow:

  ordered_keras_variables(keras_vit)   walks the reference model's attributes
        ViT.pos_embedding / patch_to_embedding / cls_token / transformer / mlp_head
        (modeling/models/vit.py:18-39), each block's LayerNorm.norm (norm.py:6) around
        Residual.fn (residual.py:5-6) around Attention.to_qkv / to_out (attention.py:17-18) or
        FeedForward.net (ffn.py:8-9); ViT_Pruned's TransformerEncoderBlock_Pruned has the same
        structure with per-layer head counts / widths. Any object with those attributes works
        (tf.Variable, numpy array, anything np.asarray accepts).
  reorder_keras_weight_list(weights, cfg)   the same from `model.get_weights()` / `model.weights`
        order: the sub-layers' variables in attribute order, with the model's own add_weight
        variables (pos_embedding, then cls_token [1, 1, dim]) either before them (tf.keras Layer
        order) or after them (tf.keras Model order since TF 2.4); the 3-D cls_token tells which.
        Checked shape by shape against cfg.

keras_vit_config(keras_vit) reads the shape (dim, depth, per-layer heads, head size h_k and FFN
width, head MLP width, classes) off the same attributes, so no head size is hard-coded.
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from .weights import ViTConfig, vit_param_shapes


def _np(v) -> np.ndarray:
    if hasattr(v, "numpy"):
        v = v.numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32))


def _blocks(keras_vit):
    layers = list(keras_vit.transformer.net.layers)  # TransformerEncoderBlock(_Pruned).net
    if len(layers) % 2:
        raise ValueError("transformer.net must alternate attention / feed-forward sublayers")
    return [(layers[2 * i], layers[2 * i + 1]) for i in range(len(layers) // 2)]


def keras_vit_config(keras_vit, image_size: int = 224) -> ViTConfig:
    """ViTConfig of a built reference ViT / ViT_Pruned, from its variables' shapes."""
    pos = _np(keras_vit.pos_embedding)
    patch_w = _np(keras_vit.patch_to_embedding.kernel)
    dim = int(pos.shape[-1])
    patch_size = int(keras_vit.patch_size)
    in_chans = patch_w.shape[0] // (patch_size * patch_size)
    heads, head_dim, ffn = [], [], []
    for att_ln, ffn_ln in _blocks(keras_vit):
        att = att_ln.fn.fn
        heads.append(int(att.num_heads))
        head_dim.append(int(att.h_k))
        ffn.append(int(_np(ffn_ln.fn.fn.net.layers[0].kernel).shape[1]))
    head1 = _np(keras_vit.mlp_head.layers[0].kernel)
    head2 = _np(keras_vit.mlp_head.layers[1].kernel)
    cfg = ViTConfig(image_size=image_size, patch_size=patch_size, in_chans=in_chans,
                    num_classes=int(head2.shape[1]), dim=dim, depth=len(heads),
                    mlp_dim=int(head1.shape[1]), heads=tuple(heads), head_dim=tuple(head_dim),
                    ffn=tuple(ffn))
    if pos.shape[0] != cfg.tokens:
        raise ValueError(f"pos_embedding has {pos.shape[0]} rows, image_size {image_size} / "
                         f"patch {patch_size} gives {cfg.tokens} tokens")
    return cfg


def keras_vit_params(keras_vit) -> Dict[str, np.ndarray]:
    """{vit_param_shapes name: fp32 array} of a built reference ViT (attribute walk)."""
    m = keras_vit
    p = {"patch_w": _np(m.patch_to_embedding.kernel), "patch_b": _np(m.patch_to_embedding.bias),
         "cls": _np(m.cls_token).reshape(-1), "pos": _np(m.pos_embedding)}
    for i, (att_ln, ffn_ln) in enumerate(_blocks(m)):
        att, ffn = att_ln.fn.fn, ffn_ln.fn.fn  # LayerNorm(Residual(...)): norm.py:11-12, residual.py:9
        p[f"l{i}.ln1_g"], p[f"l{i}.ln1_b"] = _np(att_ln.norm.gamma), _np(att_ln.norm.beta)
        p[f"l{i}.qkv_w"] = _np(att.to_qkv.kernel)  # use_bias=False (attention.py:17)
        p[f"l{i}.out_w"], p[f"l{i}.out_b"] = _np(att.to_out.kernel), _np(att.to_out.bias)
        p[f"l{i}.ln2_g"], p[f"l{i}.ln2_b"] = _np(ffn_ln.norm.gamma), _np(ffn_ln.norm.beta)
        fc1, fc2 = ffn.net.layers[0], ffn.net.layers[1]
        p[f"l{i}.fc1_w"], p[f"l{i}.fc1_b"] = _np(fc1.kernel), _np(fc1.bias)
        p[f"l{i}.fc2_w"], p[f"l{i}.fc2_b"] = _np(fc2.kernel), _np(fc2.bias)
    h1, h2 = m.mlp_head.layers[0], m.mlp_head.layers[1]
    p["head1_w"], p["head1_b"] = _np(h1.kernel), _np(h1.bias)
    p["head2_w"], p["head2_b"] = _np(h2.kernel), _np(h2.bias)
    return p


def _checked(p: Dict[str, np.ndarray], cfg: ViTConfig) -> List[np.ndarray]:
    out = []
    for name, shape in vit_param_shapes(cfg):
        if tuple(p[name].shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(p[name].shape)}, expected {tuple(shape)}")
        out.append(p[name])
    return out


def ordered_keras_variables(keras_vit, image_size: int = 224) -> List[np.ndarray]:
    """The reference model's variables as fp32 arrays in the evt_vit_num_weights order."""
    return _checked(keras_vit_params(keras_vit), keras_vit_config(keras_vit, image_size))


def keras_weight_names(cfg: ViTConfig, own_first: bool = False,
                       head_first: bool = False) -> List[str]:
    """vit_param_shapes names in Keras tracking order (model.weights / get_weights()): the
    sub-layers (patch_to_embedding, the blocks, mlp_head) in attribute order, the model's own
    pos_embedding / cls_token after them (tf.keras Model) or before them (own_first).
    head_first: the ViT_Pruned order. Its constructor assigns a new `self.transformer` after
    `ViT.__init__` (reference vit.py:74); Keras untracks the replaced block and appends the new
    one, so the blocks follow mlp_head: patch_to_embedding, mlp_head, transformer."""
    blocks = []
    for i in range(cfg.depth):
        blocks += [f"l{i}.{n}" for n in ("ln1_g", "ln1_b", "qkv_w", "out_w", "out_b", "ln2_g",
                                         "ln2_b", "fc1_w", "fc1_b", "fc2_w", "fc2_b")]
    head = ["head1_w", "head1_b", "head2_w", "head2_b"]
    names = ["patch_w", "patch_b"] + (head + blocks if head_first else blocks + head)
    return ["pos", "cls"] + names if own_first else names + ["pos", "cls"]


def reorder_keras_weight_list(weights: Sequence, cfg: ViTConfig) -> List[np.ndarray]:
    """`model.get_weights()` of a reference ViT or ViT_Pruned (Keras tracking order) -> the C-ABI
    order. The order is read off the list itself: the [1, 1, dim] cls_token at the front or the
    end (the model's own variables before / after its sub-layers), and after patch_b either the
    rank-1 [dim] LayerNorm gamma of block 0 (ViT) or the rank-2 [dim, mlp_dim] kernel of the first
    mlp_head Dense (ViT_Pruned's re-tracked transformer, keras_weight_names)."""
    n = len(keras_weight_names(cfg))
    if len(weights) != n:
        raise ValueError(f"{len(weights)} Keras weights, the config has {n}")
    if np.ndim(weights[1]) == 3:
        own_first = True
    elif np.ndim(weights[-1]) == 3:
        own_first = False
    else:
        raise ValueError("no [1, 1, dim] cls_token at either end of the weight list")
    after_patch = weights[4 if own_first else 2]
    if cfg.depth == 0 or np.ndim(after_patch) == 2:
        head_first = cfg.depth > 0
    elif np.ndim(after_patch) == 1:
        head_first = False
    else:
        raise ValueError(f"unexpected rank-{np.ndim(after_patch)} weight after patch_to_embedding")
    names = keras_weight_names(cfg, own_first=own_first, head_first=head_first)
    p = {nm: _np(w) for nm, w in zip(names, weights)}
    p["cls"] = p["cls"].reshape(-1)  # [1, 1, dim] (vit.py:24-29)
    return _checked(p, cfg)
