"""Pruned-checkpoint ingestion: turn the reference's pruning outputs into `ViT_Pruned` models.

The reference prunes DeiT in two places and benchmarks the result through `ViT_Pruned`'s
layerwise encoding (`modeling/models/vit.py:58-97`, `experiments.py:171-204`), which only carries
head COUNTS and FFN fractions. A real pruned checkpoint also says WHICH heads / neurons survive;
this module maps both reference sources onto exact per-layer shapes and sliced weights:

  * nn_pruning (`deit_pruning/vendor/nn_pruning_v1/nn_pruning/patch_coordinator.py:397-406`
    `parse_layerwise_sparsity`; `inference_model_patcher.py:26-89` `get_pruned_heads`): per-layer
    thresholds "h_{head}_d_{ffn}-h_..." and head selection by the count of non-zero rows of the
    q / k / v blocks of each head (lowest scores pruned, at least one head kept).
  * are_16_heads (`are_16_heads/deit_{tiny,small,base}_head_importance.txt`): a [layers, heads]
    importance table (whitespace separated); heads are kept by importance.

`prune_vit_params` slices a Keras-layout parameter dict (weights.vit_param_shapes) to the kept
heads / FFN neurons (q, k, v columns and out-proj rows of the kept heads in their original order;
fc1 columns / fc2 rows of the kept neurons); `build_pruned_vit` makes the MI355X model with those
exact shapes. Host-only (numpy); the forward runs on the GPU like any ViT_Pruned.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .weights import ViTConfig, vit_config


def parse_layerwise_thresholds(spec: str) -> List[Dict[str, float]]:
    """patch_coordinator.py:397-406: "h_0.5_d_0.3-h_..." -> [{'head': 0.5, 'ffn': 0.3}, ...]."""
    out = []
    for item in spec.split("-"):
        parts = item.split("_")
        out.append({"head": float(parts[1]), "ffn": float(parts[-1])})
    return out


def thresholds_to_encoding(thresholds: Sequence[Dict[str, float]], num_heads: int) -> str:
    """The ViT_Pruned layerwise encoding (vit.py:77-97) with the head counts nn_pruning keeps:
    int(threshold * heads) (inference_model_patcher.py: to_prune = heads - int(thr * heads), at
    least one head kept)."""
    toks = []
    for t in thresholds:
        keep = max(1, int(t["head"] * num_heads))
        toks.append(f"h{keep}-d{t['ffn']}")
    return "layerwise_" + "_".join(toks)


def head_scores_nonzero(qkv_w: np.ndarray, heads: int, head_size: int) -> np.ndarray:
    """inference_model_patcher.py `analyze_head` summed over q, k, v: for each head, how many of
    the three [head_size, D] weight blocks have any non-zero entry (0..3). `qkv_w` is the Keras
    [D, 3 * heads * head_size] kernel, columns (qkv h d)."""
    d = qkv_w.shape[0]
    w = qkv_w.reshape(d, 3, heads, head_size)
    return (w != 0).any(axis=(0, 3)).sum(axis=0).astype(np.int64)


def select_heads_nn_pruning(scores: np.ndarray, threshold: float) -> List[int]:
    """Kept heads as get_pruned_heads computes them: prune the H - int(thr * H) lowest-scoring
    heads (stable ascending sort, torch.sort order for ties), never all of them (head 0 stays)."""
    h = len(scores)
    n_prune = h - int(threshold * h)
    order = np.argsort(scores, kind="stable")
    pruned = set(int(i) for i in order[:n_prune])
    if len(pruned) == h:
        pruned.discard(0)
    return [i for i in range(h) if i not in pruned]


def load_head_importance(path: str) -> np.ndarray:
    """are_16_heads/deit_*_head_importance.txt -> float [layers, heads]."""
    rows = [[float(v) for v in line.split()] for line in open(path) if line.strip()]
    return np.asarray(rows, dtype=np.float64)


def heads_from_importance(importance: np.ndarray, keep_per_layer: Optional[Sequence[int]] = None,
                          keep_total: Optional[int] = None) -> List[List[int]]:
    """Kept heads per layer, most important first kept: either a per-layer count, or a global
    budget (the are-16-heads iterative scheme: the least important heads of the whole model go
    first; every layer keeps at least one head). Returned indices are sorted."""
    layers, heads = importance.shape
    if keep_per_layer is not None:
        return [sorted(int(i) for i in np.argsort(-importance[l], kind="stable")[:max(1, k)])
                for l, k in enumerate(keep_per_layer)]
    if keep_total is None:
        raise ValueError("give keep_per_layer or keep_total")
    order = np.argsort(importance.reshape(-1), kind="stable")  # least important first
    alive = np.ones((layers, heads), dtype=bool)
    to_remove = layers * heads - keep_total
    for flat in order:
        if to_remove <= 0:
            break
        l, h = divmod(int(flat), heads)
        if alive[l].sum() > 1:
            alive[l, h] = False
            to_remove -= 1
    return [[int(h) for h in np.nonzero(alive[l])[0]] for l in range(layers)]


def ffn_keep_by_norm(params: Dict[str, np.ndarray], layer: int, keep: int) -> List[int]:
    """FFN neurons to keep when only a fraction is known: the `keep` largest by
    ||fc1 column|| * ||fc2 row|| (a magnitude proxy; nn_pruning zeroes whole rows/columns, for
    which this picks exactly the non-zero neurons)."""
    w1, w2 = params[f"l{layer}.fc1_w"], params[f"l{layer}.fc2_w"]
    score = np.linalg.norm(w1, axis=0) * np.linalg.norm(w2, axis=1)
    return sorted(int(i) for i in np.argsort(-score, kind="stable")[:keep])


def prune_vit_params(params: Dict[str, np.ndarray], cfg: ViTConfig, kept_heads: List[List[int]],
                     kept_ffn: Optional[List[List[int]]] = None,
                     head_size: int = 64) -> Tuple[Dict[str, np.ndarray], ViTConfig]:
    """Slice an unpruned parameter dict to the kept heads / FFN neurons -> (params, config)."""
    depth = cfg.depth
    if len(kept_heads) != depth or (kept_ffn is not None and len(kept_ffn) != depth):
        raise ValueError("one kept list per layer")
    out = dict(params)
    heads_l, ffn_l = [], []
    for i in range(depth):
        h_all = cfg.heads[i]
        kh = list(kept_heads[i])
        if not kh or min(kh) < 0 or max(kh) >= h_all:
            raise ValueError(f"layer {i}: kept heads {kh} out of range 0..{h_all - 1}")
        d = params[f"l{i}.qkv_w"].shape[0]
        qkv = params[f"l{i}.qkv_w"].reshape(d, 3, h_all, head_size)[:, :, kh, :]
        out[f"l{i}.qkv_w"] = np.ascontiguousarray(qkv.reshape(d, 3 * len(kh) * head_size))
        ow = params[f"l{i}.out_w"].reshape(h_all, head_size, -1)[kh]
        out[f"l{i}.out_w"] = np.ascontiguousarray(ow.reshape(len(kh) * head_size, -1))
        heads_l.append(len(kh))
        if kept_ffn is not None:
            kf = list(kept_ffn[i])
            out[f"l{i}.fc1_w"] = np.ascontiguousarray(params[f"l{i}.fc1_w"][:, kf])
            out[f"l{i}.fc1_b"] = np.ascontiguousarray(params[f"l{i}.fc1_b"][kf])
            out[f"l{i}.fc2_w"] = np.ascontiguousarray(params[f"l{i}.fc2_w"][kf, :])
            ffn_l.append(len(kf))
        else:
            ffn_l.append(cfg.ffn[i])
    new_cfg = vit_config(cfg.dim, depth, max(cfg.heads), cfg.mlp_dim, image_size=cfg.image_size,
                         patch_size=cfg.patch_size, num_classes=cfg.num_classes,
                         head_size=head_size, heads_list=heads_l, ffn_list=ffn_l)
    return out, new_cfg


def build_pruned_vit(params: Dict[str, np.ndarray], cfg: ViTConfig, kept_heads: List[List[int]],
                     kept_ffn: Optional[List[List[int]]] = None, **kw):
    """The MI355X ViT of a pruned checkpoint (exact per-layer shapes; needs the GPU)."""
    from .modeling.models.vit import ViT
    p, c = prune_vit_params(params, cfg, kept_heads, kept_ffn)
    return ViT(image_size=c.image_size, patch_size=c.patch_size, num_classes=c.num_classes,
               dim=c.dim, depth=c.depth, heads=max(cfg.heads), mlp_dim=c.mlp_dim, weights=p,
               _cfg=c, **kw)
