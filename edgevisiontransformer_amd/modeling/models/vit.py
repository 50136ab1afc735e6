"""MI355X mirror of the reference `modeling/models/vit.py` (ViT, ViT_Pruned, get_deit_*).

Same public names, constructor keywords and prune-encoding grammar as the reference; the Keras
graph is replaced by one call into libevt_hip.so (`evt_vit_forward`, include/evt.h), which runs
the whole forward as hand-written gfx950 kernels on the caller's HIP stream.

    model = get_deit_base(dtype="bf16")          # reference: get_deit_base()  vit.py:100-101
    logits = model(img)                          # reference: ViT.call          vit.py:41-55

Differences that are deliberate and documented:
  * Weights. The reference random-initialises Keras variables (vit.py:18-39) and never loads a
    checkpoint on this path. Here `seed=` selects the deterministic generator of
    `edgevisiontransformer_amd.weights` (same init families); `weights=` accepts an explicit
    {name: array} dict in the Keras [in, out] layout instead.
  * `dtype`: "bf16" (bf16 MFMA, fp32 accumulate/statistics; the throughput path) or "f32" (exact
    fp32 MFMA; logits within 1e-3 of the fp64 oracle).
  * Input: fp32 NCHW [B, 3, H, W] torch tensor on the GPU (or a numpy array, copied in).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ... import _lib
from ...weights import (ViTConfig, make_std_vit_params, make_vit_params, std_vit_param_shapes,
                        vit_config, vit_param_shapes)


def decode_prune_encoding(prune_encoding: str):
    """Reference `ViT_Pruned.decode_prune_encoding` (vit.py:77-97), same grammar and asserts.

    'all_head{N}_ffn{F}'                  -> ('all', N, F)
    'layerwise_h{N}-d{F}_h{N}-d{F}_...'   -> ('layerwise', [N...], [F...])
    """
    tokens = prune_encoding.split("_")
    prune_setting = tokens[0]
    assert prune_setting in ["layerwise", "all"]
    if prune_setting == "all":
        head_setting = tokens[1]
        ffn_setting = tokens[2]
        num_heads = int(head_setting.replace("head", ""))
        ffn_threshold = float(ffn_setting.replace("ffn", ""))
        return prune_setting, num_heads, ffn_threshold
    num_heads_list = []
    ffn_threshold_list = []
    for token in tokens[1:]:
        hx, dx = token.split("-")
        num_heads_list.append(int(hx.replace("h", "")))
        ffn_threshold_list.append(float(dx.replace("d", "")))
    return prune_setting, num_heads_list, ffn_threshold_list


def _to_device_image(img, device) -> Tuple[torch.Tensor, bool]:
    if isinstance(img, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(img, dtype=np.float32)).to(device), True
    if not isinstance(img, torch.Tensor):
        raise TypeError("img must be a torch.Tensor or numpy.ndarray")
    if img.dtype != torch.float32:
        img = img.float()
    if img.device != device:
        img = img.to(device)
    return img.contiguous(), False


def _capture_graph(model, img: torch.Tensor, logits: torch.Tensor) -> None:
    b = img.shape[0]
    if b > model._max_batch:
        model._build(b)
    lib = _lib.load_library()
    stream = torch.cuda.Stream(model.device)  # capture needs a non-default stream
    stream.wait_stream(torch.cuda.current_stream(model.device))
    with torch.cuda.stream(stream):
        _lib.check(lib.evt_graph_capture(ctypes.c_void_p(model._handle),
                                         ctypes.c_void_p(img.data_ptr()), b,
                                         ctypes.c_void_p(logits.data_ptr()),
                                         ctypes.c_void_p(stream.cuda_stream)))
    torch.cuda.current_stream(model.device).wait_stream(stream)
    model._graph_io = (img, logits, b)  # keep the captured buffers alive


def _replay_graph(model) -> None:
    if not getattr(model, "_graph_io", None):
        raise RuntimeError("no captured graph: call capture_graph(img, logits) first")
    _lib.check(_lib.load_library().evt_graph_launch(
        ctypes.c_void_p(model._handle), ctypes.c_void_p(_lib.stream_ptr(model.device))))


class ViT:
    """Vision Transformer forward on MI355X (reference `ViT`, vit.py:9-55)."""

    SEMANTICS = _lib.VIT_REFERENCE
    _param_shapes = staticmethod(vit_param_shapes)
    _make_params = staticmethod(make_vit_params)
    layer_norm_eps = 0.0  # 0: the library default 1e-5 (reference norm.py:6)

    def __init__(self, *, image_size=224, patch_size=16, num_classes=1000, dim=768, depth=12,
                 heads=12, mlp_dim=3072, dtype: str = "bf16", seed: int = 0,
                 weights: Optional[Dict[str, np.ndarray]] = None, device=None, max_batch: int = 0,
                 lanes: Optional[int] = None, _cfg: Optional[ViTConfig] = None):
        assert image_size % patch_size == 0, "image dimensions must be divisible by the patch size"
        if _cfg is None:
            if dim % heads != 0:  # reference Attention raises ValueError (attention.py:8-9)
                raise ValueError(f"hidden_size {dim} must be a multiple of num_heads {heads}.")
            _cfg = vit_config(dim, depth, heads, mlp_dim, image_size=image_size,
                              patch_size=patch_size, num_classes=num_classes)
        self.cfg = _cfg
        self.image_size, self.patch_size = image_size, patch_size
        self.num_classes, self.dim, self.depth, self.mlp_dim = num_classes, dim, depth, mlp_dim
        if dtype not in _lib.DTYPE:
            raise ValueError(f"dtype must be one of {sorted(_lib.DTYPE)}")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        _lib.ensure_device(self.device.index or 0)
        params = weights if weights is not None else self._make_params(self.cfg, seed=seed)
        self._weights: List[torch.Tensor] = []
        for name, shape in self._param_shapes(self.cfg):
            a = np.asarray(params[name], dtype=np.float32)
            if tuple(a.shape) != tuple(shape):
                if a.size == int(np.prod(shape)) and name == "cls":
                    a = a.reshape(shape)
                else:
                    raise ValueError(f"weight {name}: shape {a.shape}, expected {shape}")
            self._weights.append(torch.from_numpy(np.ascontiguousarray(a)).to(self.device))
        self._handle: Optional[int] = None
        self._max_batch = 0
        self._arrays = None
        # batch lanes (evt_model_set_lanes): None = _lib.default_lanes
        self._lanes = lanes
        if max_batch:
            self._build(max_batch)

    # -- C ABI plumbing ---------------------------------------------------------------------
    def _desc(self, max_batch: int):
        c = self.cfg
        arr = lambda v: (ctypes.c_int32 * max(1, len(v)))(*v)  # noqa: E731
        heads, hd, ffn = arr(list(c.heads)), arr(list(c.head_dim)), arr(list(c.ffn))
        self._arrays = (heads, hd, ffn)  # keep alive
        return _lib.evt_vit_desc(c.image_size, c.patch_size, c.in_chans, c.num_classes, c.dim,
                                 c.depth, c.mlp_dim, heads, hd, ffn, _lib.DTYPE[self.dtype],
                                 max_batch, self.SEMANTICS, self.layer_norm_eps)

    def _build(self, max_batch: int) -> None:
        lib = _lib.load_library()
        self.close()
        self._graph_io = None
        desc = self._desc(max_batch)
        n = lib.evt_vit_num_weights(ctypes.byref(desc))
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in self._weights])
        out = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            stream = _lib.stream_ptr(self.device)
            _lib.check(lib.evt_vit_create(ctypes.byref(desc), ptrs, n, ctypes.c_void_p(stream),
                                          ctypes.byref(out)))
        self._handle = out.value
        self._max_batch = max_batch
        with torch.cuda.device(self.device):
            self._lane_streams = _lib.set_lanes(
                self._handle, self._lanes if self._lanes is not None
                else _lib.default_lanes(self.dtype, max_batch, vit=True), self.device)

    def lanes(self) -> int:
        """Batch lanes of the handle (include/evt.h evt_model_set_lanes; 1 = none)."""
        out = ctypes.c_int()
        _lib.check(_lib.load_library().evt_model_lanes(ctypes.c_void_p(self._handle),
                                                       ctypes.byref(out)))
        return out.value

    def qkv_headmajor_layers(self) -> int:
        """Encoder layers whose QKV output was stored head-major in the last forward
        (evt_model_qkv_layout; diagnostics for the layout-equality tests)."""
        out = ctypes.c_int()
        _lib.check(_lib.load_library().evt_model_qkv_layout(ctypes.c_void_p(self._handle),
                                                             ctypes.byref(out)))
        return out.value

    def workspace_bytes(self, batch: int) -> int:
        lib = _lib.load_library()
        out = ctypes.c_size_t()
        _lib.check(lib.evt_query_workspace(ctypes.byref(self._desc(batch)), batch, ctypes.byref(out)))
        return out.value

    def close(self) -> None:
        if self._handle:
            _lib.load_library().evt_model_destroy(ctypes.c_void_p(self._handle))
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- forward ------------------------------------------------------------------------------
    def forward_into(self, img: torch.Tensor, logits: torch.Tensor) -> torch.Tensor:
        """Enqueue the forward of a device-resident fp32 NCHW batch into `logits` (no allocation)."""
        b = img.shape[0]
        if b > self._max_batch:
            self._build(b)
        lib = _lib.load_library()
        _lib.check(lib.evt_vit_forward(ctypes.c_void_p(self._handle), ctypes.c_void_p(img.data_ptr()),
                                       b, ctypes.c_void_p(logits.data_ptr()),
                                       ctypes.c_void_p(_lib.stream_ptr(self.device))))
        return logits

    # -- HIP graph ----------------------------------------------------------------------------
    def capture_graph(self, img: torch.Tensor, logits: torch.Tensor) -> None:
        """Record one forward of the device buffers (img, logits) as a HIP graph
        (evt_graph_capture); replay_graph() re-runs it after the caller refills img in place."""
        _capture_graph(self, img, logits)

    def replay_graph(self) -> None:
        _replay_graph(self)

    def __call__(self, img: Union[torch.Tensor, np.ndarray]):
        x, was_numpy = _to_device_image(img, self.device)
        c = self.cfg
        if x.dim() != 4 or tuple(x.shape[1:]) != (c.in_chans, c.image_size, c.image_size):
            raise ValueError(f"expected NCHW [B, {c.in_chans}, {c.image_size}, {c.image_size}], "
                             f"got {tuple(x.shape)}")
        logits = torch.empty((x.shape[0], c.num_classes), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            self.forward_into(x, logits)
        # stream-ordered, as every torch op: a numpy input gets numpy logits (.cpu() waits for
        # them), a device tensor gets device logits without a host sync
        return logits.cpu().numpy() if was_numpy else logits

    call = __call__


class ViT_Pruned(ViT):
    """Head/FFN-pruned ViT (reference `ViT_Pruned`, vit.py:58-75)."""

    def __init__(self, *, image_size=224, patch_size=16, num_classes=1000, dim=768, depth=12,
                 heads=12, mlp_dim=3072, head_size=64, prune_encoding="all_head12_ffn1.0",
                 **kw):
        prune_setting, num_remain_heads, ffn_thresholds = self.decode_prune_encoding(prune_encoding)
        if prune_setting == "all":
            num_remain_heads_list = [num_remain_heads for _ in range(depth)]
            intermediate_size_list = [int(ffn_thresholds * mlp_dim) for _ in range(depth)]
        else:
            assert len(num_remain_heads) == depth and len(ffn_thresholds) == depth
            num_remain_heads_list = num_remain_heads
            intermediate_size_list = [int(ffn_thresholds[i] * mlp_dim) for i in range(depth)]
        self.prune_encoding = prune_encoding
        self.num_remain_heads_list = num_remain_heads_list
        self.intermediate_size_list = intermediate_size_list
        cfg = vit_config(dim, depth, heads, mlp_dim, image_size=image_size, patch_size=patch_size,
                         num_classes=num_classes, head_size=head_size,
                         heads_list=num_remain_heads_list, ffn_list=intermediate_size_list)
        super().__init__(image_size=image_size, patch_size=patch_size, num_classes=num_classes,
                         dim=dim, depth=depth, heads=heads, mlp_dim=mlp_dim, _cfg=cfg, **kw)

    @staticmethod
    def decode_prune_encoding(prune_encoding: str):
        return decode_prune_encoding(prune_encoding)


def get_deit_base(**kw) -> ViT:
    return ViT(dim=768, depth=12, **kw)


def get_deit_small(**kw) -> ViT:
    return ViT(dim=384, heads=6, mlp_dim=384 * 4, **kw)


def get_deit_tiny(**kw) -> ViT:
    return ViT(dim=192, heads=3, mlp_dim=192 * 4, **kw)


def pruned_config(prune_encoding: str, *, dim: int, depth: int, heads: int, mlp_dim: int,
                  head_size: int = 64, image_size=224, patch_size=16, num_classes=1000) -> ViTConfig:
    """The ViTConfig a `ViT_Pruned(...)` builds (host-only; no GPU needed)."""
    setting, nh, thr = decode_prune_encoding(prune_encoding)
    if setting == "all":
        hl, fl = [nh] * depth, [int(thr * mlp_dim)] * depth
    else:
        assert len(nh) == depth and len(thr) == depth
        hl, fl = nh, [int(t * mlp_dim) for t in thr]
    return vit_config(dim, depth, heads, mlp_dim, image_size=image_size, patch_size=patch_size,
                      num_classes=num_classes, head_size=head_size, heads_list=hl, ffn_list=fl)


class StandardViT(ViT):
    """The published DeiT / ViT architecture (timm `VisionTransformer`, HF `ViTForImageClassification`
    — what the reference evaluates for accuracy via `get_torch_deit`, utils.py:52-62): pre-norm
    residual x + f(LN(x)), QKV with bias, exact GELU, final LayerNorm, Linear head on the CLS token.
    Load real checkpoints with `params_from_timm_state_dict` / `params_from_hf_state_dict`."""

    SEMANTICS = _lib.VIT_STANDARD
    _param_shapes = staticmethod(std_vit_param_shapes)
    _make_params = staticmethod(make_std_vit_params)

    def __init__(self, *, image_size=224, patch_size=16, num_classes=1000, dim=768, depth=12,
                 heads=12, mlp_ratio=4.0, layer_norm_eps=1e-6, **kw):
        self.layer_norm_eps = float(layer_norm_eps)
        super().__init__(image_size=image_size, patch_size=patch_size, num_classes=num_classes,
                         dim=dim, depth=depth, heads=heads, mlp_dim=int(dim * mlp_ratio), **kw)


def deit_tiny_patch16_224(**kw) -> StandardViT:
    return StandardViT(dim=192, heads=3, **kw)


def deit_small_patch16_224(**kw) -> StandardViT:
    return StandardViT(dim=384, heads=6, **kw)


def deit_base_patch16_224(**kw) -> StandardViT:
    return StandardViT(dim=768, heads=12, **kw)


def _patch_rows(conv_w: np.ndarray) -> np.ndarray:
    """Conv2d kernel [D, C, p, p] -> patch_w [p*p*C, D] in this build's (p1 p2 c) vector order
    (the reference's einops pattern, vit.py:31-32)."""
    d = conv_w.shape[0]
    return np.ascontiguousarray(conv_w.transpose(2, 3, 1, 0).reshape(-1, d))


def params_from_timm_state_dict(sd: Dict[str, np.ndarray], depth: int) -> Dict[str, np.ndarray]:
    """timm `VisionTransformer` / `deit_*_patch16_224` state dict -> StandardViT parameters."""
    a = lambda k: np.asarray(sd[k], dtype=np.float32)  # noqa: E731
    p = {"patch_w": _patch_rows(a("patch_embed.proj.weight")), "patch_b": a("patch_embed.proj.bias"),
         "cls": a("cls_token").reshape(-1), "pos": a("pos_embed")[0],
         "norm_g": a("norm.weight"), "norm_b": a("norm.bias"),
         "head_w": a("head.weight").T, "head_b": a("head.bias")}
    for i in range(depth):
        s = f"blocks.{i}."
        p.update({f"l{i}.ln1_g": a(s + "norm1.weight"), f"l{i}.ln1_b": a(s + "norm1.bias"),
                  f"l{i}.qkv_w": a(s + "attn.qkv.weight").T, f"l{i}.qkv_b": a(s + "attn.qkv.bias"),
                  f"l{i}.out_w": a(s + "attn.proj.weight").T, f"l{i}.out_b": a(s + "attn.proj.bias"),
                  f"l{i}.ln2_g": a(s + "norm2.weight"), f"l{i}.ln2_b": a(s + "norm2.bias"),
                  f"l{i}.fc1_w": a(s + "mlp.fc1.weight").T, f"l{i}.fc1_b": a(s + "mlp.fc1.bias"),
                  f"l{i}.fc2_w": a(s + "mlp.fc2.weight").T, f"l{i}.fc2_b": a(s + "mlp.fc2.bias")})
    return {k: np.ascontiguousarray(v) for k, v in p.items()}


def params_from_hf_state_dict(sd: Dict[str, np.ndarray], depth: int) -> Dict[str, np.ndarray]:
    """HF `ViTForImageClassification` (facebook/deit-*-patch16-224) state dict -> parameters."""
    a = lambda k: np.asarray(sd[k], dtype=np.float32)  # noqa: E731
    e = "vit.embeddings."
    p = {"patch_w": _patch_rows(a(e + "patch_embeddings.projection.weight")),
         "patch_b": a(e + "patch_embeddings.projection.bias"),
         "cls": a(e + "cls_token").reshape(-1), "pos": a(e + "position_embeddings")[0],
         "norm_g": a("vit.layernorm.weight"), "norm_b": a("vit.layernorm.bias"),
         "head_w": a("classifier.weight").T, "head_b": a("classifier.bias")}
    for i in range(depth):
        s = f"vit.layers.{i}."
        q, k, v = (a(s + f"attention.{n}_proj.weight") for n in "qkv")
        qb, kb, vb = (a(s + f"attention.{n}_proj.bias") for n in "qkv")
        p.update({f"l{i}.ln1_g": a(s + "layernorm_before.weight"),
                  f"l{i}.ln1_b": a(s + "layernorm_before.bias"),
                  f"l{i}.qkv_w": np.concatenate([q, k, v], 0).T,
                  f"l{i}.qkv_b": np.concatenate([qb, kb, vb]),
                  f"l{i}.out_w": a(s + "attention.o_proj.weight").T,
                  f"l{i}.out_b": a(s + "attention.o_proj.bias"),
                  f"l{i}.ln2_g": a(s + "layernorm_after.weight"),
                  f"l{i}.ln2_b": a(s + "layernorm_after.bias"),
                  f"l{i}.fc1_w": a(s + "mlp.fc1.weight").T, f"l{i}.fc1_b": a(s + "mlp.fc1.bias"),
                  f"l{i}.fc2_w": a(s + "mlp.fc2.weight").T, f"l{i}.fc2_b": a(s + "mlp.fc2.bias")})
    return {k: np.ascontiguousarray(v) for k, v in p.items()}


_NAMED = {
    "deit_base": dict(dim=768, depth=12, heads=12, mlp_dim=3072),   # vit.py:100-101
    "deit_small": dict(dim=384, depth=12, heads=6, mlp_dim=1536),   # vit.py:104-105
    "deit_tiny": dict(dim=192, depth=12, heads=3, mlp_dim=768),     # vit.py:108-109
}


def _cfg_for(name: str) -> ViTConfig:
    """Host-only config of a named DeiT (no GPU needed)."""
    return vit_config(**_NAMED[name])


def build_named(name: str, **kw) -> ViT:
    return ViT(**_NAMED[name], **kw)
