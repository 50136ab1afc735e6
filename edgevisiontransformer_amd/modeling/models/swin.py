"""MI355X Swin Transformer: the model the reference benchmarks through `get_swin`.

The reference does not implement Swin itself: `utils.py:14-47` (`get_swin(config_file_name,
swin_root_path)`) imports `SwinTransformer` from an external microsoft/Swin-Transformer checkout
and builds it from `configs/{config_file_name}.yaml`; `tools.py:272-282` benchmarks
`swin_tiny_patch4_window7_224` on NCHW [B, 3, 224, 224]. This module keeps that interface:

    model = get_swin("swin_tiny_patch4_window7_224", dtype="bf16")  # reference utils.py:14
    logits = model(img)                                             # SwinTransformer.forward

`SwinTransformer(...)` takes the constructor keywords get_swin passes (utils.py:28-43). The yaml
files are not available offline, so the three published configs are built in
(`edgevisiontransformer_amd.weights.SWIN_VARIANTS`); `swin_root_path` is accepted and ignored.
The forward is one call into libevt_hip.so (`evt_swin_forward`, include/evt.h). Deliberate
differences: `seed=` / `weights=` select the parameters (Keras [in, out] dict, or
`params_from_state_dict` of a microsoft checkpoint), `dtype` selects bf16 MFMA or exact fp32;
inference only (dropout / drop-path are identity, as in eval mode). Unsupported options raise
ValueError: window_size != 7, head size != 32, ape=True, patch_norm=False, qkv_bias=False,
qk_scale != None, stage resolutions that are not multiples of 7.
"""
from __future__ import annotations

import ctypes
import re
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from ... import _lib
from ...weights import SwinConfig, make_swin_params, swin_config, swin_param_shapes
from .vit import _capture_graph, _replay_graph, _to_device_image


class SwinTransformer:
    """Swin Transformer forward on MI355X (microsoft `SwinTransformer`, built by reference
    `utils.py:28-43`)."""

    def __init__(self, img_size=224, patch_size=4, in_chans=3, num_classes=1000, embed_dim=96,
                 depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24), window_size=7, mlp_ratio=4.,
                 qkv_bias=True, qk_scale=None, drop_rate=0., drop_path_rate=0.1, ape=False,
                 patch_norm=True, use_checkpoint=False, *, dtype: str = "bf16", seed: int = 0,
                 weights: Optional[Dict[str, np.ndarray]] = None, device=None,
                 max_batch: int = 0, lanes: Optional[int] = None):
        if window_size != 7:
            raise ValueError("window_size must be 7 in this build")
        if ape or not patch_norm or not qkv_bias or qk_scale is not None:
            raise ValueError("this build supports ape=False, patch_norm=True, qkv_bias=True, "
                             "qk_scale=None (the published Swin configs)")
        if len(depths) != len(num_heads) or not 1 <= len(depths) <= _lib.SWIN_MAX_STAGES:
            raise ValueError("depths and num_heads must have the same length (1..8)")
        self.cfg: SwinConfig = SwinConfig(image_size=img_size, patch_size=patch_size,
                                          in_chans=in_chans, num_classes=num_classes,
                                          embed_dim=embed_dim, depths=tuple(depths),
                                          num_heads=tuple(num_heads), window_size=window_size,
                                          mlp_ratio=float(mlp_ratio))
        for i in range(self.cfg.num_stages):
            if self.cfg.dim(i) % num_heads[i] or self.cfg.dim(i) // num_heads[i] != 32:
                raise ValueError(f"stage {i}: head size {self.cfg.dim(i)}/{num_heads[i]} must be 32")
            if self.cfg.res(i) % 7 or self.cfg.res(i) < 7:
                raise ValueError(f"stage {i}: resolution {self.cfg.res(i)} is not a multiple of 7")
        self.num_classes = num_classes
        self.num_features = self.cfg.num_features
        if dtype not in _lib.DTYPE:
            raise ValueError(f"dtype must be one of {sorted(_lib.DTYPE)}")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        _lib.ensure_device(self.device.index or 0)
        params = weights if weights is not None else make_swin_params(self.cfg, seed=seed)
        self._weights: List[torch.Tensor] = []
        for name, shape in swin_param_shapes(self.cfg):
            a = np.asarray(params[name], dtype=np.float32)
            if tuple(a.shape) != tuple(shape):
                raise ValueError(f"weight {name}: shape {a.shape}, expected {shape}")
            self._weights.append(torch.from_numpy(np.ascontiguousarray(a)).to(self.device))
        self._handle: Optional[int] = None
        self._max_batch = 0
        # batch lanes (evt_model_set_lanes): None = _lib.default_lanes
        self._lanes = lanes
        if max_batch:
            self._build(max_batch)

    # -- C ABI plumbing ---------------------------------------------------------------------
    def _desc(self, max_batch: int) -> _lib.evt_swin_desc:
        c = self.cfg
        d = _lib.evt_swin_desc()
        d.image_size, d.patch_size, d.in_chans = c.image_size, c.patch_size, c.in_chans
        d.num_classes, d.embed_dim, d.num_stages = c.num_classes, c.embed_dim, c.num_stages
        for i in range(c.num_stages):
            d.depths[i] = c.depths[i]
            d.num_heads[i] = c.num_heads[i]
        d.window_size, d.mlp_ratio = c.window_size, c.mlp_ratio
        d.dtype, d.max_batch = _lib.DTYPE[self.dtype], max_batch
        return d

    def _build(self, max_batch: int) -> None:
        lib = _lib.load_library()
        self.close()
        self._graph_io = None
        desc = self._desc(max_batch)
        n = lib.evt_swin_num_weights(ctypes.byref(desc))
        if n != len(self._weights):
            raise RuntimeError(f"library expects {n} weights, mirror has {len(self._weights)}")
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in self._weights])
        out = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(lib.evt_swin_create(ctypes.byref(desc), ptrs, n,
                                           ctypes.c_void_p(_lib.stream_ptr(self.device)),
                                           ctypes.byref(out)))
        self._handle = out.value
        self._max_batch = max_batch
        with torch.cuda.device(self.device):
            self._lane_streams = _lib.set_lanes(
                self._handle, self._lanes if self._lanes is not None
                else _lib.default_lanes(self.dtype, max_batch), self.device)

    def lanes(self) -> int:
        """Batch lanes of the handle (include/evt.h evt_model_set_lanes; 1 = none)."""
        out = ctypes.c_int()
        _lib.check(_lib.load_library().evt_model_lanes(ctypes.c_void_p(self._handle),
                                                       ctypes.byref(out)))
        return out.value

    def workspace_bytes(self, batch: int) -> int:
        out = ctypes.c_size_t()
        _lib.check(_lib.load_library().evt_swin_query_workspace(
            ctypes.byref(self._desc(batch)), batch, ctypes.byref(out)))
        return out.value

    def close(self) -> None:
        if getattr(self, "_handle", None):
            _lib.load_library().evt_model_destroy(ctypes.c_void_p(self._handle))
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- forward ------------------------------------------------------------------------------
    def forward_into(self, img: torch.Tensor, logits: torch.Tensor) -> torch.Tensor:
        """Enqueue the forward of a device-resident fp32 NCHW batch into `logits`."""
        b = img.shape[0]
        if b > self._max_batch:
            self._build(b)
        _lib.check(_lib.load_library().evt_swin_forward(
            ctypes.c_void_p(self._handle), ctypes.c_void_p(img.data_ptr()), b,
            ctypes.c_void_p(logits.data_ptr()), ctypes.c_void_p(_lib.stream_ptr(self.device))))
        return logits

    def capture_graph(self, img: torch.Tensor, logits: torch.Tensor) -> None:
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
        return logits.cpu().numpy() if was_numpy else logits

    forward = __call__


_CONFIG_RE = re.compile(r"swin_(tiny|small|base)_patch(\d+)_window(\d+)_(\d+)$")


def swin_config_from_name(config_file_name: str, num_classes: int = 1000) -> SwinConfig:
    """The SwinConfig of a microsoft config name (configs/swin_{tiny,small,base}_patch4_window7_224)."""
    m = _CONFIG_RE.match(config_file_name)
    if not m:
        raise NotImplementedError(f"Unkown model: {config_file_name}")  # utils.py:45 wording
    variant, patch, window, size = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4))
    return swin_config(variant, patch_size=patch, window_size=window, image_size=size,
                       num_classes=num_classes)


def get_swin(config_file_name: str = "swin_tiny_patch4_window7_224", swin_root_path: str = "",
             **kw) -> SwinTransformer:
    """Reference `utils.py:14-47` (`get_swin`), with the published configs built in."""
    c = swin_config_from_name(config_file_name, kw.pop("num_classes", 1000))
    return SwinTransformer(img_size=c.image_size, patch_size=c.patch_size, in_chans=c.in_chans,
                           num_classes=c.num_classes, embed_dim=c.embed_dim, depths=c.depths,
                           num_heads=c.num_heads, window_size=c.window_size,
                           mlp_ratio=c.mlp_ratio, **kw)


def params_from_state_dict(sd: Dict[str, np.ndarray], cfg: SwinConfig) -> Dict[str, np.ndarray]:
    """Map a microsoft Swin-Transformer state dict (`model.state_dict()` / checkpoint['model'],
    torch [out, in] Linear weights) onto this module's Keras-layout parameter names."""
    a = lambda k: np.asarray(sd[k], dtype=np.float32)  # noqa: E731
    e = cfg.embed_dim
    p = {"patch_w": a("patch_embed.proj.weight").reshape(e, -1).T,
         "patch_b": a("patch_embed.proj.bias"),
         "pnorm_g": a("patch_embed.norm.weight"), "pnorm_b": a("patch_embed.norm.bias"),
         "norm_g": a("norm.weight"), "norm_b": a("norm.bias"),
         "head_w": a("head.weight").T, "head_b": a("head.bias")}
    for i in range(cfg.num_stages):
        if i > 0:  # microsoft attaches the merge of stage i to layers[i-1].downsample
            src = f"layers.{i - 1}.downsample."
            p[f"s{i}.merge_g"] = a(src + "norm.weight")
            p[f"s{i}.merge_b"] = a(src + "norm.bias")
            p[f"s{i}.merge_w"] = a(src + "reduction.weight").T
        for j in range(cfg.depths[i]):
            src, dst = f"layers.{i}.blocks.{j}.", f"s{i}.b{j}."
            p[dst + "ln1_g"], p[dst + "ln1_b"] = a(src + "norm1.weight"), a(src + "norm1.bias")
            p[dst + "qkv_w"], p[dst + "qkv_b"] = a(src + "attn.qkv.weight").T, a(src + "attn.qkv.bias")
            p[dst + "rpb"] = a(src + "attn.relative_position_bias_table")
            p[dst + "proj_w"], p[dst + "proj_b"] = a(src + "attn.proj.weight").T, a(src + "attn.proj.bias")
            p[dst + "ln2_g"], p[dst + "ln2_b"] = a(src + "norm2.weight"), a(src + "norm2.bias")
            p[dst + "fc1_w"], p[dst + "fc1_b"] = a(src + "mlp.fc1.weight").T, a(src + "mlp.fc1.bias")
            p[dst + "fc2_w"], p[dst + "fc2_b"] = a(src + "mlp.fc2.weight").T, a(src + "mlp.fc2.bias")
    return {k: np.ascontiguousarray(v) for k, v in p.items()}


def build_named(name: str, **kw) -> SwinTransformer:
    """'swin_tiny' | 'swin_small' | 'swin_base' (patch 4, window 7, 224)."""
    return get_swin(f"{name}_patch4_window7_224", **kw)
