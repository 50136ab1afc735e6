"""MI355X mirror of the reference `modeling/models/t2t_vit.py` (T2T_ViT, get_t2t_vit_*).

Same public names and constructor keywords as the reference; the Keras graph is replaced by one
call into libevt_hip.so (`evt_t2t_forward`, include/evt.h): soft splits (unfold), the two
TokenPerformers, the project Dense, the shared encoder and the LayerNorm-folded classifier run
as gfx950 kernels on the caller's stream.

    model = get_t2t_vit_14(dtype="bf16")   # reference: get_t2t_vit_14()    t2t_vit.py:147-148
    logits = model(img)                    # reference: T2T_ViT.call       t2t_vit.py:132-135

Input is channel-last like the reference (tf_Unfold is built with channel_last=True,
t2t_vit.py:50-52): fp32 NHWC [B, S, S, 3]. Deliberate differences, as for ViT: `seed=` /
`weights=` select the parameters (the reference random-initialises, t2t_vit.py:116-118), and
`dtype` selects the bf16 MFMA path or the exact fp32 path. Unsupported reference options fail
loudly: tokens_type other than 'performer' raises NotImplementedError (t2t_vit.py:58-59),
token_size must be 64, the head size hidden_size // num_heads at most 128.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Union

import numpy as np
import torch

from ... import _lib
from ...weights import T2TConfig, make_t2t_params, t2t_config, t2t_param_shapes
from .vit import _capture_graph, _replay_graph, _to_device_image


class T2T_ViT:
    """Tokens-to-Token ViT forward on MI355X (reference `T2T_ViT`, t2t_vit.py:91-135)."""

    def __init__(self, image_size=224, tokens_type="performer", in_channels=3, num_classes=1000,
                 hidden_size=768, depth=12, num_heads=12, mlp_ratio=4., token_size=64,
                 qkv_bias=False, qk_scale=None, drop_rate=0., attn_drop_rate=0.,
                 drop_path_rate=0., *, dtype: str = "bf16", seed: int = 0,
                 weights: Optional[Dict[str, np.ndarray]] = None, device=None,
                 max_batch: int = 0, lanes: Optional[int] = None):
        if tokens_type != "performer":  # t2t_vit.py:58-59
            raise NotImplementedError(
                "T2T_module with token_type other than performer is not supported")
        if hidden_size % num_heads != 0:  # Attention (attention.py:8-9)
            raise ValueError(f"hidden_size {hidden_size} must be a multiple of num_heads {num_heads}.")
        # qkv_bias / qk_scale / drop rates are accepted and unused, as in the reference (:92-94)
        self.cfg: T2TConfig = t2t_config(hidden_size, depth, num_heads, mlp_ratio,
                                         image_size=image_size, num_classes=num_classes,
                                         token_size=token_size, in_channels=in_channels)
        self.num_classes = num_classes
        self.num_features = self.hidden_size = hidden_size
        if dtype not in _lib.DTYPE:
            raise ValueError(f"dtype must be one of {sorted(_lib.DTYPE)}")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        _lib.ensure_device(self.device.index or 0)
        params = weights if weights is not None else make_t2t_params(self.cfg, seed=seed)
        self._weights: List[torch.Tensor] = []
        for name, shape in t2t_param_shapes(self.cfg):
            a = np.asarray(params[name], dtype=np.float32)
            if a.size != int(np.prod(shape)):
                raise ValueError(f"weight {name}: shape {a.shape}, expected {shape}")
            self._weights.append(torch.from_numpy(np.ascontiguousarray(a.reshape(shape)))
                                 .to(self.device))
        self._handle: Optional[int] = None
        self._max_batch = 0
        # batch lanes (evt_model_set_lanes): None = _lib.default_lanes
        self._lanes = lanes
        if max_batch:
            self._build(max_batch)

    def _desc(self, max_batch: int):
        c = self.cfg
        return _lib.evt_t2t_desc(c.image_size, c.in_chans, c.num_classes, c.dim, c.depth, c.heads,
                                 c.mlp_dim, c.token_size, _lib.DTYPE[self.dtype], max_batch)

    def _build(self, max_batch: int) -> None:
        lib = _lib.load_library()
        self.close()
        self._graph_io = None
        desc = self._desc(max_batch)
        n = lib.evt_t2t_num_weights(ctypes.byref(desc))
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in self._weights])
        out = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            stream = _lib.stream_ptr(self.device)
            _lib.check(lib.evt_t2t_create(ctypes.byref(desc), ptrs, n, ctypes.c_void_p(stream),
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
        lib = _lib.load_library()
        out = ctypes.c_size_t()
        _lib.check(lib.evt_t2t_query_workspace(ctypes.byref(self._desc(batch)), batch,
                                               ctypes.byref(out)))
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

    def forward_into(self, img: torch.Tensor, logits: torch.Tensor) -> torch.Tensor:
        """Enqueue the forward of a device-resident fp32 NHWC batch into `logits`."""
        b = img.shape[0]
        if b > self._max_batch:
            self._build(b)
        lib = _lib.load_library()
        _lib.check(lib.evt_t2t_forward(ctypes.c_void_p(self._handle), ctypes.c_void_p(img.data_ptr()),
                                       b, ctypes.c_void_p(logits.data_ptr()),
                                       ctypes.c_void_p(_lib.stream_ptr(self.device))))
        return logits

    def capture_graph(self, img: torch.Tensor, logits: torch.Tensor) -> None:
        """HIP graph of one forward of (img, logits); see ViT.capture_graph."""
        _capture_graph(self, img, logits)

    def replay_graph(self) -> None:
        _replay_graph(self)

    def __call__(self, img: Union[torch.Tensor, np.ndarray]):
        x, was_numpy = _to_device_image(img, self.device)
        c = self.cfg
        if x.dim() != 4 or tuple(x.shape[1:]) != (c.image_size, c.image_size, c.in_chans):
            raise ValueError(f"expected NHWC [B, {c.image_size}, {c.image_size}, {c.in_chans}], "
                             f"got {tuple(x.shape)}")
        logits = torch.empty((x.shape[0], c.num_classes), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            self.forward_into(x, logits)
        return logits.cpu().numpy() if was_numpy else logits

    call = __call__


def get_t2t_vit_7(**kw) -> T2T_ViT:
    return T2T_ViT(hidden_size=256, depth=7, num_heads=4, mlp_ratio=2, **kw)


def get_t2t_vit_10(**kw) -> T2T_ViT:
    return T2T_ViT(hidden_size=256, depth=10, num_heads=4, mlp_ratio=2, **kw)


def get_t2t_vit_12(**kw) -> T2T_ViT:
    return T2T_ViT(hidden_size=256, depth=12, num_heads=4, mlp_ratio=2, **kw)


def get_t2t_vit_14(**kw) -> T2T_ViT:
    return T2T_ViT(hidden_size=384, depth=14, num_heads=6, mlp_ratio=3, **kw)


_NAMED = {  # t2t_vit.py:138-148
    "t2t_vit_7": (256, 7, 4, 2),
    "t2t_vit_10": (256, 10, 4, 2),
    "t2t_vit_12": (256, 12, 4, 2),
    "t2t_vit_14": (384, 14, 6, 3),
}


def t2t_cfg_for(name: str) -> T2TConfig:
    """Host-only config of a named T2T-ViT (no GPU needed)."""
    return t2t_config(*_NAMED[name])


def build_named(name: str, **kw) -> T2T_ViT:
    h, d, nh, r = _NAMED[name]
    return T2T_ViT(hidden_size=h, depth=d, num_heads=nh, mlp_ratio=r, **kw)
