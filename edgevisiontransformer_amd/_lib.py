"""ctypes binding of libevt_hip.so (C ABI in include/evt.h).

There is deliberately no CPU or PyTorch fallback: if the HIP library is missing or the device is
not a gfx950 GPU, every call raises. torch is imported first so that the HIP runtime torch ships
(SONAME libamdhip64.so.7) is the one the library binds to: one runtime per process, and torch
device pointers / streams are valid handles for the library.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EVT_LIB", os.path.join(_HERE, "libevt_hip.so"))

EVT_OK = 0
EVT_EINVAL = -22
EVT_ENOMEM = -12
EVT_EHIP = -5
EVT_ENODEV = -19
DTYPE = {"f32": 0, "fp32": 0, "float32": 0, "bf16": 1, "bfloat16": 1, "mx8": 2}

# GEMM epilogue flags (include/evt.h EVT_EPI_*)
EPI_BIAS, EPI_GELU, EPI_RESID, EPI_POS, EPI_OUT_F32 = 1, 2, 4, 8, 16
EPI_LNIN, EPI_RESLN, EPI_STATS, EPI_GELU_ERF = 32, 64, 128, 256
EPI_OUT_MX8 = 512
# evt_model_profile roles (include/evt.h EVT_PROF_*)
PROF_ROLES = ("patchify", "patch_embed", "qkv", "attention", "out_proj", "fc1", "fc2", "head",
              "(unused)", "t2t_unfold", "t2t_kqv", "t2t_performer", "merge", "attn_sublayer",
              "mlp")
SWIN_MAX_STAGES = 8


class EvtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"evt error {code}: {msg}")
        self.code = code


class evt_vit_desc(ctypes.Structure):
    _fields_ = [("image_size", ctypes.c_int32), ("patch_size", ctypes.c_int32),
                ("in_chans", ctypes.c_int32), ("num_classes", ctypes.c_int32),
                ("dim", ctypes.c_int32), ("depth", ctypes.c_int32), ("mlp_dim", ctypes.c_int32),
                ("heads", ctypes.POINTER(ctypes.c_int32)),
                ("head_dim", ctypes.POINTER(ctypes.c_int32)),
                ("ffn", ctypes.POINTER(ctypes.c_int32)),
                ("dtype", ctypes.c_int32), ("max_batch", ctypes.c_int32),
                ("semantics", ctypes.c_int32), ("layer_norm_eps", ctypes.c_float)]


VIT_REFERENCE, VIT_STANDARD = 0, 1


class evt_dense_args(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_int32), ("A", ctypes.c_void_p), ("lda", ctypes.c_int64),
                ("Wp", ctypes.c_void_p), ("Kpad", ctypes.c_int32), ("Npad", ctypes.c_int32),
                ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64), ("M", ctypes.c_int32),
                ("N", ctypes.c_int32), ("bias", ctypes.c_void_p), ("resid", ctypes.c_void_p),
                ("ldr", ctypes.c_int64), ("pos", ctypes.c_void_p), ("ldp", ctypes.c_int64),
                ("P", ctypes.c_int32), ("colsum", ctypes.c_void_p), ("stats_in", ctypes.c_void_p),
                ("rstats", ctypes.c_void_p), ("rgamma", ctypes.c_void_p),
                ("rbeta", ctypes.c_void_p), ("stats_out", ctypes.c_void_p),
                ("ln_width", ctypes.c_int32), ("ln_eps", ctypes.c_float),
                ("stats_step", ctypes.c_int32)]


class evt_dense_mx8_args(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_int32), ("A", ctypes.c_void_p), ("lda", ctypes.c_int64),
                ("a_scales", ctypes.c_void_p), ("ld_as", ctypes.c_int64),
                ("Wq", ctypes.c_void_p), ("Kpad", ctypes.c_int32), ("Npad", ctypes.c_int32),
                ("w_scales", ctypes.c_void_p), ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64),
                ("c_scales", ctypes.c_void_p), ("ld_cs", ctypes.c_int64),
                ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("bias", ctypes.c_void_p),
                ("resid", ctypes.c_void_p), ("ldr", ctypes.c_int64),
                ("rstats", ctypes.c_void_p), ("rgamma", ctypes.c_void_p),
                ("rbeta", ctypes.c_void_p)]


class evt_t2t_desc(ctypes.Structure):
    _fields_ = [("image_size", ctypes.c_int32), ("in_chans", ctypes.c_int32),
                ("num_classes", ctypes.c_int32), ("dim", ctypes.c_int32),
                ("depth", ctypes.c_int32), ("heads", ctypes.c_int32),
                ("mlp_dim", ctypes.c_int32), ("token_size", ctypes.c_int32),
                ("dtype", ctypes.c_int32), ("max_batch", ctypes.c_int32)]


class evt_swin_desc(ctypes.Structure):
    _fields_ = [("image_size", ctypes.c_int32), ("patch_size", ctypes.c_int32),
                ("in_chans", ctypes.c_int32), ("num_classes", ctypes.c_int32),
                ("embed_dim", ctypes.c_int32), ("num_stages", ctypes.c_int32),
                ("depths", ctypes.c_int32 * SWIN_MAX_STAGES),
                ("num_heads", ctypes.c_int32 * SWIN_MAX_STAGES),
                ("window_size", ctypes.c_int32), ("mlp_ratio", ctypes.c_float),
                ("dtype", ctypes.c_int32), ("max_batch", ctypes.c_int32)]


# name -> (restype, argtypes); this is the full symbol list of include/evt.h
_P, _I, _I64, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
SIGNATURES = {
    "evt_init": (_I, [_I]),
    "evt_last_error": (ctypes.c_char_p, []),
    "evt_vit_num_weights": (_I, [ctypes.POINTER(evt_vit_desc)]),
    "evt_vit_create": (_I, [ctypes.POINTER(evt_vit_desc), ctypes.POINTER(_P), _I, _P,
                            ctypes.POINTER(_P)]),
    "evt_vit_forward": (_I, [_P, _P, _I, _P, _P]),
    "evt_query_workspace": (_I, [ctypes.POINTER(evt_vit_desc), _I, ctypes.POINTER(ctypes.c_size_t)]),
    "evt_model_destroy": (_I, [_P]),
    "evt_model_set_lanes": (_I, [_P, _I, _P]),
    "evt_model_lanes": (_I, [_P, ctypes.POINTER(_I)]),
    "evt_model_set_lane_streams": (_I, [_P, _I, ctypes.POINTER(_P)]),
    "evt_graph_capture": (_I, [_P, _P, _I, _P, _P]),
    "evt_graph_launch": (_I, [_P, _P]),
    "evt_set_gemm_variant": (_I, [_I]),
    "evt_model_qkv_layout": (_I, [_P, ctypes.POINTER(_I)]),
    "evt_model_profile": (_I, [_P, _I]),
    "evt_model_profile_read": (_I, [_P, _P, _P]),
    "evt_model_profile_work": (_I, [_P, _P, _P]),
    "evt_pack_weight": (_I, [_I, _P, _P, _I, _I, _P, _I, _I, _P]),
    "evt_ln_fold": (_I, [_I, _P, _I, _I, _P, _P, _P, _I, _I, _P, _P, _P]),
    "evt_dense": (_I, [_I, ctypes.POINTER(evt_dense_args), _P]),
    "evt_dense_splitk": (_I, [_I, ctypes.POINTER(evt_dense_args), _I, _P, _P]),
    "evt_attention": (_I, [_I, _P, _I64, _P, _I64, _I, _I, _I, _F, _P]),
    "evt_attention_hd": (_I, [_I, _P, _I64, _P, _I64, _I, _I, _I, _I, _F, _P]),
    "evt_layernorm": (_I, [_I, _P, _I64, _P, _I64, _P, _P, _I, _I, _F, _P]),
    "evt_patchify": (_I, [_I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P]),
    "evt_patchify_cm": (_I, [_I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P, _P]),
    "evt_t2t_num_weights": (_I, [ctypes.POINTER(evt_t2t_desc)]),
    "evt_t2t_create": (_I, [ctypes.POINTER(evt_t2t_desc), ctypes.POINTER(_P), _I, _P,
                            ctypes.POINTER(_P)]),
    "evt_t2t_forward": (_I, [_P, _P, _I, _P, _P]),
    "evt_t2t_query_workspace": (_I, [ctypes.POINTER(evt_t2t_desc), _I,
                                     ctypes.POINTER(ctypes.c_size_t)]),
    "evt_unfold": (_I, [_I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P]),
    "evt_performer": (_I, [_I, _P, _I64, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                           _I64, _P]),
    "evt_performer_scratch": (_I64, [_I, _I]),
    "evt_swin_num_weights": (_I, [ctypes.POINTER(evt_swin_desc)]),
    "evt_swin_create": (_I, [ctypes.POINTER(evt_swin_desc), ctypes.POINTER(_P), _I, _P,
                             ctypes.POINTER(_P)]),
    "evt_swin_forward": (_I, [_P, _P, _I, _P, _P]),
    "evt_swin_query_workspace": (_I, [ctypes.POINTER(evt_swin_desc), _I,
                                      ctypes.POINTER(ctypes.c_size_t)]),
    "evt_window_attention": (_I, [_I, _P, _I64, _P, _I64, _P, _I, _I, _I, _I, _I, _P]),
    "evt_patch_merge": (_I, [_I, _P, _I64, _I, _I, _I, _P, _P, _I, _P]),
    "evt_mx8_quantize": (_I, [_I, _P, _I64, _I, _I, _I, _P, _I64, _P, _I64, _P]),
    "evt_mx8_pack_weight": (_I, [_P, _P, _I, _I, _P, _I, _I, _P, _P]),
    "evt_dense_mx8": (_I, [ctypes.POINTER(evt_dense_mx8_args), _P]),
    "evt_mx8_layernorm": (_I, [_P, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P]),
    "evt_attention_mx8": (_I, [_P, _I64, _P, _I64, _P, _I64, _I, _I, _I, _F, _P]),
}

_lib = None
_lock = threading.Lock()
_initialized_devices = set()


def load_library() -> ctypes.CDLL:
    """Load (once) and type the library; raises if it is not built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not found: build it with `python -m edgevisiontransformer_amd.build`"
                    " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            # an EVT_LIB override (a lab build, or an older build for an A/B measurement) may lack
            # entry points added since: those stay unbound there; the in-tree library must export
            # every one (tests/test_capi.py)
            lenient = "EVT_LIB" in os.environ
            for name, (res, args) in SIGNATURES.items():
                if lenient and not hasattr(lib, name):
                    continue
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def last_error() -> str:
    return load_library().evt_last_error().decode(errors="replace")


def check(rc: int) -> None:
    if rc != EVT_OK:
        raise EvtError(rc, last_error())


def ensure_device(device_index: int) -> None:
    """evt_init once per device: requires a visible gfx950 GPU (fails loudly otherwise)."""
    if device_index in _initialized_devices:
        return
    if not torch.cuda.is_available():
        raise RuntimeError("edgevisiontransformer_amd needs a ROCm GPU (MI355X / gfx950); "
                           "torch.cuda.is_available() is False and there is no CPU fallback")
    lib = load_library()
    check(lib.evt_init(device_index))
    _initialized_devices.add(device_index)


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


# evt_model_set_lanes policy of the mirrors: two lanes from 128 images for T2T-ViT / Swin in bf16
# and for ViT in fp32. Measured round 6 (bench.py A/B on one box per call, profiles/
# r06_lanes_ab.txt): T2T-ViT-14 bs256 +3.1 %, Swin-T bs256 +0.5-3.3 %, DeiT-tiny fp32 bs256
# +19 %, logits bitwise equal; bf16 ViT stays one lane (DeiT-base bs512 / bs64 slower split).
LANES_MIN_BATCH = 128


def default_lanes(dtype: str, max_batch: int, vit: bool = False) -> int:
    """Lane count for a new handle; EVT_LANES=<k> overrides it (A/B runs)."""
    env = os.environ.get("EVT_LANES", "")
    if env:
        return int(env)
    if max_batch < LANES_MIN_BATCH:
        return 1
    want = DTYPE["f32"] if vit else DTYPE["bf16"]
    return 2 if DTYPE[dtype] == want else 1


def set_lanes(handle: int, lanes: int, device) -> list:
    """Give the handle `lanes` batch lanes on the streams the library creates, or with
    EVT_LANE_STREAMS=torch on streams of torch's pool (evt_model_set_lane_streams; measured equal,
    profiles/r06_lanes_probe.txt). Returns the torch streams (the model keeps them alive)."""
    if lanes <= 1:
        return []
    lib = load_library()
    check(lib.evt_model_set_lanes(ctypes.c_void_p(handle), lanes,
                                  ctypes.c_void_p(stream_ptr(device))))
    if os.environ.get("EVT_LANE_STREAMS", "") != "torch":
        return []
    streams = [torch.cuda.Stream(device) for _ in range(lanes)]
    ptrs = (ctypes.c_void_p * lanes)(*[s.cuda_stream for s in streams])
    check(lib.evt_model_set_lane_streams(ctypes.c_void_p(handle), lanes, ptrs))
    return streams
