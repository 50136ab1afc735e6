"""Device-side per-kernel timing of real forwards (evt_model_profile, include/evt.h).

The reference measures whole-model latency (`tools.py:82-116`, `test_keras_latency` `:170-213`)
and per-layer micro-models (`utils.py:322-406`); here every launch of a forward is bracketed by
HIP events on the model's stream, so the numbers are those of the kernels inside the model (not
of an isolated, back-to-back launch of one kernel, which runs hotter and slower)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def kernel_times(model, img: torch.Tensor, logits: torch.Tensor, forwards: int = 5) -> dict:
    """Run `forwards` profiled forwards of `model` (any of the ViT / T2T / Swin mirrors with a
    built handle and `forward_into`) and return {role: {"us_per_launch", "launches"}} averaged over
    them (roles: _lib.PROF_ROLES; roles with no launch are omitted)."""
    lib = _lib.load_library()
    model.forward_into(img, logits)  # builds the handle for this batch if needed
    h = ctypes.c_void_p(model._handle)
    n = len(_lib.PROF_ROLES)
    tot_us, tot_n = [0.0] * n, [0] * n
    _lib.check(lib.evt_model_profile(h, 1))
    try:
        for _ in range(forwards):
            model.forward_into(img, logits)
            us = (ctypes.c_float * n)()
            cnt = (ctypes.c_int * n)()
            _lib.check(lib.evt_model_profile_read(h, us, cnt))
            for r in range(n):
                tot_us[r] += us[r]
                tot_n[r] += cnt[r]
    finally:
        _lib.check(lib.evt_model_profile(h, 0))
    torch.cuda.synchronize(model.device)
    return {role: {"us_per_launch": tot_us[r] / tot_n[r], "launches": tot_n[r] // forwards}
            for r, role in enumerate(_lib.PROF_ROLES) if tot_n[r]}
