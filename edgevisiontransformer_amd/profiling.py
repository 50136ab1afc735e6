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
    built handle and `forward_into`) and return, per role with a launch (_lib.PROF_ROLES):
      us_per_launch  device time of one launch (HIP events), averaged over the forwards
      launches       launches per forward
      us_per_forward the role's device time per forward
      gflop, gbytes  the role's algorithmic work per forward (evt_model_profile_work: 2 x MACs of
                     its contractions; bytes its kernels must move at least)."""
    lib = _lib.load_library()
    model.forward_into(img, logits)  # builds the handle for this batch if needed
    h = ctypes.c_void_p(model._handle)
    n = len(_lib.PROF_ROLES)
    tot_us, tot_n = [0.0] * n, [0] * n
    gf, gb = (ctypes.c_double * n)(), (ctypes.c_double * n)()
    _lib.check(lib.evt_model_profile(h, 1))
    try:
        for _ in range(forwards):
            model.forward_into(img, logits)
            us = (ctypes.c_float * n)()
            cnt = (ctypes.c_int * n)()
            _lib.check(lib.evt_model_profile_read(h, us, cnt))
            _lib.check(lib.evt_model_profile_work(h, gf, gb))
            for r in range(n):
                tot_us[r] += us[r]
                tot_n[r] += cnt[r]
    finally:
        _lib.check(lib.evt_model_profile(h, 0))
    torch.cuda.synchronize(model.device)
    return {role: {"us_per_launch": tot_us[r] / tot_n[r], "launches": tot_n[r] // forwards,
                   "us_per_forward": tot_us[r] / forwards, "gflop": gf[r], "gbytes": gb[r]}
            for r, role in enumerate(_lib.PROF_ROLES) if tot_n[r]}


def roofline_table(kt: dict, peak_tflops: float, peak_gbps: float) -> dict:
    """Per role: achieved TFLOP/s and GB/s of its algorithmic work over its device time, as
    fractions of the MFMA and HBM peaks (both reported for every role: the bound is whichever
    fraction is higher)."""
    out = {}
    for role, v in kt.items():
        t = v["us_per_forward"] * 1e-6
        tf = v["gflop"] / t / 1e3 if t > 0 else 0.0
        gbs = v["gbytes"] / t if t > 0 else 0.0
        out[role] = {"us": round(v["us_per_forward"], 1), "launches": v["launches"],
                     "us_per_launch": round(v["us_per_launch"], 1),
                     "tflops": round(tf, 1), "mfma_frac": round(tf / peak_tflops, 4),
                     "gbps": round(gbs, 1), "hbm_frac": round(gbs / peak_gbps, 4)}
    return out
