"""evt_model_profile: per-role HIP-event timing of real forwards (the measurement bench.py's
roofline uses). Launch counts follow the model structure; times are positive and add up to no
more than the wall time of the profiled forwards."""
import time

import pytest
import torch

from edgevisiontransformer_amd import _lib
from edgevisiontransformer_amd.profiling import kernel_times

pytestmark = pytest.mark.gpu


def test_profile_roles_deit_tiny(gpu):
    from edgevisiontransformer_amd.modeling.models.vit import build_named
    m = build_named("deit_tiny", dtype="bf16", seed=0, max_batch=8)
    img = torch.randn((8, 3, 224, 224), device=gpu)
    logits = torch.empty((8, 1000), device=gpu)
    kernel_times(m, img, logits, forwards=1)  # warm-up (event pool)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kt = kernel_times(m, img, logits, forwards=3)
    wall_us = (time.perf_counter() - t0) / 3 * 1e6  # per profiled forward (+ one extra)
    expect = {"patchify": 1, "patch_embed": 1, "qkv": 12, "attention": 12, "out_proj": 12,
              "fc1": 12, "fc2": 12, "head": 1}
    assert {k: v["launches"] for k, v in kt.items()} == expect
    assert all(v["us_per_launch"] > 0 for v in kt.values())
    # the bracketed intervals are disjoint and in stream order: their sum fits in the wall time
    total = sum(v["us_per_launch"] * v["launches"] for v in kt.values())
    assert total <= wall_us, (total, wall_us)


def test_profile_off_leaves_forward_unchanged(gpu):
    from edgevisiontransformer_amd.modeling.models.vit import build_named
    m = build_named("deit_tiny", dtype="bf16", seed=0, max_batch=2)
    img = torch.randn((2, 3, 224, 224), device=gpu)
    a, b = torch.empty((2, 1000), device=gpu), torch.empty((2, 1000), device=gpu)
    m.forward_into(img, a)
    kernel_times(m, img, b, forwards=1)
    m.forward_into(img, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_profile_work_matches_flop_count(gpu):
    """evt_model_profile_work: the per-role GFLOPs of a forward add up to the model's matmul FLOP
    count (weights.py gflop_per_image, cross-checked against the reference's flops_calculation.py
    in SURVEY.md 8d), and every role moves a positive number of bytes."""
    from edgevisiontransformer_amd.modeling.models.vit import build_named
    m = build_named("deit_base", dtype="bf16", seed=0, max_batch=4)
    img = torch.randn((4, 3, 224, 224), device=gpu)
    logits = torch.empty((4, 1000), device=gpu)
    kt = kernel_times(m, img, logits, forwards=1)
    total = sum(v["gflop"] for v in kt.values())
    assert abs(total - 4 * m.cfg.gflop_per_image()) <= 1e-3 * total, (total, m.cfg.gflop_per_image())
    assert all(v["gbytes"] > 0 for v in kt.values())
