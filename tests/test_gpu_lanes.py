"""Batch lanes of the model handles (include/evt.h evt_model_set_lanes): the batch is
split into contiguous parts run by child handles (the parent's weights, their own workspaces) on
their own HIP streams, forked from and joined to the caller's stream by events. The reference has
no cross-image op (t2t_vit.py:120-135, the Swin forward), so a lane split may change rows only
through a different kernel selection for the smaller part: at the BASELINE batch (256, two lanes
of 128) every part takes the whole batch's kernels and the logits are bitwise those of one lane.
Checked as well: odd batches and 3 / 4 lanes (within the bf16 gate), batches below the lane count
and profiled forwards (one lane: bitwise), a HIP-graph capture of a laned forward (bitwise), and
the argument checks. Cases: the default-laned configs (T2T-ViT-14 and Swin-T bf16, DeiT-tiny
fp32 at 256 images)."""
import ctypes

import pytest
import torch

from edgevisiontransformer_amd import _lib
from edgevisiontransformer_amd.modeling.models import swin, t2t_vit, vit
from edgevisiontransformer_amd.weights import make_images

pytestmark = pytest.mark.gpu
CASES = [("t2t_vit_14", t2t_vit, "NHWC", "bf16"), ("swin_tiny", swin, "NCHW", "bf16"),
         ("deit_tiny", vit, "NCHW", "f32")]


def _img(n, layout, gpu, seed=41):
    return torch.from_numpy(make_images(n, seed=seed, layout=layout)).to(gpu)


@pytest.mark.parametrize("name,mod,layout,dtype", CASES)
def test_lanes_bitwise_at_benchmark_batch(gpu, name, mod, layout, dtype):
    img = _img(256, layout, gpu)
    m2 = mod.build_named(name, dtype=dtype, seed=0, max_batch=256)  # default policy: 2 lanes
    m1 = mod.build_named(name, dtype=dtype, seed=0, max_batch=256, lanes=1)
    assert m2.lanes() == 2 and m1.lanes() == 1
    a, b = m2(img), m1(img)
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    # a batch below the lane count runs on the parent handle: the one-lane kernels, bitwise
    assert torch.equal(m2(img[:1].contiguous()), m1(img[:1].contiguous()))
    # profiled forwards run as one lane (the per-role events belong to the parent's stream)
    lib = _lib.load_library()
    _lib.check(lib.evt_model_profile(ctypes.c_void_p(m2._handle), 1))
    try:
        p = m2(img)
        torch.cuda.synchronize()
    finally:
        _lib.check(lib.evt_model_profile(ctypes.c_void_p(m2._handle), 0))
    assert torch.equal(p, b)
    # a HIP graph of a laned forward: the lanes as parallel branches of one graph
    logits = torch.empty_like(a)
    m2.capture_graph(img, logits)
    m2.replay_graph()
    torch.cuda.synchronize()
    assert torch.equal(logits, a)


@pytest.mark.parametrize("name,mod,layout,dtype", CASES)
@pytest.mark.parametrize("lanes,batch", [(2, 37), (3, 50), (4, 9)])
def test_lanes_odd_splits(gpu, name, mod, layout, dtype, lanes, batch):
    img = _img(batch, layout, gpu, seed=42)
    mk = mod.build_named(name, dtype=dtype, seed=0, max_batch=batch, lanes=lanes)
    m1 = mod.build_named(name, dtype=dtype, seed=0, max_batch=batch, lanes=1)
    assert mk.lanes() == lanes
    a, b = mk(img), m1(img)
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    err = float((a - b).abs().max())
    print(f"{name} lanes {lanes} batch {batch}: max |laned - one lane| = {err:.3e}")
    assert err <= 3e-2
    # every row equals its own part's forward on a one-lane handle bitwise
    lo = 0
    for i in range(lanes):
        hi = batch * (i + 1) // lanes
        if hi > lo:
            assert torch.equal(a[lo:hi], m1(img[lo:hi].contiguous()))
        lo = hi


def test_lanes_errors(gpu):
    lib = _lib.load_library()
    m = vit.build_named("deit_tiny", dtype="bf16", seed=0, max_batch=4)
    assert m.lanes() == 1  # bf16 ViT: one lane by default
    s = ctypes.c_void_p(_lib.stream_ptr(gpu))
    _lib.check(lib.evt_model_set_lanes(ctypes.c_void_p(m._handle), 2, s))
    assert m.lanes() == 2
    t = t2t_vit.build_named("t2t_vit_7", dtype="bf16", seed=0, max_batch=8, lanes=1)
    assert lib.evt_model_set_lanes(ctypes.c_void_p(t._handle), 5, s) == _lib.EVT_EINVAL
    assert lib.evt_model_set_lanes(ctypes.c_void_p(t._handle), 0, s) == _lib.EVT_EINVAL
    _lib.check(lib.evt_model_set_lanes(ctypes.c_void_p(t._handle), 2, s))
    assert t.lanes() == 2
    one = (ctypes.c_void_p * 1)(s.value)
    assert lib.evt_model_set_lane_streams(ctypes.c_void_p(t._handle), 1, one) == _lib.EVT_EINVAL
    streams = [torch.cuda.Stream(gpu) for _ in range(2)]
    two = (ctypes.c_void_p * 2)(*[x.cuda_stream for x in streams])
    _lib.check(lib.evt_model_set_lane_streams(ctypes.c_void_p(t._handle), 2, two))
    _lib.check(lib.evt_model_set_lanes(ctypes.c_void_p(t._handle), 1, s))
    assert t.lanes() == 1
