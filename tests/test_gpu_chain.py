"""Chained GEMM launches (EVT_FUSE_GEMM_CHAIN, gemm.hip gemm_chain_kernel): each DeiT-base layer's
out-proj -> FC1 in one persistent launch, FC1's M panels handed over per panel inside the launch
(write-through stores, per-panel counters, agent-scope acquire; counters self-cleaning). The chained forward computes every tile with the same code and reduction order as the
separate launches, so the logits must be BITWISE equal to the unchained forward (a stale read of
a handed-off panel shows as a difference), on every one of several repeated forwards. Reference
ops: `attention.py:35`, `ffn.py:8-9`, `residual.py:9`."""
import pytest
import torch

from edgevisiontransformer_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [111, 128, 512])
def test_chain_bitwise_equals_separate_launches(gpu, batch):
    from edgevisiontransformer_amd.modeling.models.vit import build_named
    m = build_named("deit_base", dtype="bf16", seed=3, max_batch=batch)
    g = torch.Generator(device=gpu).manual_seed(batch)
    img = torch.randn((batch, 3, 224, 224), generator=g, device=gpu)
    ref = torch.empty((batch, 1000), device=gpu)
    m.set_fusion(0)
    m.forward_into(img, ref)
    torch.cuda.synchronize()
    m.set_fusion(_lib.FUSE_GEMM_CHAIN)
    out = torch.empty_like(ref)
    bad = []
    for r in range(6):
        out.fill_(float("nan"))
        m.forward_into(img, out)
        torch.cuda.synchronize()
        if not torch.equal(out, ref):
            bad.append((r, int((out != ref).sum())))
    assert not bad, f"chained forwards differing from the separate launches (run, elements): {bad}"
    assert torch.isfinite(ref).all()
