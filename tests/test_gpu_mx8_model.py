"""End-to-end MXFP8 ViT (EVT_DTYPE_MX8: encoder Dense layers in OCP MX e4m3 on the block-scaled
MFMA, LayerNorm in the quantizer, bf16 elsewhere) against the fp64 goldens of the reference
model (tests/golden, produced from the reference's own torch_layers).

Tolerance (the accuracy of an 8-bit model, not a rounding check): per-row cosine >= 0.98 and
max |logits - golden| <= 0.25 * max |golden|. Measured on DeiT-tiny bs2: cosine 0.9901, max-abs
0.17 (13 % of max |golden|; the other fixtures 0.9956 / 0.9988 / 0.9930), about 15x the bf16
path's error, the ratio of the two formats' precision (2^-4 vs 2^-8 relative): no systematic
error on top of the e4m3 rounding. The MX8 path is
also checked to be batch-independent bit for bit and rejected for the STANDARD semantics."""
import os

import numpy as np
import pytest
import torch

from edgevisiontransformer_amd import _lib
from edgevisiontransformer_amd.modeling.models.vit import ViT
from tests.golden.make_golden import CASES
from tests.test_gpu_model import GOLDEN, _cos_rows, _model_for

pytestmark = pytest.mark.gpu

MX8_COS, MX8_REL = 0.98, 0.25


# EVT_DTYPE_MX8 is built for head size 64 and widths that are multiples of 64 (include/evt.h); the
# other head sizes run in bf16 / fp32 (tests/test_gpu_model.py)
MX8_CASES = [n for n in CASES if CASES[n][0]["dim"] % 64 == 0
             and CASES[n][0]["dim"] // CASES[n][0]["heads"] == 64]


@pytest.mark.parametrize("name", MX8_CASES)
def test_golden_mx8(gpu, name):
    m, img = _model_for(name, "mx8", gpu)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    out = m(torch.from_numpy(img).to(gpu))
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.float64)
    ref = z["logits"]
    assert np.all(np.isfinite(got))
    cos = _cos_rows(got, ref).min()
    err = np.abs(got - ref).max()
    print(f"{name}: mx8 min cosine {cos:.5f}, max-abs {err:.3e}, max|golden| {np.abs(ref).max():.3f}")
    assert cos >= MX8_COS, f"{name}: cosine {cos:.4f}"
    assert err <= MX8_REL * np.abs(ref).max(), f"{name}: max-abs {err:.3e}"


def test_mx8_batch_independent(gpu):
    m, img = _model_for(list(CASES)[0], "mx8", gpu)
    x = torch.from_numpy(img).to(gpu)
    full = m(x).cpu()
    one = m(x[1:2]).cpu()
    torch.cuda.synchronize()
    assert torch.equal(full[1:2], one)


def test_mx8_rejects_standard(gpu):
    from edgevisiontransformer_amd.modeling.models.vit import StandardViT
    with pytest.raises(_lib.EvtError):
        m = StandardViT(image_size=32, patch_size=16, num_classes=10, dim=64, depth=1, heads=1,
                        dtype="mx8", device=gpu)
        m(torch.zeros((1, 3, 32, 32), device=gpu))  # the handle is created on first use
