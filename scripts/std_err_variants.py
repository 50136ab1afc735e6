"""bf16 max-abs error of the standard-semantics goldens (tests/golden/std_*.npz) per GEMM kernel
selection (evt_set_gemm_variant: 0 automatic, 31 automatic without the 128 x 384 tiles, 30 those
tiles wherever they apply, 1 128 x 128, 9 256 x 256 persistent)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from edgevisiontransformer_amd import _lib  # noqa: E402
from edgevisiontransformer_amd.modeling.models import vit as vitmod  # noqa: E402
from tests.test_std_vit import CASES, EPS, GOLDEN, case  # noqa: E402

dev = torch.device("cuda", 0)
for name in CASES:
    cfg, params, img = case(name)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    res = []
    for v in (0, 31, 30, 1, 9):
        _lib.check(_lib.load_library().evt_set_gemm_variant(v))
        m = vitmod.StandardViT(dim=cfg.dim, depth=cfg.depth, heads=cfg.heads[0],
                               mlp_ratio=cfg.ffn[0] / cfg.dim, num_classes=cfg.num_classes,
                               layer_norm_eps=EPS, dtype="bf16", weights=params, device=dev)
        out = m(torch.from_numpy(img).to(dev)).cpu().numpy().astype(np.float64)
        res.append(f"v{v} {np.abs(out - z['logits']).max():.4f}")
        m.close()
    _lib.check(_lib.load_library().evt_set_gemm_variant(0))
    print(name, cfg.dim, cfg.depth, " ".join(res), flush=True)
