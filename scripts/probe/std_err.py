"""bf16 max-abs / min cosine of the STANDARD-ViT golden cases for whichever library EVT_LIB loads
(numerics A/B of kernel variants)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from edgevisiontransformer_amd.modeling.models import vit as vitmod  # noqa: E402
from tests.golden.make_golden_std import CASES, EPS, case  # noqa: E402

G = os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden")
for name in CASES:
    cfg, params, img = case(name)
    z = np.load(os.path.join(G, f"{name}.npz"))
    m = vitmod.StandardViT(dim=cfg.dim, depth=cfg.depth, heads=cfg.heads[0],
                           mlp_ratio=cfg.ffn[0] / cfg.dim, num_classes=cfg.num_classes,
                           layer_norm_eps=EPS, dtype="bf16", weights=params, device="cuda:0")
    out = m(torch.from_numpy(img).to("cuda:0")).cpu().numpy().astype(np.float64)
    ref = z["logits"]
    cos = ((out * ref).sum(1) / (np.linalg.norm(out, axis=1) * np.linalg.norm(ref, axis=1))).min()
    print(name, os.path.basename(os.environ.get("EVT_LIB", "product")), f"maxabs {np.abs(out - ref).max():.4f}",
          f"max|ref| {np.abs(ref).max():.3f} cos {cos:.6f}")
