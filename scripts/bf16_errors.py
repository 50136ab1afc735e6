"""Print the bf16 path's max-abs error and min per-row cosine against every model golden fixture
(the numbers behind the tests' bf16 gate, SURVEY.md 8c: <= 3e-2, >= 0.9995)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from edgevisiontransformer_amd.modeling.models.swin import SwinTransformer  # noqa: E402
from edgevisiontransformer_amd.modeling.models.t2t_vit import T2T_ViT  # noqa: E402
from edgevisiontransformer_amd.modeling.models.vit import ViT, ViT_Pruned  # noqa: E402
from edgevisiontransformer_amd.weights import (make_images, make_t2t_params, make_vit_params,  # noqa: E402
                                               t2t_config)
from tests.golden.make_golden import CASES, T2T_CASES, case_config  # noqa: E402
from tests.test_swin_oracle import golden_case  # noqa: E402

G = os.path.join(REPO, "tests", "golden")
dev = torch.device("cuda", 0)


def report(name, out, gold):
    out, gold = np.asarray(out, np.float64), np.asarray(gold, np.float64)
    err = np.abs(out - gold).max()
    cos = ((out * gold).sum(1) / np.linalg.norm(out, axis=1) / np.linalg.norm(gold, axis=1)).min()
    print(f"{name:40s} bf16 max-abs {err:.3e}  min cos {cos:.6f}  max|golden| {np.abs(gold).max():.3f}",
          flush=True)


for name, (kw, enc, batch, pseed, iseed) in CASES.items():
    cfg = case_config(name)
    params = make_vit_params(cfg, seed=pseed)
    common = dict(image_size=cfg.image_size, patch_size=cfg.patch_size, num_classes=cfg.num_classes,
                  dim=kw["dim"], depth=kw["depth"], heads=kw["heads"], mlp_dim=kw["mlp_dim"],
                  dtype="bf16", weights=params, device=dev)
    m = ViT_Pruned(head_size=64, prune_encoding=enc, **common) if enc else ViT(**common)
    img = make_images(batch, seed=iseed, image_size=cfg.image_size)
    report(name, m(img), np.load(os.path.join(G, f"{name}.npz"))["logits"])

for name, (args, batch, pseed, iseed) in T2T_CASES.items():
    h, depth, heads, ratio = args
    params = make_t2t_params(t2t_config(*args), seed=pseed)
    m = T2T_ViT(hidden_size=h, depth=depth, num_heads=heads, mlp_ratio=ratio, dtype="bf16",
                weights=params, device=dev)
    img = make_images(batch, seed=iseed, layout="NHWC")
    report(name, m(img), np.load(os.path.join(G, f"{name}.npz"))["logits"])

for name in ("swin_micro_b2", "swin_tiny_b1", "swin_base_micro_b3"):
    z, cfg, params, img = golden_case(name)
    m = SwinTransformer(img_size=cfg.image_size, patch_size=cfg.patch_size,
                        num_classes=cfg.num_classes, embed_dim=cfg.embed_dim, depths=cfg.depths,
                        num_heads=cfg.num_heads, dtype="bf16", weights=params, device=dev)
    report(name, m(img), z["logits"])
