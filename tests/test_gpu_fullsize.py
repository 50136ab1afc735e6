"""Every BASELINE.json GPU config at its benchmarked size.

Each test runs the full-size forward of the benchmarked batch twice, then checks:
  * batch independence, bitwise: the second forward runs the same images rolled by a prime
    number of positions (new neighbours, new offsets against the 256-row GEMM M-tiles); every
    image's logits row must be bit-identical in both (the reference has no cross-image op:
    `modeling/models/vit.py:41-55`, `t2t_vit.py:120-135`);
  * bs=1 vs full batch: rows {0, 1, mid, last, images straddling an M-tile boundary} against the
    bs=1 forward of the same image. Bitwise where both batch sizes run the same kernels (the f32
    path); the bf16 path switches from the 128x128 GEMM (bs=1: too few tiles) to the persistent
    256x256 GEMM at full size, whose epilogues round in a different order, so there the rows
    must agree within the bf16 gate below (measured max diffs are printed);
  * parity: the reference-pinned golden image (`tests/golden/*_b1.npz`) is placed at a
    tile-straddling position of the batch; its row is checked against the fp64 golden logits
    (f32 path: max-abs <= 1e-3; bf16 path: max-abs <= 3e-2 and cosine >= 0.9995);
  * all logits finite.
The other images are seeded N(0,1) (the bench's synthetic distribution).

Configs (BASELINE.json configs[1..4]): DeiT-tiny bs256 f32, DeiT-base bs512 bf16, T2T-ViT-14
bs256 bf16, Swin-T bs256 bf16 (the per-GPU share of bs2048 over 8 GPUs).
"""
import os

import numpy as np
import pytest
import torch

from edgevisiontransformer_amd.modeling.models.swin import SwinTransformer
from edgevisiontransformer_amd.modeling.models.t2t_vit import T2T_ViT
from edgevisiontransformer_amd.modeling.models.vit import ViT
from edgevisiontransformer_amd.weights import (digest, make_images, make_swin_params,
                                               make_t2t_params, make_vit_params, t2t_config,
                                               vit_config)
from tests.golden.make_golden import CASES, T2T_CASES

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
F32_TOL = 1e-3
BF16_ABS, BF16_COS = 3e-2, 0.9995
TILE = 256


def straddlers(batch, rows_per_image, count=3):
    """Images whose token rows cross a TILE-row boundary of the [batch * rows, D] GEMM operand,
    spread over the batch (first, middle, last such image)."""
    s = [i for i in range(batch)
         if (i * rows_per_image) // TILE != (i * rows_per_image + rows_per_image - 1) // TILE]
    if not s:
        return []
    return sorted({s[0], s[len(s) // 2], s[-1]})[:count]


def check_golden(row, gold, dtype, what):
    row, gold = np.asarray(row, np.float64), np.asarray(gold, np.float64)
    err = float(np.abs(row - gold).max())
    if dtype == "f32":
        assert err <= F32_TOL, f"{what}: f32 max-abs {err:.3e} > {F32_TOL}"
    else:
        cos = float((row * gold).sum() / (np.linalg.norm(row) * np.linalg.norm(gold)))
        assert err <= BF16_ABS and cos >= BF16_COS, \
            f"{what}: bf16 max-abs {err:.3e} (<= {BF16_ABS}), cosine {cos:.6f} (>= {BF16_COS})"
    return err


def run_fullsize(m, batch, shape, gold_img, gold_pos, rows_per_image, gpu, seed,
                 exact_bs1=False):
    g = torch.Generator(device=gpu).manual_seed(seed)
    img = torch.randn((batch, *shape), generator=g, device=gpu, dtype=torch.float32)
    img[gold_pos] = torch.from_numpy(gold_img).to(gpu)
    full = m(img)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(full).all()), "non-finite logits at full size"
    shift = 37
    rolled = m(torch.roll(img, shift, 0).contiguous())
    torch.cuda.synchronize()
    bad = (torch.roll(rolled, -shift, 0) != full).any(1).nonzero().flatten().tolist()
    assert not bad, f"{len(bad)} images change with their batch position (first: {bad[:5]})"
    idx = sorted({0, 1, batch // 2, batch - 1, gold_pos, *straddlers(batch, rows_per_image)})
    worst = 0.0
    for i in idx:
        one = m(img[i:i + 1].contiguous())
        torch.cuda.synchronize()
        if exact_bs1:
            assert torch.equal(one[0], full[i]), f"image {i}: bs=1 and bs={batch} rows differ"
        else:
            worst = max(worst, check_golden(one[0].cpu().numpy(), full[i].cpu().numpy(), "bf16",
                                            f"image {i} bs=1 vs bs={batch}"))
    print(f"bs=1 vs bs={batch}: max |diff| {worst:.3e} over images {idx}")
    return full


def test_deit_tiny_bs256_f32(gpu):
    kw, _, _, pseed, iseed = CASES["deit_tiny_b2"]
    cfg = vit_config(**kw)
    params = make_vit_params(cfg, seed=pseed)
    z = np.load(os.path.join(GOLDEN, "deit_tiny_b2.npz"))
    gimg = make_images(2, seed=iseed)
    assert digest([gimg]) == str(z["image_digest"])
    m = ViT(dtype="f32", weights=params, device=gpu, max_batch=256, **kw)
    pos = straddlers(256, cfg.tokens)[1]
    full = run_fullsize(m, 256, (3, 224, 224), gimg[1], pos, cfg.tokens, gpu, seed=31,
                        exact_bs1=True)
    check_golden(full[pos].cpu().numpy(), z["logits"][1], "f32", "deit_tiny bs256")


def test_deit_base_bs512_bf16(gpu):
    kw, _, _, pseed, iseed = CASES["deit_base_b1"]
    cfg = vit_config(**kw)
    params = make_vit_params(cfg, seed=pseed)
    z = np.load(os.path.join(GOLDEN, "deit_base_b1.npz"))
    gimg = make_images(1, seed=iseed)
    assert digest([gimg]) == str(z["image_digest"])
    m = ViT(dtype="bf16", weights=params, device=gpu, max_batch=512, **kw)
    pos = straddlers(512, cfg.tokens)[1]
    full = run_fullsize(m, 512, (3, 224, 224), gimg[0], pos, cfg.tokens, gpu, seed=32)
    err = check_golden(full[pos].cpu().numpy(), z["logits"][0], "bf16", "deit_base bs512")
    print(f"deit_base bs512 bf16: golden row {pos} max-abs {err:.3e}")


def test_t2t_vit_14_bs256_bf16(gpu):
    args, _, pseed, iseed = T2T_CASES["t2t_vit_14_b1"]
    h, depth, heads, ratio = args
    params = make_t2t_params(t2t_config(*args), seed=pseed)
    z = np.load(os.path.join(GOLDEN, "t2t_vit_14_b1.npz"))
    gimg = make_images(1, seed=iseed, layout="NHWC")
    assert digest([gimg]) == str(z["image_digest"])
    m = T2T_ViT(hidden_size=h, depth=depth, num_heads=heads, mlp_ratio=ratio, dtype="bf16",
                weights=params, device=gpu, max_batch=256)
    pos = straddlers(256, 197)[1]
    full = run_fullsize(m, 256, (224, 224, 3), gimg[0], pos, 197, gpu, seed=33)
    err = check_golden(full[pos].cpu().numpy(), z["logits"][0], "bf16", "t2t_vit_14 bs256")
    print(f"t2t_vit_14 bs256 bf16: golden row {pos} max-abs {err:.3e}")


def test_swin_tiny_bs256_bf16(gpu):
    from tests.test_swin_oracle import golden_case
    z, cfg, params, gimg = golden_case("swin_tiny_b1")
    m = SwinTransformer(img_size=cfg.image_size, patch_size=cfg.patch_size,
                        num_classes=cfg.num_classes, embed_dim=cfg.embed_dim, depths=cfg.depths,
                        num_heads=cfg.num_heads, dtype="bf16", weights=params, device=gpu,
                        max_batch=256)
    # stage-4 rows per image (7 x 7 = 49) straddle the 256-row tiles most often
    pos = straddlers(256, 49)[1]
    full = run_fullsize(m, 256, (3, 224, 224), gimg[0], pos, 49, gpu, seed=34)
    err = check_golden(full[pos].cpu().numpy(), z["logits"][0], "bf16", "swin_tiny bs256")
    print(f"swin_tiny bs256 bf16: golden row {pos} max-abs {err:.3e}")
