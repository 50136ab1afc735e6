"""CPU: pruned-checkpoint ingestion (edgevisiontransformer_amd/pruning.py). The sliced model must
equal the unpruned model with the pruned heads' out-proj rows and the pruned neurons' fc2 rows
zeroed (the definition of removing them), checked with the oracle."""
import os

import numpy as np
import pytest

from edgevisiontransformer_amd import pruning
from edgevisiontransformer_amd.modeling.models.vit import decode_prune_encoding
from edgevisiontransformer_amd.weights import make_images, make_vit_params, vit_config
from oracle.vit_ref import vit_forward

REF_IMPORTANCE = "/root/reference/are_16_heads/deit_tiny_head_importance.txt"


def test_prune_equals_zeroed_full_model():
    cfg = vit_config(128, 3, 2, 256, image_size=32, patch_size=16, num_classes=11, head_size=64,
                     heads_list=[2, 2, 2])
    params = make_vit_params(cfg, seed=4)
    kept_heads = [[1], [0, 1], [0]]
    kept_ffn = [list(range(0, 256, 3)), list(range(100)), [5, 77, 200]]
    p2, c2 = pruning.prune_vit_params(params, cfg, kept_heads, kept_ffn)
    assert list(c2.heads) == [1, 2, 1] and list(c2.ffn) == [86, 100, 3]
    zeroed = {k: v.copy() for k, v in params.items()}
    for i in range(3):
        ow = zeroed[f"l{i}.out_w"].reshape(2, 64, -1)
        for h in range(2):
            if h not in kept_heads[i]:
                ow[h] = 0
        mask = np.ones(256, bool)
        mask[kept_ffn[i]] = False
        zeroed[f"l{i}.fc2_w"][mask] = 0
    img = make_images(2, seed=5, image_size=32)
    a = vit_forward(p2, c2, img)
    b = vit_forward(zeroed, cfg, img)
    assert np.abs(a - b).max() < 1e-10


def test_nn_pruning_threshold_parsing_and_head_selection():
    th = pruning.parse_layerwise_thresholds("h_0.5_d_0.3-h_0.34_d_1.0-h_0.0_d_0.1")
    assert th == [{"head": 0.5, "ffn": 0.3}, {"head": 0.34, "ffn": 1.0}, {"head": 0.0, "ffn": 0.1}]
    enc = pruning.thresholds_to_encoding(th, 3)
    assert enc == "layerwise_h1-d0.3_h1-d1.0_h1-d0.1"
    assert decode_prune_encoding(enc) == ("layerwise", [1, 1, 1], [0.3, 1.0, 0.1])
    w = np.random.default_rng(0).standard_normal((64, 3 * 4 * 8))
    w4 = w.reshape(64, 3, 4, 8)
    w4[:, :, 2] = 0          # head 2: all of q, k, v zero -> score 0
    w4[:, 0, 1] = 0          # head 1: q zero -> score 2
    s = pruning.head_scores_nonzero(w, 4, 8)
    assert list(s) == [3, 2, 0, 3]
    assert pruning.select_heads_nn_pruning(s, 0.5) == [0, 3]
    assert pruning.select_heads_nn_pruning(np.zeros(4, int), 0.0) == [0]  # keep at least one


def test_heads_from_importance_budget():
    imp = np.array([[0.9, 0.1, 0.5], [0.2, 0.3, 0.4]])
    assert pruning.heads_from_importance(imp, keep_per_layer=[1, 2]) == [[0], [1, 2]]
    kept = pruning.heads_from_importance(imp, keep_total=3)
    assert kept == [[0, 2], [2]]
    assert pruning.heads_from_importance(np.array([[0.1, 0.2]]), keep_total=0) == [[1]]


@pytest.mark.skipif(not os.path.exists(REF_IMPORTANCE), reason="reference not mounted")
def test_reference_importance_file():
    """The reference's own are_16_heads table loads as [12 layers, 3 heads] (read as data)."""
    imp = pruning.load_head_importance(REF_IMPORTANCE)
    assert imp.shape == (12, 3)
    kept = pruning.heads_from_importance(imp, keep_per_layer=[2] * 12)
    assert all(len(k) == 2 for k in kept)


@pytest.mark.gpu
def test_pruned_checkpoint_on_gpu(gpu):
    """A sliced checkpoint (ragged heads 1..3 and arbitrary neuron sets) through the HIP path."""
    import torch
    cfg = vit_config(192, 12, 3, 768, num_classes=50)
    params = make_vit_params(cfg, seed=8)
    rng = np.random.default_rng(9)
    kept_heads = [sorted(rng.choice(3, size=1 + i % 3, replace=False).tolist()) for i in range(12)]
    kept_ffn = [sorted(rng.choice(768, size=64 + 50 * i, replace=False).tolist()) for i in range(12)]
    p2, c2 = pruning.prune_vit_params(params, cfg, kept_heads, kept_ffn)
    img = make_images(3, seed=10)
    ref = vit_forward(p2, c2, img)
    m = pruning.build_pruned_vit(params, cfg, kept_heads, kept_ffn, dtype="f32", device=gpu)
    out = m(torch.from_numpy(img).to(gpu)).cpu().numpy()
    assert np.abs(out - ref).max() <= 1e-3
