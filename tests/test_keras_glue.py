"""CPU: the reference-side weight glue of INTEGRATION.md section 2 (keras_glue). No TensorFlow:
the reference ViT / ViT_Pruned is stood in for by plain objects with the reference's attribute
structure (modeling/models/vit.py:18-39, layers/norm.py:6, residual.py:5-6, attention.py:6-18,
ffn.py:8-9) holding numpy arrays in the Keras shapes (cls_token [1, 1, dim]). Checked: the C-ABI
order and shapes, the config read off the model (per-layer heads, head size, FFN width: nothing
hard-coded), both Keras weight-list orders, and that the ordered list drives the golden-pinned
oracle forward to the golden logits."""
import os
from types import SimpleNamespace as NS

import numpy as np
import pytest

from edgevisiontransformer_amd import keras_glue
from edgevisiontransformer_amd.weights import (make_images, make_vit_params, vit_config,
                                               vit_param_shapes)
from oracle import vit_ref
from tests.golden.make_golden import case_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dense(w, b=None):
    return NS(kernel=w, bias=b)


def fake_keras_vit(params, cfg):
    """An object graph shaped like the reference's built Keras ViT (variables as numpy arrays)."""
    blocks = []
    for i in range(cfg.depth):
        att = NS(num_heads=cfg.heads[i], h_k=cfg.head_dim[i],
                 to_qkv=_dense(params[f"l{i}.qkv_w"]),
                 to_out=_dense(params[f"l{i}.out_w"], params[f"l{i}.out_b"]))
        ffn = NS(net=NS(layers=[_dense(params[f"l{i}.fc1_w"], params[f"l{i}.fc1_b"]),
                                _dense(params[f"l{i}.fc2_w"], params[f"l{i}.fc2_b"])]))
        blocks += [NS(norm=NS(gamma=params[f"l{i}.ln1_g"], beta=params[f"l{i}.ln1_b"]), fn=NS(fn=att)),
                   NS(norm=NS(gamma=params[f"l{i}.ln2_g"], beta=params[f"l{i}.ln2_b"]), fn=NS(fn=ffn))]
    return NS(patch_size=cfg.patch_size, pos_embedding=params["pos"],
              cls_token=params["cls"].reshape(1, 1, -1),
              patch_to_embedding=_dense(params["patch_w"], params["patch_b"]),
              transformer=NS(net=NS(layers=blocks)),
              mlp_head=NS(layers=[_dense(params["head1_w"], params["head1_b"]),
                                  _dense(params["head2_w"], params["head2_b"])]))


CFGS = {
    "deit_tiny": vit_config(192, 12, 3, 768),
    # ViT_Pruned layerwise: ragged heads / widths per layer, head size 64 kept (vit.py:58-75)
    "pruned": vit_config(192, 3, 3, 768, head_size=64, heads_list=(1, 3, 2),
                         ffn_list=(284, 76, 768)),
}


@pytest.mark.parametrize("name", list(CFGS))
def test_ordered_keras_variables(name):
    cfg = CFGS[name]
    params = make_vit_params(cfg, seed=7)
    kv = fake_keras_vit(params, cfg)
    assert keras_glue.keras_vit_config(kv) == cfg
    out = keras_glue.ordered_keras_variables(kv)
    shapes = vit_param_shapes(cfg)
    assert len(out) == len(shapes)
    for (pname, shape), arr in zip(shapes, out):
        assert arr.dtype == np.float32 and arr.shape == shape, pname
        np.testing.assert_array_equal(arr, params[pname])


@pytest.mark.parametrize("head_first", [False, True])
@pytest.mark.parametrize("own_first", [False, True])
def test_reorder_keras_weight_list(own_first, head_first):
    """Every Keras tracking order: own variables first / last, and blocks before mlp_head (ViT)
    or after it (ViT_Pruned re-assigns self.transformer after ViT.__init__, reference vit.py:74,
    so Keras tracks the new block last)."""
    cfg = CFGS["pruned"]
    params = make_vit_params(cfg, seed=8)
    names = keras_glue.keras_weight_names(cfg, own_first=own_first, head_first=head_first)
    if head_first:
        k = names.index("patch_b")
        assert names[k + 1] == "head1_w" and names.index("l0.ln1_g") > names.index("head2_b")
    keras_list = [params[n].reshape(1, 1, -1) if n == "cls" else params[n] for n in names]
    out = keras_glue.reorder_keras_weight_list(keras_list, cfg)
    for (pname, _), arr in zip(vit_param_shapes(cfg), out):
        np.testing.assert_array_equal(arr, params[pname])
    with pytest.raises(ValueError):
        keras_glue.reorder_keras_weight_list(keras_list[:-1], cfg)
    bad = list(keras_list)
    k = names.index("l1.qkv_w")
    bad[k] = bad[k][:, :-64]  # a width that does not match the config
    with pytest.raises(ValueError):
        keras_glue.reorder_keras_weight_list(bad, cfg)


def test_ordered_list_drives_the_golden_forward():
    """The list, re-keyed in the C-ABI order, gives the oracle the golden logits (the same list
    evt_vit_create takes: INTEGRATION.md's MI355XViT)."""
    z = np.load(os.path.join(GOLDEN, "deit_tiny_b2.npz"))
    cfg = case_config("deit_tiny_b2")
    params = make_vit_params(cfg, seed=int(z["param_seed"]))
    ordered = keras_glue.ordered_keras_variables(fake_keras_vit(params, cfg))
    rekeyed = {name: arr for (name, _), arr in zip(vit_param_shapes(cfg), ordered)}
    img = make_images(int(z["batch"]), seed=int(z["image_seed"]))
    out = vit_ref.vit_forward(rekeyed, cfg, img)
    assert np.abs(out - z["logits"]).max() < 1e-9
