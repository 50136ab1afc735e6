"""bench.py's multi-rank code path (N > 1) on a one-GPU box: two ranks under torch.distributed.run
with --dist-backend gloo, both on cuda:0 (RCCL needs one GPU per rank; the driver's 8-GPU node
runs the same code with nccl). Checked: the JSON line reports n_gpus 2, weak and strong modes,
and the gathered logits equal single-process forwards of the same images bit for bit (strong:
the shards of one global batch, uneven at 13 images; weak: every rank's own batch). Reference
launch pattern: README.md:78 (torch.distributed.launch --nproc_per_node), deit_pruning/src/
train_main.py:404-409. This is a plumbing check of the N > 1 path, not a scaling number."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run_two_ranks(tmp_path, extra, port):
    dump = str(tmp_path / "logits.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1",
           "--cpu-seconds", "0", "--no-probe", "--dist-timeout", "90", "--dump-logits", dump, *extra]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=REPO, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0]), np.load(dump)


def _single(images):
    from edgevisiontransformer_amd.modeling.models import vit
    m = vit.build_named("deit_base", dtype="bf16", seed=0, max_batch=images.shape[0])
    out = m(images)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("global_batch", [13, 128])
def test_bench_strong_two_ranks(gpu, tmp_path, global_batch):
    line, got = _run_two_ranks(tmp_path, ["--global-batch", str(global_batch)], 29611 + global_batch % 7)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["dist_backend"] == "gloo"
    assert line["config"]["global_batch"] == global_batch and line["logits_finite"]
    assert got.shape == (global_batch, 1000)
    # bench.py's global batch (seed 1000 on cuda), each shard forwarded alone in this process
    g = torch.Generator(device="cuda").manual_seed(1000)
    gimg = torch.randn((global_batch, 3, 224, 224), generator=g, device="cuda", dtype=torch.float32)
    half = (global_batch + 1) // 2
    ref = np.concatenate([_single(gimg[:half]), _single(gimg[half:])])
    assert np.array_equal(got, ref)


def test_bench_weak_two_ranks(gpu, tmp_path):
    line, got = _run_two_ranks(tmp_path, ["--batch", "8"], 29627)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_batch"] == 16 and got.shape == (16, 1000)
    parts = []
    for rank in range(2):  # bench.py's weak-mode images of rank r: seed 1000 + r
        g = torch.Generator(device="cuda").manual_seed(1000 + rank)
        parts.append(_single(torch.randn((8, 3, 224, 224), generator=g, device="cuda",
                                         dtype=torch.float32)))
    assert np.array_equal(got, np.concatenate(parts))


def test_bench_weak_two_ranks_laned(gpu, tmp_path):
    """The multi-rank path with laned handles (T2T-ViT-14, 128 images per rank: two batch lanes
    each), both ranks on cuda:0: the line reports the lanes and finite gathered logits."""
    line, got = _run_two_ranks(tmp_path, ["--model", "t2t_vit_14", "--batch", "128"], 29633)
    assert line["n_gpus"] == 2 and line["config"]["lanes"] == 2 and line["logits_finite"]
    assert got.shape == (256, 1000)

