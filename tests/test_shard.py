"""Multi-process (gloo, world_size 2 and 3) checks of the batch-shard + logits-gather path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from edgevisiontransformer_amd.shard import gather_logits, shard_range, sharded_forward


def test_shard_range_partitions():
    for B in (0, 1, 7, 512, 513):
        for G in (1, 2, 3, 8):
            spans = [shard_range(B, G, r) for r in range(G)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(spans[i][1] == spans[i + 1][0] for i in range(G - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _fake_forward(x):
    # deterministic per-image "logits": any cross-image mixing or reordering would show
    return torch.stack([x.sum(dim=(1, 2, 3)), x.amax(dim=(1, 2, 3)), x[:, 0, 0, 0]], 1)


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(5)
    imgs = torch.randn((B, 3, 8, 8), generator=g)
    out = sharded_forward(_fake_forward, imgs, world, rank)
    ref = _fake_forward(imgs)
    q.put((rank, bool(torch.equal(out, ref)), tuple(out.shape)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,B", [(2, 9), (3, 10), (2, 1)])
def test_sharded_forward_gloo(world, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and shape == (B, 3) for _, ok, shape in res), res


def test_gather_single_rank_is_identity():
    x = torch.randn(5, 4)
    assert gather_logits(x, 5, 1) is x


def _timeout_worker(rank, world, port, q):
    import time
    from edgevisiontransformer_amd.shard import GatherTimeout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = torch.full((2, 3), float(rank))
    if rank == 0:  # rank 1 is "hung": it never enters the gather
        t0 = time.time()
        try:
            gather_logits(local, 4, world, timeout=2.0)
            q.put((rank, "no timeout", time.time() - t0))
        except GatherTimeout as e:
            q.put((rank, "timeout", time.time() - t0, str(e)))
    else:
        time.sleep(6.0)
        q.put((rank, "skipped"))
    q.close()
    q.join_thread()  # flush the result before the hard exit
    os._exit(0)  # the group is broken on purpose: no destroy_process_group handshake


def test_gather_timeout_gloo():
    """A peer that never joins the logits gather: the waiting rank raises GatherTimeout within
    its timeout instead of hanging (SURVEY.md 5 failure detection)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r[0]: r for r in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
    assert res[0][1] == "timeout", res
    assert res[0][2] < 5.0, res  # bounded by the 2 s timeout, not by the peer's 6 s
    assert "rank 0" in res[0][3]


def _sharded_model_worker(rank, world, port, B, q):
    """sharded_forward over a real (CPU) restatement of the ViT forward, not a fake: every rank
    runs the numpy oracle on its shard; the gathered logits equal the single-process forward."""
    import numpy as np
    from oracle.vit_ref import vit_forward
    from edgevisiontransformer_amd.weights import make_images, make_vit_params, vit_config
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = vit_config(64, 1, 1, 128, image_size=32, patch_size=16, num_classes=5)
    params = make_vit_params(cfg, seed=3)
    imgs = torch.from_numpy(make_images(B, seed=4, image_size=32))

    def forward(x):
        return torch.from_numpy(vit_forward(params, cfg, x.numpy(), dtype=np.float32))
    out = sharded_forward(forward, imgs, world, rank, timeout=60.0)
    ref = forward(imgs)
    # numpy BLAS rounds differently per batch size: close, not bitwise (the GPU path is bitwise,
    # tests/test_gpu_fullsize.py)
    q.put((rank, bool(torch.allclose(out, ref, rtol=1e-5, atol=1e-6)), tuple(out.shape)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 5), (3, 7)])
def test_sharded_model_forward_gloo(world, B):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_model_worker, args=(r, world, port, B, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok and shape == (B, 5) for _, ok, shape in res), res
