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
