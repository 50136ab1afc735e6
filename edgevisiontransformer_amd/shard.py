"""Batch sharding across the GPUs of one node + the logits gather (the path's only exchange).

Images are independent in the reference forward (`modeling/models/vit.py:41-55`: no op mixes
images), so a batch splits into contiguous per-rank shards with no data-path collective; the only
exchange is collecting the [B/G, C] fp32 logits, done with one all-gather (RCCL over xGMI on the
GPU box, gloo in the CPU tests). This is the inference analogue of the reference's distributed
evaluation (`deit_pruning/src/utils.py:151-228`: DistributedSampler shards, then dist.reduce).
"""
from __future__ import annotations

import datetime
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


class GatherTimeout(TimeoutError):
    """A rank's logits gather did not complete within its timeout (a peer is dead or hung)."""


def shard_range(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [start, stop) of rank `rank`; the first `global_batch % world` ranks
    take one extra image (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world or global_batch < 0:
        raise ValueError("bad world/rank/global_batch")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_logits(local: torch.Tensor, global_batch: int, world: int,
                  group: Optional[dist.ProcessGroup] = None,
                  timeout: Optional[float] = None) -> torch.Tensor:
    """All-gather every rank's [n_r, C] logits into [global_batch, C] in rank order.

    Shards may be uneven by one row; each rank pads to the largest shard so a single
    all_gather_into_tensor moves ceil(B/G)*C*4 bytes per rank.
    timeout (seconds): wait for the collective at most this long, then raise GatherTimeout
    instead of blocking forever on a dead peer (failure detection; the process
    group's own timeout, set at init_process_group, bounds it as well).
    """
    if world == 1:
        return local
    C = local.shape[1]
    cap = -(-global_batch // world)
    # gloo moves host tensors: stage device logits through the host (RCCL gathers in place)
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else local.device
    buf = torch.zeros((cap, C), dtype=local.dtype, device=dev)
    buf[: local.shape[0]] = local.to(dev)
    out = torch.empty((world * cap, C), dtype=local.dtype, device=dev)
    if timeout is None:
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        work = dist.all_gather_into_tensor(out, buf, group=group, async_op=True)
        try:
            done = work.wait(timeout=datetime.timedelta(seconds=timeout))
        except Exception as e:  # gloo raises on timeout; NCCL aborts the communicator
            raise GatherTimeout(f"rank {dist.get_rank(group)}: logits gather did not complete "
                                f"within {timeout:.1f} s ({type(e).__name__}: {e})") from e
        if done is False:
            raise GatherTimeout(f"rank {dist.get_rank(group)}: logits gather did not complete "
                                f"within {timeout:.1f} s")
    rows = []
    for r in range(world):
        s, e = shard_range(global_batch, world, r)
        rows.append(out[r * cap: r * cap + (e - s)])
    return torch.cat(rows, 0)


def sharded_forward(forward: Callable[[torch.Tensor], torch.Tensor], images: torch.Tensor,
                    world: int, rank: int, group: Optional[dist.ProcessGroup] = None,
                    timeout: Optional[float] = None) -> torch.Tensor:
    """Run `forward` on this rank's shard of `images` (global batch) and gather all logits."""
    s, e = shard_range(images.shape[0], world, rank)
    local = forward(images[s:e])
    return gather_logits(local, images.shape[0], world, group, timeout)
