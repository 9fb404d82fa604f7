"""Batch data parallelism for the detector: one process per GPU, windows sharded
across ranks, one gradient all-reduce per step (RCCL over xGMI with backend
"nccl"; gloo on CPU for tests).

The reference is single-device; this is the one collective the
multi-GPU path adds.  The gradient of the 60,418-parameter detector is 241.7 KB.
GradAllReduce here is the EAGER form: one flat bucket, all-reduced once after backward
(the trainer's eager steps, the bench's kernel-timing pass).  The captured training step
(models/graph_step.py) splits it in two buckets and overlaps the heads' bucket (33,282
values, final at the trunk boundary) with the trunk and GRU backward; at ~242 KB the
exchange is latency-bound, so two buckets beat finer splits.
Mean-reduction semantics: each rank's loss is the mean over its local windows,
the all-reduce averages over ranks, so with equal shards the gradient equals the
single-process gradient of the global batch.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist


def dist_env() -> tuple:
    """(rank, local_rank, world_size) from torchrun's environment (1-process defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(backend: Optional[str] = None) -> tuple:
    rank, local_rank, world = dist_env()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, local_rank, world


class GradAllReduce:
    """Average gradients of `params` across the default process group in ONE flat bucket."""

    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.group = group
        numel = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.empty(numel, device=dev, dtype=torch.float32)

    def __call__(self) -> None:
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return
        world = dist.get_world_size(self.group)
        # one gather into the bucket, one collective, gradients re-pointed at the bucket.  After
        # the first call every p.grad is a view of the bucket; a caller that zeroes or
        # accumulates in place (zero_grad(set_to_none=False), micro-batches) keeps it that way,
        # and then the gradient is already in place: copy only the ones that are not.
        off = 0
        for p in self.params:
            n = p.numel()
            view = self.flat[off:off + n]
            if p.grad is None:
                view.zero_()
            elif not (p.grad.data_ptr() == view.data_ptr() and p.grad.is_contiguous()):
                view.copy_(p.grad.reshape(-1))
            off += n
        if dist.get_backend(self.group) == "nccl":
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=self.group)
        else:  # gloo has no AVG
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
            self.flat.div_(world)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n


def rank_generator_seed(seed: int, rank: int) -> int:
    """torch generator seed of `rank` for everything drawn AFTER the model is built.  Every
    rank builds the model from the same seed (identical initial weights), then reseeds
    with this: the dropout seeds the library draws per step (library.seed_tensor, the
    captured step's SeedSlots) come from torch's generator, and dropout masks are indexed
    by the rank-LOCAL row, so with one seed on every rank local window i would get the
    same mask on all ranks (a global batch of 512 on 8 ranks: 64 distinct patterns).
    Callers reseed only at world > 1, so a 1-process run draws what it always drew."""
    return (int(seed) + 0x9E3779B1 * int(rank)) % (1 << 63)


def reseed_rank(seed: int, rank: int, world: int) -> None:
    """Called once the model is built (identical weights everywhere): from here on every rank
    draws its own dropout seeds.  No-op at world 1."""
    if world > 1:
        torch.manual_seed(rank_generator_seed(seed, rank))


def shard_range(global_batch: int, rank: int, world: int) -> range:
    """Contiguous per-rank slice of the global sample index range (datasets are seeded by
    seed + idx, datasets.py:236,490, so the global batch is the same at any world size)."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} not divisible by world size {world}")
    per = global_batch // world
    return range(rank * per, (rank + 1) * per)
