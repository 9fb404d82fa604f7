"""The training loss, nn.CrossEntropyLoss() (reference train_detector.py:235, 311), as a
registered op on one HIP launch each way (csrc/loss.hip: lg_cross_entropy_fwd / _bwd).

torch's cross_entropy is six launches per step here (log_softmax, nll forward, two fills,
nll backward, log_softmax backward).  `CrossEntropyLoss` is a drop-in for the reference's
default-constructed module — mean reduction, ignore_index -100, no class weights, no label
smoothing, (B, C) fp32 logits with int64 targets on the GPU; anything else is handed to
torch's own implementation unchanged.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from ._native import check, load_library, ptr, stream_of

NS = "leakgnn"
_POOL_SLOTS = 256
_POOLS: dict = {}   # device -> int32 [_POOL_SLOTS] of completion counters, zeros at rest
_SLOTS: dict = {}   # (device, stream handle) -> index into the device's pool


def _counter(dev: torch.device, stream: int) -> Tensor:
    """lg_cross_entropy_fwd's completion counter for launches on `stream` (include/leakgnn.h:
    one per stream that may run the loss concurrently; the launch leaves it at 0).  Counters are
    slots of one per-device pool allocated (zeroed) on the first call, so a stream first seen
    while a HIP graph is being captured takes a slot without a captured fill; the graph keeps
    that slot's address for every replay (a shared per-device counter let an eager
    loss on one stream and a replayed step on another interleave their tickets)."""
    key = (dev, stream)
    i = _SLOTS.get(key)
    pool = _POOLS.get(dev)
    if pool is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("leakgnn cross_entropy: run the loss once eagerly before capturing it "
                               "(its counter pool is allocated on the first call)")
        pool = _POOLS[dev] = torch.zeros(_POOL_SLOTS, dtype=torch.int32, device=dev)
    if i is None:
        i = len([k for k in _SLOTS if k[0] == dev])
        if i >= _POOL_SLOTS:
            raise RuntimeError(f"leakgnn cross_entropy: more than {_POOL_SLOTS} streams on {dev}")
        _SLOTS[key] = i
    return pool[i:i + 1]


@torch.library.custom_op(f"{NS}::cross_entropy", mutates_args=(), device_types="cuda")
def cross_entropy(logits: Tensor, target: Tensor, ignore_index: int) -> Tuple[Tensor, Tensor]:
    """(mean loss, per-row logsumexp).  The row losses are summed in row order by the last
    workgroup to finish (deterministic)."""
    lib = load_library()
    x, t = logits.contiguous(), target.contiguous()
    B, C = x.shape
    loss = torch.empty((), device=x.device, dtype=torch.float32)
    lse = torch.empty(B, device=x.device, dtype=torch.float32)
    rowloss = torch.empty(B, device=x.device, dtype=torch.float32)
    st = stream_of(x)
    check(lib.lg_cross_entropy_fwd(ptr(x), ptr(t), B, C, C, ignore_index, ptr(loss), ptr(lse), ptr(rowloss),
                                   ptr(_counter(x.device, st)), st), "lg_cross_entropy_fwd")
    return loss, lse


@cross_entropy.register_fake
def _(logits, target, ignore_index):
    return logits.new_empty(()), logits.new_empty(logits.shape[0])


@torch.library.custom_op(f"{NS}::cross_entropy_backward", mutates_args=(), device_types="cuda")
def cross_entropy_backward(grad: Tensor, logits: Tensor, target: Tensor, lse: Tensor, ignore_index: int) -> Tensor:
    lib = load_library()
    x, t, g = logits.contiguous(), target.contiguous(), grad.contiguous().float()
    B, C = x.shape
    dx = torch.empty_like(x)
    check(lib.lg_cross_entropy_bwd(ptr(x), ptr(t), ptr(lse), ptr(g), B, C, C, ignore_index, ptr(dx), C,
                                   stream_of(x)), "lg_cross_entropy_bwd")
    return dx


@cross_entropy_backward.register_fake
def _(grad, logits, target, lse, ignore_index):
    return torch.empty_like(logits)


def _ce_setup(ctx, inputs, output):
    logits, target, ignore_index = inputs
    ctx.ignore_index = ignore_index
    ctx.mark_non_differentiable(output[1])
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(logits, target, output[1])


def _ce_bwd(ctx, g, _glse):
    if g is None:
        return None, None, None
    logits, target, lse = ctx.saved_tensors
    return torch.ops.leakgnn.cross_entropy_backward(g, logits, target, lse, ctx.ignore_index), None, None


cross_entropy.register_autograd(_ce_bwd, setup_context=_ce_setup)


class CrossEntropyLoss(torch.nn.CrossEntropyLoss):
    """nn.CrossEntropyLoss with the default configuration on the fused HIP op; any other
    configuration or input falls through to torch."""

    def forward(self, input: Tensor, target: Tensor) -> Tensor:
        if (self.weight is None and self.reduction == "mean" and self.label_smoothing == 0.0 and input.is_cuda
                and input.dim() == 2 and input.dtype == torch.float32 and target.dtype == torch.int64
                and target.dim() == 1):
            return torch.ops.leakgnn.cross_entropy(input, target, int(self.ignore_index))[0]
        return super().forward(input, target)
