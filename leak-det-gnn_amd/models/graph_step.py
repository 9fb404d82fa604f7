"""Whole-step HIP-graph capture of a LeakDetector training step.

The reference runs its training step (train_detector.py:310-317: forward, CE, backward,
clip_grad_norm_(1.0), AdamW) as ~60 eagerly launched kernels, each paying Python +
autograd + launch latency on the host.  At the benchmark shape (B = 256 windows) the
device work of one step is ~1 ms, so the host side is as long as the GPU side.  Here the
whole step is captured ONCE into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm)
and replayed: one graph launch per step, the kernels back to back on the device.

  * Inputs are static device tensors; a caller with new data copies it into
    `step.inputs` / `step.label` before calling the step (the copy is part of its loop,
    as the reference's `.to(device)` is, train_detector.py:297-299).
  * Dropout stays random per replay: while capturing, the library's dropout call sites
    read their seeds from device slots (ops.SeedSlots, include/leakgnn.h
    LG_SALT_SEED_PTR) that a captured torch RNG op re-draws at the head of every replay.
  * The optimizer must be built with capturable=True (device-side step counters).
  * world > 1: the step is two graphs around ONE eager RCCL all-reduce of a flat
    gradient bucket (graph A: forward + backward + pack; all-reduce; graph B: unpack +
    clip + AdamW), so no collective is ever captured.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch
import torch.distributed as dist

from . import ops


def _world() -> int:
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


class CapturedTrainStep:
    """step() == one training step of `model` on the static (inputs, label), replayed from a
    captured graph.  Returns the (static) loss tensor of the step."""

    def __init__(self, model: torch.nn.Module, loss_fn: Callable, opt: torch.optim.Optimizer,
                 inputs: Sequence[torch.Tensor], label: torch.Tensor, clip: Optional[float] = 1.0,
                 warmup: int = 3, seed_slots: int = 16):
        for group in opt.param_groups:
            if not group.get("capturable", False):
                raise ValueError("CapturedTrainStep needs an optimizer built with capturable=True")
        self.model, self.loss_fn, self.opt, self.clip = model, loss_fn, opt, clip
        self.inputs, self.label = tuple(inputs), label
        self.params = [p for p in model.parameters() if p.requires_grad]
        dev = label.device
        self.world = _world()
        self.slots = ops.SeedSlots(dev, seed_slots)
        self._one: Optional[torch.Tensor] = None

        # eager warm-up on a side stream (allocator pools, optimizer state, cached graph CSR)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager_step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)

        self.opt.zero_grad(set_to_none=True)
        self.graph_a = torch.cuda.CUDAGraph()
        self.graph_b = None
        ops.use_device_seeds(self.slots)
        try:
            with torch.cuda.graph(self.graph_a):
                self.slots.refresh()
                # detached: the static loss must not keep the capture-time autograd graph
                # (and its AccumulateGrad nodes, bound to the capture stream) alive, or a
                # later eager backward on another stream would sync on them
                self.loss = self._forward_backward().detach()
                if self.world == 1:
                    self._update()
                else:
                    self.grads = [p.grad for p in self.params]
                    self.flat = torch.cat([g.reshape(-1) for g in self.grads])
        finally:
            ops.use_device_seeds(None)
        if self.world > 1:
            views, off = [], 0
            for g in self.grads:
                views.append(self.flat[off:off + g.numel()].view_as(g))
                off += g.numel()
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b):
                torch._foreach_copy_(self.grads, views)
                self._update()

    def _forward_backward(self) -> torch.Tensor:
        loss = self.loss_fn(self.model(*self.inputs), self.label)
        # the seed gradient is a resident constant: autograd's ones_like would be one more
        # (fill) launch per step
        if self._one is None or self._one.shape != loss.shape:
            self._one = torch.ones_like(loss)
        loss.backward(self._one)
        return loss

    def _update(self) -> None:
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        self.opt.step()

    def _eager_step(self) -> None:
        self.opt.zero_grad(set_to_none=True)
        self._forward_backward()
        if self.world > 1:
            flat = torch.cat([p.grad.reshape(-1) for p in self.params])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat.div_(self.world)
            off = 0
            for p in self.params:
                p.grad.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
        self._update()

    def __call__(self) -> torch.Tensor:
        self.graph_a.replay()
        if self.graph_b is not None:
            if dist.get_backend() == "nccl":
                dist.all_reduce(self.flat, op=dist.ReduceOp.AVG)
            else:  # gloo has no AVG
                dist.all_reduce(self.flat, op=dist.ReduceOp.SUM)
                self.flat.div_(self.world)
            self.graph_b.replay()
        return self.loss
