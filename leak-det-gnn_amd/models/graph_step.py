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
    LG_SALT_SEED_PTR) that are re-drawn on the device for every replay: by the optimizer's
    own launch at the END of the previous replay when the optimizer can (ClipAdamW:
    lg_clip_adamw_seeds; one eager draw before the first replay), else by a launch at the
    head of the step (lg_seed_slots_advance).
  * The optimizer must be built with capturable=True (device-side step counters).
  * world > 1: no collective is ever captured.  A model that names a gradient split
    (`overlap_split()` -> the parameters whose gradients are final at a boundary tensor
    it keeps as `model.boundary`, LeakDetector: the two heads, 33,282 of 60,418 values)
    runs THREE graphs around two eager RCCL all-reduces:
      A1: forward + backward down to the boundary (CE, heads) + pack the head bucket;
      all-reduce(head bucket, async: RCCL's stream runs it while A2 runs);
      A2: backward from the boundary (trunk, GRU) + pack the trunk bucket;
      all-reduce(trunk bucket); wait for both;
      B:  unpack both + clip + optimizer.
    Without a split: graph A (forward + backward + pack), one all-reduce, graph B.
    `comm = False` skips the collectives (bench.py's exposed-exchange measurement only).
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
                 warmup: int = 3, seed_slots: int = 16, preserve_state: bool = False):
        """preserve_state: the eager warm-up steps (allocator pools, optimizer state) leave the
        parameters, the optimizer state and torch's CPU generator as they found them, so the
        first replay is the caller's next step (the training CLI switching to the graph
        mid-run).  Optimizer state created by the warm-up is zeroed (AdamW's initial value)."""
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
        self._build(model, warmup, preserve_state)

    def _build(self, model, warmup: int, preserve_state: bool) -> None:
        dev = self.label.device
        snap = self._snapshot() if preserve_state else None
        # eager warm-up on a side stream (allocator pools, optimizer state, cached graph CSR)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager_step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)

        self.opt.zero_grad(set_to_none=True)
        self.comm = True
        self.graph_a = torch.cuda.CUDAGraph()
        self.graph_a2 = None
        self.graph_b = None
        split = getattr(model, "overlap_split", None)
        self.heads = [p for p in split() if p.requires_grad] if (self.world > 1 and split is not None) else []
        hid = {id(p) for p in self.heads}
        self.trunk = [p for p in self.params if id(p) not in hid]
        ops.use_device_seeds(self.slots)
        # the optimizer draws the next replay's seeds in its own launch (ClipAdamW)
        self.fold_seeds = hasattr(self.opt, "seed_slots")
        head_refresh = not self.fold_seeds
        try:
            if self.world == 1:
                with torch.cuda.graph(self.graph_a):
                    if head_refresh:
                        self.slots.refresh()
                    # detached: the static loss must not keep the capture-time autograd graph
                    # (and its AccumulateGrad nodes, bound to the capture stream) alive, or a
                    # later eager backward on another stream would sync on them
                    self.loss = self._forward_backward().detach()
                    self._update(fold=self.fold_seeds)
            elif self.heads:
                model.keep_boundary = True
                try:
                    with torch.cuda.graph(self.graph_a):
                        if head_refresh:
                            self.slots.refresh()
                        loss = self.loss_fn(self.model(*self.inputs), self.label)
                        bnd = model.boundary
                        self._one = torch.ones_like(loss)
                        # retain_graph: A2 walks the trunk half of this autograd graph
                        torch.autograd.backward(loss, self._one, retain_graph=True, inputs=self.heads + [bnd])
                        self.loss = loss.detach()
                        self.flat_h = torch.cat([p.grad.reshape(-1) for p in self.heads])
                    self.graph_a2 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self.graph_a2, pool=self.graph_a.pool()):
                        torch.autograd.backward(bnd, bnd.grad, inputs=self.trunk)
                        self.flat_t = torch.cat([p.grad.reshape(-1) for p in self.trunk])
                finally:
                    model.keep_boundary = False
                    model.boundary = None
                del loss, bnd
                self.buckets = [(self.flat_h, self.heads), (self.flat_t, self.trunk)]
            else:
                with torch.cuda.graph(self.graph_a):
                    if head_refresh:
                        self.slots.refresh()
                    self.loss = self._forward_backward().detach()
                    self.flat = torch.cat([p.grad.reshape(-1) for p in self.params])
                self.buckets = [(self.flat, self.params)]
        finally:
            ops.use_device_seeds(None)
        if snap is not None:
            self._restore(snap)
        if self.fold_seeds and self.world == 1:
            self.slots.refresh()  # the first replay's seeds (each replay then draws the next one's)
            torch.cuda.synchronize(dev)
        if self.world > 1:
            grads, views = [], []
            for flat, ps in self.buckets:
                off = 0
                for p in ps:
                    grads.append(p.grad)
                    views.append(flat[off:off + p.numel()].view_as(p))
                    off += p.numel()
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b):
                torch._foreach_copy_(grads, views)
                self._update(fold=self.fold_seeds)
            if self.fold_seeds:
                self.slots.refresh()
                torch.cuda.synchronize(dev)

    def _opt_tensors(self) -> list:
        out = []
        for st in self.opt.state.values():
            out += [v for v in st.values() if torch.is_tensor(v)]
        for g in self.opt.param_groups:
            out += [v for v in g.values() if torch.is_tensor(v)]
        return out

    def _snapshot(self) -> tuple:
        with torch.no_grad():
            params = [(p, p.detach().clone()) for p in self.model.parameters()]
            opt = {id(t): (t, t.detach().clone()) for t in self._opt_tensors()}
        return params, opt, torch.get_rng_state()

    def _restore(self, snap: tuple) -> None:
        params, opt, rng = snap
        with torch.no_grad():
            for p, v in params:
                p.copy_(v)
            for t in self._opt_tensors():
                if id(t) in opt:
                    t.copy_(opt[id(t)][1])
                else:
                    t.zero_()
        torch.set_rng_state(rng)
        torch.cuda.synchronize()

    def _forward_backward(self) -> torch.Tensor:
        loss = self.loss_fn(self.model(*self.inputs), self.label)
        # the seed gradient is a resident constant: autograd's ones_like would be one more
        # (fill) launch per step
        if self._one is None or self._one.shape != loss.shape:
            self._one = torch.ones_like(loss)
        loss.backward(self._one)
        return loss

    def _update(self, fold: bool = False) -> None:
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip)
        if fold:  # the optimizer's launch also draws the next replay's dropout seeds
            self.opt.seed_slots = self.slots
        try:
            self.opt.step()
        finally:
            if fold:
                self.opt.seed_slots = None

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

    def _all_reduce(self, flat: torch.Tensor, async_op: bool = False):
        if dist.get_backend() == "nccl":
            return dist.all_reduce(flat, op=dist.ReduceOp.AVG, async_op=async_op)
        work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=async_op)  # gloo has no AVG
        if work is not None:
            work.wait()
        flat.div_(self.world)
        return None

    def __call__(self) -> torch.Tensor:
        self.graph_a.replay()
        if self.graph_b is not None:
            if self.graph_a2 is not None:
                # the head bucket's exchange overlaps the trunk backward (RCCL's own stream
                # waits for A1, the current stream runs A2 meanwhile)
                work = self._all_reduce(self.flat_h, async_op=True) if self.comm else None
                self.graph_a2.replay()
                if self.comm:
                    self._all_reduce(self.flat_t)
                    if work is not None:
                        work.wait()
            elif self.comm:
                self._all_reduce(self.flat)
            self.graph_b.replay()
        return self.loss
