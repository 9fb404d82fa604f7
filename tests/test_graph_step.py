"""Whole-step HIP-graph capture (models/graph_step.py) and device-resident dropout seeds
(include/leakgnn.h LG_SALT_SEED_PTR): the replayed step must compute exactly what the
eager step computes."""
from __future__ import annotations

import copy
import os
import socket

import pytest
import torch

from helpers import LTA_INP, assert_close, lta_ids

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _model(dropout: float, seed: int = 0):
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(seed)
    return LeakDetector(LTA_INP, sensors, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2,
                        dropout=dropout).to(DEV).train()


def _batch(B: int, seed: int = 1):
    gen = torch.Generator().manual_seed(seed)
    r = torch.randn(B, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(B, 36, 9, generator=gen).to(DEV)
    lab = torch.randint(0, 765, (B,), generator=gen).to(DEV)
    return r, tf, lab


def _opt(m):
    return torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4, fused=True, capturable=True)


def _eager_step(m, opt, r, tf, lab):
    opt.zero_grad(set_to_none=True)
    loss = torch.nn.functional.cross_entropy(m(r, tf), lab)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    opt.step()
    return loss


def test_captured_step_matches_eager_without_dropout():
    """dropout = 0: warm-up + K replays == warm-up + K eager steps (same kernels, same
    order, deterministic reductions), parameters and loss."""
    from models.graph_step import CapturedTrainStep
    r, tf, lab = _batch(6)
    m1 = _model(0.0)
    m2 = copy.deepcopy(m1)
    o1, o2 = _opt(m1), _opt(m2)
    step = CapturedTrainStep(m2, torch.nn.functional.cross_entropy, o2, (r, tf), lab, clip=1.0, warmup=3)
    for _ in range(3):
        _eager_step(m1, o1, r, tf, lab)
    for _ in range(4):
        l1 = _eager_step(m1, o1, r, tf, lab)
        l2 = step()
    torch.cuda.synchronize()
    assert_close(l2, l1, rtol=1e-6, what="loss")
    for (n, a), b in zip(m2.named_parameters(), m1.parameters()):
        assert_close(a, b, rtol=1e-5, what=n)


def test_captured_forward_reads_device_seeds():
    """Train mode: a captured forward takes its dropout seeds from device slots; an eager
    forward given the same seed VALUES (read back after the replay) is bit-identical."""
    from models import ops
    r, tf, _ = _batch(5)
    m = _model(0.1)
    with torch.no_grad():
        m(r, tf)  # device state (graph CSR, incidence) built outside the capture
    slots = ops.SeedSlots(DEV)
    g = torch.cuda.CUDAGraph()
    ops.use_device_seeds(slots)
    try:
        with torch.no_grad(), torch.cuda.graph(g):
            slots.refresh()
            out = m(r, tf)
    finally:
        ops.use_device_seeds(None)
    outs, seeds = [], []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        outs.append(out.clone())
        seeds.append([int(v) for v in slots.buf[:slots.i].cpu()])
    assert seeds[0] != seeds[1] and not torch.equal(outs[0], outs[1])  # re-drawn per replay
    from models import library
    orig = library.seed_tensor
    for got, sd in zip(outs, seeds):
        it = iter(sd)
        library.seed_tensor = lambda device=None: torch.tensor([next(it)], dtype=torch.long)
        try:
            with torch.no_grad():
                ref = m(r, tf)
        finally:
            library.seed_tensor = orig
        assert torch.equal(got, ref)


def test_captured_train_step_with_dropout_learns():
    """Train mode through the graph: finite losses that fall on a fixed batch."""
    from models.graph_step import CapturedTrainStep
    r, tf, lab = _batch(8)
    m = _model(0.1)
    step = CapturedTrainStep(m, torch.nn.functional.cross_entropy, _opt(m), (r, tf), lab, clip=1.0, warmup=2)
    losses = [float(step()) for _ in range(30)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert sum(losses[-5:]) < sum(losses[:5])


def _dp_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from models.graph_step import CapturedTrainStep
    r, tf, lab = _batch(8)
    sl = slice(4 * rank, 4 * rank + 4)
    m = _model(0.0)
    step = CapturedTrainStep(m, torch.nn.functional.cross_entropy, _opt(m), (r[sl], tf[sl]), lab[sl], warmup=2)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({n: p.detach().cpu() for n, p in m.named_parameters()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_captured_step_two_ranks_equals_full_batch(tmp_path):
    """world = 2 (gloo, both ranks on this GPU): graph A + eager all-reduce + graph B ==
    one process on the concatenated batch (mean CE: averaged grads are the full-batch
    grads), up to summation order."""
    import torch.multiprocessing as mp
    from models.graph_step import CapturedTrainStep
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "p.pt")
    mp.start_processes(_dp_worker, args=(2, port, out), nprocs=2, start_method="spawn")
    got = torch.load(out, weights_only=True)
    r, tf, lab = _batch(8)
    m = _model(0.0)
    step = CapturedTrainStep(m, torch.nn.functional.cross_entropy, _opt(m), (r, tf), lab, warmup=2)
    for _ in range(3):
        step()
    for n, p in m.named_parameters():
        assert_close(got[n], p, rtol=2e-5, what=n)


def test_captured_step_with_clip_adamw_matches_eager():
    """The bench's step: the fused cross-entropy and ClipAdamW (clip_grad_norm_ + AdamW,
    device step counter) inside the captured graph == the same loss and optimizer stepped
    eagerly (each is checked against torch's in test_gpu_library.py)."""
    from models.graph_step import CapturedTrainStep
    from models.optim import ClipAdamW
    r, tf, lab = _batch(6)
    m1 = _model(0.0)
    m2 = copy.deepcopy(m1)
    o1 = ClipAdamW(m1.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    o2 = ClipAdamW(m2.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    from models.loss import CrossEntropyLoss
    ce = CrossEntropyLoss()  # the bench's loss: the fused HIP op, inside the graph too
    step = CapturedTrainStep(m2, ce, o2, (r, tf), lab, clip=None, warmup=3)

    def eager():
        o1.zero_grad(set_to_none=True)
        loss = ce(m1(r, tf), lab)
        loss.backward()
        o1.step()
        return loss
    for _ in range(3):
        eager()
    for _ in range(4):
        l1 = eager()
        l2 = step()
    torch.cuda.synchronize()
    assert_close(l2, l1, rtol=1e-6, what="loss")
    for (n, a), b in zip(m2.named_parameters(), m1.parameters()):
        assert_close(a, b, rtol=1e-5, what=n)
