"""Autograd-level operators over libleakgnn (HIP kernels for gfx950).

Graph state lives on the device once per graph:
  * ``GCNGraph``   - gcn_norm'ed CSR keyed by destination and its transpose
                     (lg_graph_build; replaces PyG gcn_norm, recomputed per call in
                     the reference because GCNConv is built with cached=False,
                     detector.py:163,199).
  * ``Incidence``  - pipe-endpoint incidence CSR (lg_incidence_build) for the
                     deterministic backward of the EdgeHead gathers (detector.py:206-210).

The differentiable operators themselves are registered with torch.library
(namespace ``leakgnn``, models/library.py): gcn_conv, mean_pool, sensor_proj,
gru_encoder, gnn_trunk, detector_heads, each with a registered autograd formula.
This module keeps the device-side graph state, dropout-seed sources, the kernel timer
and the non-differentiable helpers (batchify, pipe_features, spmm).
"""
from __future__ import annotations

import ctypes
import os
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from . import _native as nat
from ._native import check, load_library, ptr, require_device, stream_of

SUPPORTED_D = (32, 64)

# Layout of the LeakDetector node features between GNNTrunkFn and HeadsFn.  "node"
# (default): [N][B][D], row n*B + b — the B windows of a node are contiguous, so a GCN
# tile (1 node x 16 windows) gathers one contiguous block per neighbour (lg_gcn_fwd_nm /
# lg_gcn_bwd_nm).  "window": the reference's disjoint-union order [B][N][D]
# (detector.py:105-114, 192-196) through lg_gcn_fwd / lg_gcn_bwd.  Both give the same
# results (same dropout masks); only the memory order differs.
TRUNK_NODE_MAJOR = os.environ.get("LEAKGNN_LAYOUT", "node") != "window"
NM_MAX_BYTES = 0x7FFFF000  # lg_gcn_fwd_nm / lg_gcn_bwd_nm: one [N][B][D] activation per launch


def use_node_major(B: int, N: int, D: int, bf16: bool = False) -> bool:
    """Trunk layout for a batch: node-major when a 16-window tile is mostly full (B >= 16)
    and the activation fits one node-major launch; window-major otherwise (B = 1 graphs
    such as C5, where a node-major tile would carry 1 window in 16).  The bf16 node-MLP
    tier exists only in the node-major kernels (the window-major ones compute fp32), so
    bf16 takes the node-major layout at every B: the tier's precision never depends on the
    batch size (a small per-rank batch, a ragged eval batch)."""
    fits = N * B * D * 4 <= NM_MAX_BYTES
    if bf16:
        if not fits:
            raise NotImplementedError(f"bf16 tier: a node-major activation of {N * B * D * 4} bytes exceeds "
                                      f"one launch ({NM_MAX_BYTES}); use a smaller batch or fp32")
        return True
    return TRUNK_NODE_MAJOR and B >= 16 and fits


# lg_gcn_fwd_nm kernel / transform bits (LG_F_NM3, LG_F_BF16X3, LG_F_F32_MFMA; include/leakgnn.h) for
# A/B timing of the trunk forward inside the training step (bench.py --trunk-fwd-flags).
GCN_FWD_NM_EXTRA_FLAGS = int(os.environ.get("LEAKGNN_GCN_FWD_NM_FLAGS", "0"), 0)
# the dense (non-x0) trunk layers' forward only (layer 0 keeps its x0 kernel): the same-box in-step A/B
# of the forward pipelines (LG_F_NM3 = 0x20000: nm3, one wave per tile, 3-way bf16 split)
GCN_FWD_DENSE_EXTRA_FLAGS = int(os.environ.get("LEAKGNN_GCN_FWD_DENSE_FLAGS", "0"), 0)
# lg_gcn_bwd_nm* transform bits on the fp32 tier.  Default LG_F_BF16X3 (0x8000): the 3-way bf16
# split, measured faster in the step than the kernel's f16x2 default on the same box (r05r:
# 48.2 / 37.2 against 50.2 / 38.1 us for layers 2 / 1, step 0.5848 against 0.5882 ms; VERDICT
# r04 item 4's "restore bf16x3 unless f16x2 is >= 3 % faster").  LEAKGNN_GCN_BWD_NM_FLAGS=0
# selects the f16x2 split.
GCN_BWD_NM_EXTRA_FLAGS = int(os.environ.get("LEAKGNN_GCN_BWD_NM_FLAGS", "0x8000"), 0)


# ----------------------------------------------------------------------------- timing hook
class KernelTimer:
    """Optional HIP-event timing of named kernel launches (used by bench.py).

    Each named library call arms one event pair of the library (lg_timing_arm,
    include/leakgnn.h): its main kernel is then launched with hipExtLaunchKernelGGL and
    that pair, so the elapsed time is the kernel's own execution on its stream — what a
    profiler's kernel trace reports — not the enqueue gaps a pair of event commands
    around the call would add.
    """

    def __init__(self, names: Sequence[str]):
        self.names = set(names)
        self.events: dict = {n: [] for n in names}  # name -> [slot]
        self.enabled = False
        self._next = 0

    def wrap(self, name: str, device: torch.device):
        timer = self

        class _Ctx:
            def __enter__(self_inner):
                self_inner.slot = None
                if timer.enabled and name in timer.names:
                    slot = timer._next
                    timer._next += 1
                    check(load_library().lg_timing_arm(slot), "lg_timing_arm")
                    self_inner.slot = slot
                return self_inner

            def __exit__(self_inner, *exc):
                if self_inner.slot is not None:
                    if load_library().lg_timing_disarm():
                        raise RuntimeError(f"KernelTimer: {name} launched no timed kernel")
                    timer.events[name].append(self_inner.slot)
                return False

        return _Ctx()

    def mean_ms(self, name: str) -> Optional[float]:
        slots = self.events.get(name, [])
        if not slots:
            return None
        torch.cuda.synchronize()
        lib, ms = load_library(), ctypes.c_float()
        tot = 0.0
        for s in slots:
            check(lib.lg_timing_elapsed(s, ctypes.byref(ms)), "lg_timing_elapsed")
            tot += ms.value
        return tot / len(slots)

    def count(self, name: str) -> int:
        return len(self.events.get(name, []))

    def reset(self) -> None:
        for n in self.events:
            self.events[n] = []
        self._next = 0


_TIMER: Optional[KernelTimer] = None


def set_kernel_timer(timer: Optional[KernelTimer]) -> None:
    global _TIMER
    _TIMER = timer


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _timed(name: str, device: torch.device):
    if _TIMER is None:
        return _NullCtx()
    return _TIMER.wrap(name, device)


# ----------------------------------------------------------------------------- graph state
def _validate_edge_index(edge_index: torch.Tensor, num_nodes: int) -> None:
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"edge_index must be (2, E), got {tuple(edge_index.shape)}")
    if edge_index.dtype != torch.long:
        raise TypeError("edge_index must be int64")
    if edge_index.numel() and not edge_index.is_cuda:
        lo, hi = int(edge_index.min()), int(edge_index.max())
        if lo < 0 or hi >= num_nodes:
            raise IndexError(f"edge_index values must lie in [0, {num_nodes}), got [{lo}, {hi}]")


@dataclass
class GCNGraph:
    num_nodes: int
    num_edges: int
    rowptr: torch.Tensor
    col: torch.Tensor
    w: torch.Tensor
    rowptr_t: torch.Tensor
    col_t: torch.Tensor
    w_t: torch.Tensor
    pairs: Optional[torch.Tensor] = None    # int32 (cap, 2): (col, float bits of w), node-major kernels
    pairs_t: Optional[torch.Tensor] = None  # same for the transposed CSR
    nodetab: Optional[torch.Tensor] = None    # int32 (2N, 16): node-major kernels' per-node records
    nodetab_t: Optional[torch.Tensor] = None  # same for the transposed CSR
    order: Optional[torch.Tensor] = None      # int32 (N,): their schedule order (reverse Cuthill-McKee)


    @staticmethod
    def build(edge_index: torch.Tensor, num_nodes: int, device: torch.device, add_self_loops: bool = True,
              normalize: bool = True, improved: bool = False) -> "GCNGraph":
        """gcn_norm + CSR on the device (lg_graph_build)."""
        lib = load_library()
        _validate_edge_index(edge_index, num_nodes)
        ei = edge_index.to(device=device, dtype=torch.long).contiguous()
        E, N = int(ei.size(1)), int(num_nodes)
        cap = E + N
        i32 = dict(device=device, dtype=torch.int32)
        f32 = dict(device=device, dtype=torch.float32)
        g = GCNGraph(N, E, torch.empty(N + 1, **i32), torch.empty(cap, **i32), torch.empty(cap, **f32),
                     torch.empty(N + 1, **i32), torch.empty(cap, **i32), torch.empty(cap, **f32))
        g.nnz_cap = cap
        ws = torch.empty(int(lib.lg_graph_workspace_bytes(E, N)), device=device, dtype=torch.uint8)
        fill = 2.0 if improved else 1.0
        check(lib.lg_graph_build(ptr(ei), E, N, int(add_self_loops), int(normalize), fill, ptr(g.rowptr),
                                 ptr(g.col), ptr(g.w), ptr(g.rowptr_t), ptr(g.col_t), ptr(g.w_t), ptr(ws), ws.numel(),
                                 stream_of(ei)), "lg_graph_build")
        g._keepalive = (ei, ws)  # freed after the stream consumes them
        g.pairs = torch.stack([g.col, g.w.view(torch.int32)], dim=1).contiguous()
        g.pairs_t = torch.stack([g.col_t, g.w_t.view(torch.int32)], dim=1).contiguous()
        # node-major schedule order: reverse Cuthill-McKee (host, once per graph), so a tile's
        # neighbour rows were gathered by the tiles just before it (L2 reuse); results do
        # not depend on it
        g.order = schedule_order(edge_index, N).to(device)
        g.nodetab = torch.empty(2 * N, 16, **i32)
        g.nodetab_t = torch.empty(2 * N, 16, **i32)
        check(lib.lg_nm_table_build(ptr(g.rowptr), ptr(g.pairs), N, ptr(g.order), ptr(g.nodetab), stream_of(ei)),
              "lg_nm_table_build")
        check(lib.lg_nm_table_build(ptr(g.rowptr_t), ptr(g.pairs_t), N, ptr(g.order), ptr(g.nodetab_t),
                                    stream_of(ei)), "lg_nm_table_build")
        return g


@dataclass
class SensorMarks:
    """The compressed layer-0 input's view of a graph (lg_nm_table_sensor_mark): the forward
    node table and pair array with every sensor column rewritten to 0x40000000 | slot, and the
    transposed table's schedule-section slots (pos_slot_t) for the backward's own rows."""
    nodetab_s: torch.Tensor
    pairs_s: torch.Tensor
    pos_slot_t: torch.Tensor

    @staticmethod
    def build(g: GCNGraph, node_slot: torch.Tensor) -> "SensorMarks":
        lib = load_library()
        N = g.num_nodes
        slot = node_slot.to(device=g.nodetab.device, dtype=torch.int32).contiguous()
        tab_s, pairs_s = torch.empty_like(g.nodetab), torch.empty_like(g.pairs)
        pos, pos_t = torch.empty(N, dtype=torch.int32, device=slot.device), torch.empty_like(slot)
        scratch_t, scratch_p = torch.empty_like(g.nodetab_t), torch.empty_like(g.pairs_t)
        st = stream_of(slot)
        check(lib.lg_nm_table_sensor_mark(ptr(g.nodetab), ptr(g.pairs), N, g.pairs.shape[0], ptr(slot), ptr(tab_s),
                                          ptr(pairs_s), ptr(pos), st), "lg_nm_table_sensor_mark")
        check(lib.lg_nm_table_sensor_mark(ptr(g.nodetab_t), ptr(g.pairs_t), N, g.pairs_t.shape[0], ptr(slot),
                                          ptr(scratch_t), ptr(scratch_p), ptr(pos_t), st), "lg_nm_table_sensor_mark")
        marks = SensorMarks(tab_s, pairs_s, pos_t)
        marks._keepalive = (slot, pos, scratch_t, scratch_p)  # live until the stream has consumed them
        return marks


def schedule_order(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """int32 (N,) reverse Cuthill-McKee order of the graph (lg_rcm_order, host)."""
    ei = edge_index.detach().to("cpu", torch.long).contiguous()
    order = torch.empty(int(num_nodes), dtype=torch.int32)
    check(load_library().lg_rcm_order(ei.data_ptr() if ei.numel() else None, int(ei.size(1)), int(num_nodes),
                                      order.data_ptr()), "lg_rcm_order")
    return order


@dataclass
class Incidence:
    num_nodes: int
    num_pipes: int
    ends: torch.Tensor      # int64 (P, 2) device
    rowptr: torch.Tensor    # int32 (N+1,)
    item: torch.Tensor      # int32 (2P,): ascending per node, or (schedule) in the pipe schedule's order
    # D -> (device int32 schedule, its 16 header words): lg_pipe_schedule_build, the streamed
    # node sums of the EdgeHead backward (ABI 22); empty when built without a schedule
    sched: dict = None

    @staticmethod
    def build(pipe_ends: torch.Tensor, num_nodes: int, device: torch.device, schedule: bool = True) -> "Incidence":
        """schedule=True: the pipe schedules for D = 32 and 64 (host-built, uploaded) and the
        incidence CSR in schedule order, from the same build, so every scatter path of the
        EdgeHead backward sums each node's incidences in one order; False: lg_incidence_build
        (items ascending, the reference order of index_add over item ids)."""
        lib = load_library()
        ends = pipe_ends.to(device=device, dtype=torch.long).contiguous()
        P, N = int(ends.size(0)), int(num_nodes)
        if P and not pipe_ends.is_cuda:
            lo, hi = int(pipe_ends.min()), int(pipe_ends.max())
            if lo < 0 or hi >= N:
                raise IndexError(f"pipe_ends values must lie in [0, {N}), got [{lo}, {hi}]")
        inc = Incidence(N, P, ends, torch.empty(N + 1, device=device, dtype=torch.int32),
                        torch.empty(max(2 * P, 1), device=device, dtype=torch.int32), {})
        if schedule and P > 0:
            he = pipe_ends.detach().to("cpu", torch.long).contiguous()
            rp = torch.empty(N + 1, dtype=torch.int32)
            it = torch.empty(2 * P, dtype=torch.int32)
            built = {}
            for D in (32, 64):
                words = int(lib.lg_pipe_schedule_words(P, N, D))
                sc = torch.zeros(max(words, 16), dtype=torch.int32)
                rc = lib.lg_pipe_schedule_build(he.data_ptr(), P, N, D, sc.data_ptr(), words, rp.data_ptr(), it.data_ptr())
                if rc != 0:
                    built = {}
                    break
                hdr = tuple(int(v) for v in sc[:16].tolist())
                built[D] = (sc[:hdr[13]].to(device), hdr)
            if built:
                inc.rowptr.copy_(rp)
                inc.item[:2 * P].copy_(it)
                inc.sched = built
                return inc
        ws = torch.empty(int(lib.lg_incidence_workspace_bytes(P, N)), device=device, dtype=torch.uint8)
        check(lib.lg_incidence_build(ptr(ends), P, N, ptr(inc.rowptr), ptr(inc.item), ptr(ws), ws.numel(), stream_of(ends)),
              "lg_incidence_build")
        inc._keepalive = ws
        return inc

    def schedule(self, D: int):
        """(device schedule or None, header words as a list) for the heads ops."""
        t = (self.sched or {}).get(int(D))
        return (t[0], list(t[1])) if t is not None else (None, [])


def batchify_edge_index(edge_index_single: torch.Tensor, num_nodes: int, batch_size: int) -> torch.Tensor:
    """Disjoint union of B copies (bit-exact with detector.py:105-114), on the device."""
    require_device(edge_index_single)
    lib = load_library()
    ei = edge_index_single.to(torch.long).contiguous()
    E = int(ei.size(1))
    out = torch.empty(2, E * batch_size, device=ei.device, dtype=torch.long)
    check(lib.lg_batchify_edge_index(ptr(ei), E, int(num_nodes), int(batch_size), ptr(out), stream_of(ei)),
          "lg_batchify_edge_index")
    return out


class SeedSlots:
    """Device-resident dropout seeds for a captured HIP graph (include/leakgnn.h
    LG_SALT_SEED_PTR).  While installed (use_device_seeds), every forward that needs a
    dropout seed takes the next slot and passes its ADDRESS with salt bit 31 set; the
    kernels read the seed at launch.  refresh(), captured at the head of the step, re-draws
    all slots on the device (lg_seed_slots_advance: a device state word advanced per call,
    hashed per slot), so every replay gets new masks with one launch.  The state starts from
    torch's generator (torch.manual_seed reproduces the sequence)."""

    def __init__(self, device, n: int = 16):
        self.buf = torch.zeros(n, dtype=torch.int64, device=device)
        self.state = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(device)
        self.n, self.i = n, 0

    def refresh(self) -> None:
        if self.buf.is_cuda:
            check(load_library().lg_seed_slots_advance(ptr(self.buf), self.n, ptr(self.state), stream_of(self.buf)),
                  "lg_seed_slots_advance")
        else:
            self.buf.random_(0, 2 ** 62)
        self.i = 0

    def take(self) -> int:
        return self.take_tensor().data_ptr()

    def take_tensor(self) -> torch.Tensor:
        """The next slot as a 1-element device tensor (the seed argument of library ops)."""
        if self.i >= self.n:
            raise RuntimeError(f"more than {self.n} dropout seeds in one captured step")
        t = self.buf[self.i:self.i + 1]
        self.i += 1
        return t


_SEED_SLOTS: Optional[SeedSlots] = None


def use_device_seeds(slots: Optional[SeedSlots]) -> None:
    """Install (or, with None, remove) the device seed source of a graph capture
    (library.seed_tensor takes its slots while installed)."""
    global _SEED_SLOTS
    _SEED_SLOTS = slots


def _f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The kernels read fp32: a half/bf16 tensor (model.half(), or an autocast-produced
    activation that reached an op outside its custom_fwd cast) is converted, never
    reinterpreted.  Gradients come back as fp32 and autograd casts them to the input's
    dtype."""
    if t is None or t.dtype == torch.float32:
        return t
    if not t.is_floating_point():
        raise TypeError(f"leakgnn ops take floating-point tensors, got {t.dtype}")
    return t.float()


def _check_d(D: int) -> None:
    if D not in SUPPORTED_D:
        raise NotImplementedError(f"feature width {D} not supported by the HIP kernels (supported: {SUPPORTED_D})")


EDGE_HEAD_SALT = 101    # dropout stream of the EdgeHead hidden layer (trunk layers use salts 0..L)
NOLEAK_HEAD_SALT = 102  # dropout stream of the NoLeakHead hidden layer


def pipe_features(h: torch.Tensor, inc: Incidence) -> torch.Tensor:
    """feat = cat[h_u, h_v, |h_u - h_v|] per pipe (lg_pipe_gather_fwd); no autograd."""
    lib = load_library()
    h = _f32(h).contiguous()
    require_device(h)
    B, N, D = h.shape
    _check_d(D)
    feat = torch.empty(B, inc.num_pipes, 3 * D, device=h.device)
    check(lib.lg_pipe_gather_fwd(ptr(inc.ends), ptr(h), ptr(feat), B, N, inc.num_pipes, D, stream_of(h)),
          "lg_pipe_gather_fwd")
    return feat


def spmm(graph: GCNGraph, x: torch.Tensor, B: int = 1) -> torch.Tensor:
    """y = Ahat x (PyG propagate with gcn_norm weights) for B stacked windows; no autograd."""
    lib = load_library()
    x = _f32(x).contiguous()
    require_device(x)
    D = x.shape[-1]
    _check_d(D)
    y = torch.empty_like(x)
    with _timed("spmm", x.device):
        check(lib.lg_spmm(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(y), B, graph.num_nodes, D,
                          graph.nnz_cap, stream_of(x)), "lg_spmm")
    return y


def wall_ms(fn, iters: int = 10) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters
