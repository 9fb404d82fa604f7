"""Autograd-level operators over libleakgnn (HIP kernels for gfx950).

Graph state lives on the device once per graph:
  * ``GCNGraph``   - gcn_norm'ed CSR keyed by destination and its transpose
                     (lg_graph_build; replaces PyG gcn_norm, recomputed per call in
                     the reference because GCNConv is built with cached=False,
                     detector.py:163,199).
  * ``Incidence``  - pipe-endpoint incidence CSR (lg_incidence_build) for the
                     deterministic backward of the EdgeHead gathers (detector.py:206-210).

Autograd functions:
  * ``GCNLayerFn``    - one GCNConv (lin -> propagate -> +bias), PyG semantics.
  * ``GNNTrunkFn``    - LeakDetector node init + all conv/relu/dropout layers
                        (detector.py:178-201) as one fused forward / backward chain.
  * ``HeadsFn``       - fused EdgeHead over every pipe + per-window mean pool
                        (detector.py:76-88, 206-215); backward ends in one
                        deterministic incidence reduce.
  * ``GRUEncoderFn``  - SharedSensorGRUEncoder's GRU (detector.py:28-73).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

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


def use_node_major(B: int, N: int, D: int) -> bool:
    """Trunk layout for a batch: node-major when a 16-window tile is mostly full (B >= 16)
    and the activation fits one node-major launch; window-major otherwise (B = 1 graphs
    such as C5, where a node-major tile would carry 1 window in 16)."""
    return TRUNK_NODE_MAJOR and B >= 16 and N * B * D * 4 <= NM_MAX_BYTES


# lg_gcn_fwd_nm schedule / transform bits (LG_F_F32_MFMA, LG_F_LAB_*; include/leakgnn.h) for A/B
# timing of the trunk; the schedule bits never change results.
GCN_FWD_NM_EXTRA_FLAGS = int(os.environ.get("LEAKGNN_GCN_FWD_NM_FLAGS", "0"), 0)


# ----------------------------------------------------------------------------- timing hook
class KernelTimer:
    """Optional HIP-event bracketing of named kernel launches (used by bench.py).

    Events are recorded on the stream the kernel is enqueued on (torch's current
    stream), so elapsed times are the device-side durations of those launches.
    """

    def __init__(self, names: Sequence[str]):
        self.names = set(names)
        self.events: dict = {n: [] for n in names}
        self.enabled = False

    def wrap(self, name: str, device: torch.device):
        timer = self

        class _Ctx:
            def __enter__(self_inner):
                if timer.enabled and name in timer.names:
                    s = torch.cuda.current_stream(device)
                    self_inner.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    self_inner.ev[0].record(s)
                else:
                    self_inner.ev = None
                return self_inner

            def __exit__(self_inner, *exc):
                if self_inner.ev is not None:
                    self_inner.ev[1].record(torch.cuda.current_stream(device))
                    timer.events[name].append(self_inner.ev)
                return False

        return _Ctx()

    def mean_ms(self, name: str) -> Optional[float]:
        evs = self.events.get(name, [])
        if not evs:
            return None
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in evs) / len(evs)

    def count(self, name: str) -> int:
        return len(self.events.get(name, []))

    def reset(self) -> None:
        for n in self.events:
            self.events[n] = []


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
    nodetab: Optional[torch.Tensor] = None    # int32 (N, 16): node-major kernels' per-node record
    nodetab_t: Optional[torch.Tensor] = None  # same for the transposed CSR


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
                                 ptr(g.col), ptr(g.w), ptr(g.rowptr_t), ptr(g.col_t), ptr(g.w_t), ptr(ws),
                                 stream_of(ei)), "lg_graph_build")
        g._keepalive = (ei, ws)  # freed after the stream consumes them
        g.pairs = torch.stack([g.col, g.w.view(torch.int32)], dim=1).contiguous()
        g.pairs_t = torch.stack([g.col_t, g.w_t.view(torch.int32)], dim=1).contiguous()
        g.nodetab = torch.empty(N, 16, **i32)
        g.nodetab_t = torch.empty(N, 16, **i32)
        check(lib.lg_nm_table_build(ptr(g.rowptr), ptr(g.pairs), N, ptr(g.nodetab), stream_of(ei)), "lg_nm_table_build")
        check(lib.lg_nm_table_build(ptr(g.rowptr_t), ptr(g.pairs_t), N, ptr(g.nodetab_t), stream_of(ei)),
              "lg_nm_table_build")
        return g


@dataclass
class Incidence:
    num_nodes: int
    num_pipes: int
    ends: torch.Tensor      # int64 (P, 2) device
    rowptr: torch.Tensor    # int32 (N+1,)
    item: torch.Tensor      # int32 (2P,)

    @staticmethod
    def build(pipe_ends: torch.Tensor, num_nodes: int, device: torch.device) -> "Incidence":
        lib = load_library()
        ends = pipe_ends.to(device=device, dtype=torch.long).contiguous()
        P, N = int(ends.size(0)), int(num_nodes)
        if P and not pipe_ends.is_cuda:
            lo, hi = int(pipe_ends.min()), int(pipe_ends.max())
            if lo < 0 or hi >= N:
                raise IndexError(f"pipe_ends values must lie in [0, {N}), got [{lo}, {hi}]")
        inc = Incidence(N, P, ends, torch.empty(N + 1, device=device, dtype=torch.int32),
                        torch.empty(max(2 * P, 1), device=device, dtype=torch.int32))
        ws = torch.empty(int(lib.lg_incidence_workspace_bytes(P, N)), device=device, dtype=torch.uint8)
        check(lib.lg_incidence_build(ptr(ends), P, N, ptr(inc.rowptr), ptr(inc.item), ptr(ws), stream_of(ends)),
              "lg_incidence_build")
        inc._keepalive = ws
        return inc


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
    all slots from torch's CUDA generator (graph-safe), so every replay gets new masks."""

    def __init__(self, device, n: int = 16):
        self.buf = torch.zeros(n, dtype=torch.int64, device=device)
        self.n, self.i = n, 0

    def refresh(self) -> None:
        self.buf.random_(0, 2 ** 62)
        self.i = 0

    def take(self) -> int:
        if self.i >= self.n:
            raise RuntimeError(f"more than {self.n} dropout seeds in one captured step")
        addr = self.buf.data_ptr() + 8 * self.i
        self.i += 1
        return addr


_SEED_SLOTS: Optional[SeedSlots] = None


def use_device_seeds(slots: Optional[SeedSlots]) -> None:
    """Install (or, with None, remove) the device seed source of a graph capture."""
    global _SEED_SLOTS
    _SEED_SLOTS = slots


def _new_seed(device: torch.device) -> tuple:
    """(seed, salt bits, keep-alive) of one dropout call site.

    Eager: drawn from torch's CPU generator (reproducible under torch.manual_seed, no
    device sync), salt bits 0.  Under use_device_seeds: a device seed slot's address and
    LG_SALT_SEED_PTR.  Inside any other stream capture (a plain torch.cuda.graph or
    torch.compile's cudagraphs) a host integer would be frozen into the graph and every
    replay would reuse the same masks, so the seed is drawn on the device by torch's
    graph-safe CUDA generator (a fresh draw per replay) and passed by address; the
    returned tensor must stay referenced until the kernel has been enqueued."""
    if _SEED_SLOTS is not None:
        return _SEED_SLOTS.take(), nat.LG_SALT_SEED_PTR, None
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        t = torch.randint(0, 2 ** 62, (1,), dtype=torch.long, device=device)
        return t.data_ptr(), nat.LG_SALT_SEED_PTR, t
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item()), 0, None


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


# autocast: every op runs its fp32 kernels; floating inputs are cast to fp32 on entry
_fwd32 = torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
_bwd32 = torch.amp.custom_bwd(device_type="cuda")


def _check_d(D: int) -> None:
    if D not in SUPPORTED_D:
        raise NotImplementedError(f"feature width {D} not supported by the HIP kernels (supported: {SUPPORTED_D})")


# ----------------------------------------------------------------------------- GCNConv
class GCNLayerFn(torch.autograd.Function):
    """y = Ahat (x W^T) + b for one graph (B=1 view of the kernels)."""

    @staticmethod
    @_fwd32
    def forward(ctx, x, weight, bias, graph: GCNGraph):
        lib = load_library()
        x = _f32(x).contiguous()
        weight = _f32(weight).contiguous()
        bias = _f32(bias)
        require_device(x, weight, bias)
        Ntot, D = x.shape
        _check_d(D)
        if weight.shape != (D, D):
            raise NotImplementedError("GCNConv kernels need in_channels == out_channels")
        y = torch.empty_like(x)
        flags = nat.LG_F_BIAS if bias is not None else 0
        with _timed("gcn_fwd", x.device):
            check(lib.lg_gcn_fwd(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(weight), ptr(bias),
                                 ptr(y), 1, Ntot, D, graph.nnz_cap, flags, 0.0, 0, 0, stream_of(x)), "lg_gcn_fwd")
        ctx.graph = graph
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    @_bwd32
    def backward(ctx, dy):
        lib = load_library()
        x, weight = ctx.saved_tensors
        g = ctx.graph
        dy = _f32(dy).contiguous()
        Ntot, D = x.shape
        dx = torch.empty_like(x)
        dW = torch.empty_like(weight)
        db = torch.empty(D, device=x.device, dtype=x.dtype)
        ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=x.device, dtype=torch.uint8)
        with _timed("gcn_bwd", x.device):
            check(lib.lg_gcn_bwd(ptr(g.rowptr_t), ptr(g.col_t), ptr(g.w_t), ptr(dy), None, ptr(x), ptr(weight),
                                 ptr(dx), ptr(dW), ptr(db), None, None, 1, Ntot, D, g.nnz_cap, 0, 1.0, 1.0, ptr(ws),
                                 stream_of(x)),
                  "lg_gcn_bwd")
        return dx, dW, (db if ctx.has_bias else None), None


# ----------------------------------------------------------------------------- detector trunk
@dataclass
class TrunkConfig:
    graph: GCNGraph
    sensor_slot: torch.Tensor      # int32 (N,), -1 for non-sensor nodes
    sensor_idx: torch.Tensor       # int64 (S,): node row of sensor slot s
    slot_live: Optional[torch.Tensor]  # float (S,) 1 where slot s owns its node (None: all unique)
    nonsensor_idx: torch.Tensor    # int64 (N - #sensors,)
    dropout_p: float
    training: bool
    capture: Optional[list] = None     # tests: receives the saved activations x_0 .. x_L, as (B, N, D)
    node_major: bool = False           # True: node features [N][B][D] (see TRUNK_NODE_MAJOR)


class SensorProjFn(torch.autograd.Function):
    """sensor_to_node on the rows that carry a sensor (detector.py:160, 184-189): their
    Linear input is [h_s, 1], so proj = h_s W[:, :Ds]^T + (W[:, Ds] + b) — one addmm.
    Backward: dh_s = dproj W[:, :Ds] (torch mm); dW (incl. the mask column) and db in one
    split-K MFMA kernel (lg_linear_dw) instead of autograd's skinny-K (K = B*S) mm."""

    @staticmethod
    @_fwd32
    def forward(ctx, h_s, W, b):
        h_s, W, b = _f32(h_s), _f32(W), _f32(b)
        B, S, Ds = h_s.shape
        D = W.shape[0]
        h2 = h_s.reshape(B * S, Ds).contiguous()
        proj = torch.addmm(W[:, Ds] + b, h2, W[:, :Ds].t()).view(B, S, D)
        ctx.save_for_backward(h2, W)
        ctx.shape = (B, S)
        return proj

    @staticmethod
    @_bwd32
    def backward(ctx, dproj):
        lib = load_library()
        h2, W = ctx.saved_tensors
        dproj = _f32(dproj)
        B, S = ctx.shape
        K, Ds = h2.shape
        D = W.shape[0]
        d2 = dproj.reshape(K, D).contiguous()
        dh = (d2 @ W[:, :Ds]).view(B, S, Ds) if ctx.needs_input_grad[0] else None
        dW = torch.empty(D, Ds + 1, device=d2.device, dtype=torch.float32)
        db = torch.empty(D, device=d2.device, dtype=torch.float32)
        ws = torch.empty(int(lib.lg_linear_dw_workspace_bytes(K, D, Ds)), device=d2.device, dtype=torch.uint8)
        with _timed("linear_dw", d2.device):
            check(lib.lg_linear_dw(ptr(d2), ptr(h2), K, D, Ds, ptr(dW), ptr(db), ptr(ws), stream_of(d2)),
                  "lg_linear_dw")
        return dh, dW, db


class GNNTrunkFn(torch.autograd.Function):
    """Node init (detector.py:178-190) + L x [GCNConv, ReLU, Dropout] (detector.py:198-201).

    Forward:  x0 = dropout(relu(slot>=0 ? proj[b, slot] : node_bias))        (lg_node_init_fwd)
              x_{l+1} = dropout(relu(Ahat x_l W_l^T + b_l))                   (lg_gcn_fwd, fused)
    Backward: one lg_gcn_bwd per layer; the ReLU/dropout masks of a layer's
              output and of its input are applied inside the kernel, read back
              from the saved activations ([x > 0]), so no mask is stored.
    cfg.node_major: the same chain on [N][B][D] features (lg_gcn_fwd_nm / lg_gcn_bwd_nm);
    the output is then (N, B, D).
    """

    @staticmethod
    @_fwd32
    def forward(ctx, cfg: TrunkConfig, proj, node_bias, *wb):
        lib = load_library()
        proj = _f32(proj).contiguous()
        node_bias = _f32(node_bias)
        wb = tuple(_f32(t) for t in wb)
        require_device(proj, node_bias)
        B, S, D = proj.shape
        _check_d(D)
        N = cfg.graph.num_nodes
        L = len(wb) // 2
        drop = cfg.training and cfg.dropout_p > 0.0
        p = float(cfg.dropout_p) if drop else 0.0
        seed, sbit, seed_keep = _new_seed(proj.device) if drop else (0, 0, None)
        dflag = nat.LG_F_DROPOUT if drop else 0
        nm = bool(cfg.node_major)
        st = stream_of(proj)
        x0 = torch.empty((N, B, D) if nm else (B, N, D), device=proj.device, dtype=torch.float32)
        with _timed("node_init", proj.device):
            check(lib.lg_node_init_fwd(ptr(cfg.sensor_slot), ptr(proj), ptr(node_bias.contiguous()), ptr(x0), B, N,
                                       S, D, dflag | (nat.LG_F_NODE_MAJOR if nm else 0), p, seed, 0 | sbit, st),
                  "lg_node_init_fwd")
        xs = [x0]
        g = cfg.graph
        for l in range(L):
            W, b = wb[2 * l].contiguous(), wb[2 * l + 1].contiguous()
            require_device(W, b)
            y = torch.empty_like(x0)
            flags = nat.LG_F_BIAS | nat.LG_F_RELU | dflag
            with _timed("gcn_fwd", proj.device):
                if nm:
                    check(lib.lg_gcn_fwd_nm(ptr(g.nodetab), ptr(g.pairs), ptr(xs[-1]), ptr(W), ptr(b), ptr(y), B, N, D,
                                            g.nnz_cap, flags | GCN_FWD_NM_EXTRA_FLAGS, p, seed, (l + 1) | sbit, st),
                          "lg_gcn_fwd_nm")
                else:
                    check(lib.lg_gcn_fwd(ptr(g.rowptr), ptr(g.col), ptr(g.w), ptr(xs[-1]), ptr(W), ptr(b), ptr(y), B,
                                         N, D, g.nnz_cap, flags, p, seed, (l + 1) | sbit, st), "lg_gcn_fwd")
            xs.append(y)
        if cfg.capture is not None:
            cfg.capture.extend((t.transpose(0, 1) if nm else t).detach().clone() for t in xs)
        ctx.cfg = cfg
        ctx.seed_keep = seed_keep
        ctx.scale = 1.0 / (1.0 - p) if drop else 1.0
        ctx.dims = (B, S, N, D, L)
        ctx.save_for_backward(*xs, *[t.contiguous() for t in wb[0::2]])
        return xs[-1]

    @staticmethod
    @_bwd32
    def backward(ctx, grad_out):
        lib = load_library()
        cfg = ctx.cfg
        grad_out = _f32(grad_out)
        B, S, N, D, L = ctx.dims
        saved = ctx.saved_tensors
        xs, Ws = saved[:L + 1], saved[L + 1:]
        g = cfg.graph
        st = stream_of(xs[0])
        dy = grad_out.contiguous()
        nm = bool(cfg.node_major)
        wsb = lib.lg_gcn_bwd_nm_workspace_bytes(D) if nm else lib.lg_gcn_bwd_workspace_bytes(D)
        ws = torch.empty(int(wsb), device=dy.device, dtype=torch.uint8)
        grads_wb: List[Optional[torch.Tensor]] = [None] * (2 * L)
        dbias = torch.empty(D, device=dy.device, dtype=torch.float32)
        for l in range(L - 1, -1, -1):
            flags = nat.LG_F_MASK_OUT | (nat.LG_F_MASK_IN if l == L - 1 else 0)
            dx = torch.empty_like(dy)
            dW = torch.empty(D, D, device=dy.device, dtype=torch.float32)
            db = torch.empty(D, device=dy.device, dtype=torch.float32)
            first = l == 0  # layer 0's dx is the node-init gradient: its bias rows are summed in-kernel
            slot_p, dbias_p = (ptr(cfg.sensor_slot), ptr(dbias)) if first else (None, None)
            with _timed("gcn_bwd" if l == L - 1 else f"gcn_bwd_l{l}", dy.device):
                if nm:
                    check(lib.lg_gcn_bwd_nm(ptr(g.nodetab_t), ptr(g.pairs_t), ptr(dy), ptr(xs[l + 1]), ptr(xs[l]),
                                            ptr(Ws[l]), ptr(dx), ptr(dW), ptr(db), slot_p, dbias_p, B, N, D, flags,
                                            ctx.scale, ctx.scale, ptr(ws), st), "lg_gcn_bwd_nm")
                else:
                    check(lib.lg_gcn_bwd(ptr(g.rowptr_t), ptr(g.col_t), ptr(g.w_t), ptr(dy), ptr(xs[l + 1]),
                                         ptr(xs[l]), ptr(Ws[l]), ptr(dx), ptr(dW), ptr(db), slot_p, dbias_p, B, N, D,
                                         g.nnz_cap, flags, ctx.scale, ctx.scale, ptr(ws), st), "lg_gcn_bwd")
            grads_wb[2 * l], grads_wb[2 * l + 1] = dW, db
            dy = dx  # already masked by the previous op's relu/dropout
        if nm:
            dproj = dy.index_select(0, cfg.sensor_idx).transpose(0, 1)
        else:
            dproj = dy.index_select(1, cfg.sensor_idx)
        if cfg.slot_live is not None:
            dproj = dproj * cfg.slot_live.view(1, -1, 1)
        if L == 0:
            dbias = dy.index_select(0 if nm else 1, cfg.nonsensor_idx).sum(dim=(0, 1))
        return (None, dproj, dbias, *grads_wb)


EDGE_HEAD_SALT = 101    # dropout stream of the EdgeHead hidden layer (trunk layers use salts 0..L)
NOLEAK_HEAD_SALT = 102  # dropout stream of the NoLeakHead hidden layer


@dataclass
class HeadsConfig:
    inc: Incidence
    dropout_p: float         # EdgeHead dropout (edge_head.mlp[2].p)
    training: bool
    noleak_p: Optional[float] = None  # NoLeakHead dropout (noleak_head.mlp[2].p); None -> dropout_p
    node_major: bool = False          # h is (N, B, D) (GNNTrunkFn with node_major) instead of (B, N, D)


class HeadsFn(torch.autograd.Function):
    """EdgeHead over every pipe + mean pool + NoLeakHead (detector.py:87-102, 206-216).

    forward:  logits (B, P+1) written in place: columns [0, P) by lg_edge_head_fwd (gather
              -> MFMA MLP -> dot, fused), column P by lg_pool_head_fwd (mean pool +
              NoLeakHead) — the torch.cat of detector.py:216 is never a separate copy.
    backward: lg_edge_head_bwd -> per-pipe endpoint grads; lg_pool_head_bwd -> dpooled and
              the NoLeakHead weight grads; ONE deterministic incidence reduce
              (lg_pipe_scatter_bwd) adds dpooled / N to every node row.
    """

    @staticmethod
    @_fwd32
    def forward(ctx, cfg: HeadsConfig, h, w1, b1, w2, b2, nw1, nb1, nw2, nb2):
        lib = load_library()
        h, w1, b1, w2, b2, nw1, nb1, nw2, nb2 = (_f32(t) for t in (h, w1, b1, w2, b2, nw1, nb1, nw2, nb2))
        h = h.contiguous()
        require_device(h, w1, b1, w2, b2, nw1, nb1, nw2, nb2)
        nm = bool(cfg.node_major)
        N, B, D = h.shape if nm else (h.shape[1], h.shape[0], h.shape[2])
        lay = nat.LG_F_NODE_MAJOR if nm else 0
        _check_d(D)
        hidden, nhidden = w1.shape[0], nw1.shape[0]
        inc = cfg.inc
        P = inc.num_pipes
        pe = float(cfg.dropout_p) if cfg.training else 0.0
        pn = float(cfg.dropout_p if cfg.noleak_p is None else cfg.noleak_p) if cfg.training else 0.0
        seed, sbit, seed_keep = _new_seed(h.device) if (pe > 0.0 or pn > 0.0) else (0, 0, None)
        fe = nat.LG_F_DROPOUT if pe > 0.0 else 0
        fn = nat.LG_F_DROPOUT if pn > 0.0 else 0
        st = stream_of(h)
        logits = torch.empty(B, P + 1, device=h.device, dtype=torch.float32)
        pooled = torch.empty(B, D, device=h.device, dtype=torch.float32)
        hid = torch.empty(B, nhidden, device=h.device, dtype=torch.float32)
        w1c, w2c, nw1c, nw2c = w1.contiguous(), w2.contiguous(), nw1.contiguous(), nw2.contiguous()
        # the EdgeHead hidden layer is kept for the backward (no recompute) when any grad is needed
        keep = any(ctx.needs_input_grad[1:])
        ehid = torch.empty(B * P, hidden, device=h.device, dtype=torch.float32) if keep else None
        with _timed("edge_fwd", h.device):
            check(lib.lg_edge_head_fwd(ptr(inc.ends), ptr(h), ptr(w1c), ptr(b1), ptr(w2c), ptr(b2), ptr(logits),
                                       P + 1, ptr(ehid) if keep else None, B, N, P, D, hidden, fe | lay, pe, seed,
                                       EDGE_HEAD_SALT | sbit, st),
                  "lg_edge_head_fwd")
        with _timed("pool_head", h.device):
            check(lib.lg_pool_head_fwd(ptr(h), ptr(nw1c), ptr(nb1), ptr(nw2c), ptr(nb2), ptr(pooled), ptr(hid),
                                       ptr(logits), P + 1, P, B, N, D, nhidden, fn | lay, pn, seed,
                                       NOLEAK_HEAD_SALT | sbit, st),
                  "lg_pool_head_fwd")
        ctx.cfg, ctx.drop, ctx.seed_keep = cfg, (pe, fe, pn, fn, seed), seed_keep
        ctx.save_for_backward(h, w1c, w2c, ehid, pooled, hid, nw1c, nw2c)
        return logits

    @staticmethod
    @_bwd32
    def backward(ctx, dlogits):
        lib = load_library()
        h, w1, w2, ehid, pooled, hid, nw1, nw2 = ctx.saved_tensors
        pe, fe, pn, fn, seed = ctx.drop
        inc = ctx.cfg.inc
        nm = bool(ctx.cfg.node_major)
        N, B, D = h.shape if nm else (h.shape[1], h.shape[0], h.shape[2])
        lay = nat.LG_F_NODE_MAJOR if nm else 0
        P, hidden, nhidden = inc.num_pipes, w1.shape[0], nw1.shape[0]
        dev = h.device
        st = stream_of(h)
        dl = _f32(dlogits).contiguous()
        dpipe = torch.empty(B, P, 2, D, device=dev)
        dw1, db1 = torch.empty_like(w1), torch.empty(hidden, device=dev)
        dw2, db2 = torch.empty_like(w2), torch.empty(1, device=dev)
        ws = torch.empty(int(lib.lg_edge_head_bwd_workspace_bytes(B, P, D, hidden)), device=dev, dtype=torch.uint8)
        with _timed("edge_bwd", dev):
            check(lib.lg_edge_head_bwd(ptr(inc.ends), ptr(h), ptr(w1), ptr(w2), ptr(ehid), ptr(dl), P + 1, ptr(dpipe),
                                       ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), B, N, P, D, hidden, fe | lay, pe,
                                       ptr(ws), st), "lg_edge_head_bwd")
        dpooled = torch.empty(B, D, device=dev)
        ndw1, ndb1 = torch.empty_like(nw1), torch.empty(nhidden, device=dev)
        ndw2, ndb2 = torch.empty_like(nw2), torch.empty(1, device=dev)
        wsn = torch.empty(int(lib.lg_pool_head_bwd_workspace_bytes(B, D, nhidden)), device=dev, dtype=torch.uint8)
        with _timed("pool_head_bwd", dev):
            check(lib.lg_pool_head_bwd(ptr(pooled), ptr(hid), ptr(nw1), ptr(nw2), ptr(dl), P + 1, P, ptr(dpooled),
                                       ptr(ndw1), ptr(ndb1), ptr(ndw2), ptr(ndb2), B, D, nhidden, fn, pn, ptr(wsn),
                                       st), "lg_pool_head_bwd")
        dh = torch.empty_like(h)
        with _timed("pipe_scatter", dev):
            check(lib.lg_pipe_scatter_bwd(ptr(inc.rowptr), ptr(inc.item), ptr(dpipe), ptr(dpooled), ptr(dh), B, N, P,
                                          D, lay, st), "lg_pipe_scatter_bwd")
        return None, dh, dw1, db1, dw2, db2, ndw1, ndb1, ndw2, ndb2


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


class MeanPoolWindowsFn(torch.autograd.Function):
    """global_mean_pool for B equal windows of N rows (batch = arange(B).repeat_interleave(N))."""

    @staticmethod
    @_fwd32
    def forward(ctx, x, B: int, N: int):
        lib = load_library()
        x = _f32(x).contiguous()
        require_device(x)
        D = x.shape[-1]
        _check_d(D)
        out = torch.empty(B, D, device=x.device, dtype=torch.float32)
        check(lib.lg_mean_pool_fwd(ptr(x), ptr(out), B, N, D, stream_of(x)), "lg_mean_pool_fwd")
        ctx.dims = (B, N)
        return out

    @staticmethod
    @_bwd32
    def backward(ctx, dout):
        B, N = ctx.dims
        return (dout / float(N)).unsqueeze(1).expand(B, N, dout.shape[-1]).reshape(B * N, -1), None, None


class GRUEncoderFn(torch.autograd.Function):
    """SharedSensorGRUEncoder core (detector.py:60-73): h_L of nn.GRU over the B*S sensor
    sequences, x_t = [residual[b, t, s], tfeat[b, t, :]] read in place (lg_gru_fwd / lg_gru_bwd)."""

    @staticmethod
    @_fwd32
    def forward(ctx, residual, tfeat, w_ih, w_hh, b_ih, b_hh):
        lib = load_library()
        residual = _f32(residual).contiguous()
        tfeat = _f32(tfeat).contiguous() if tfeat is not None else None
        w_ih, w_hh, b_ih, b_hh = (_f32(t).contiguous() for t in (w_ih, w_hh, b_ih, b_hh))
        require_device(residual, tfeat, w_ih, w_hh, b_ih, b_hh)
        B, L, S = residual.shape
        G, I = w_ih.shape
        H = w_hh.shape[1]
        if tfeat is not None and tuple(tfeat.shape) != (B, L, 9):
            raise ValueError(f"tfeat must be (B, L, 9), got {tuple(tfeat.shape)}")
        need_bwd = any(ctx.needs_input_grad)
        dev = residual.device
        h_seq = torch.empty(L, B * S, H, device=dev) if need_bwd else None
        gates = torch.empty(L, B * S, 4, H, device=dev) if need_bwd else None
        h_last = torch.empty(B * S, H, device=dev)
        with _timed("gru_fwd", dev):
            check(lib.lg_gru_fwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh), ptr(h_seq),
                                 ptr(gates), ptr(h_last), B, L, S, I, H, stream_of(residual)), "lg_gru_fwd")
        ctx.dims = (B, L, S, I, H)
        ctx.save_for_backward(residual, tfeat, w_ih, w_hh, h_seq, gates)
        return h_last.view(B, S, H)

    @staticmethod
    @_bwd32
    def backward(ctx, dh):
        lib = load_library()
        residual, tfeat, w_ih, w_hh, h_seq, gates = ctx.saved_tensors
        dh = _f32(dh)
        B, L, S, I, H = ctx.dims
        dev = residual.device
        need_dx = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        dx = torch.empty(B * S, L, I, device=dev) if need_dx else None
        dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
        db_ih, db_hh = torch.empty(3 * H, device=dev), torch.empty(3 * H, device=dev)
        ws = torch.empty(int(lib.lg_gru_bwd_workspace_bytes(B, S, I, H)), device=dev, dtype=torch.uint8)
        with _timed("gru_bwd", dev):
            check(lib.lg_gru_bwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(h_seq), ptr(gates),
                                 ptr(dh.contiguous()), ptr(dx), ptr(dw_ih), ptr(dw_hh), ptr(db_ih), ptr(db_hh), B, L,
                                 S, I, H, ptr(ws), stream_of(residual)), "lg_gru_bwd")
        dres = dtf = None
        if ctx.needs_input_grad[0]:
            dres = dx[..., 0].reshape(B, S, L).transpose(1, 2)
        if tfeat is not None and ctx.needs_input_grad[1]:
            dtf = dx[..., 1:].reshape(B, S, L, I - 1).sum(dim=1)
        return dres, dtf, dw_ih, dw_hh, db_ih, db_hh


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
