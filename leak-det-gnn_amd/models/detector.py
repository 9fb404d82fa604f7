"""LeakDetector on MI355X: drop-in for reference models/detector.py.

Same module tree, constructor / forward signatures and state-dict keys as the
reference (detector.py:28-218), so models/train_detector.py, eval/event_evaluator.py
and models/window_evaluator.py use it unchanged:

  sensor_encoder.gru.*              SharedSensorGRUEncoder   (detector.py:28-73)
  sensor_to_node.{weight,bias}      node init Linear(65, 64)  (detector.py:160, 184-190)
  convs.{i}.lin.weight, convs.{i}.bias   GCNConv               (detector.py:162-164)
  edge_head.mlp.{0,3}.*             EdgeHead                  (detector.py:76-88)
  noleak_head.mlp.{0,3}.*           NoLeakHead                (detector.py:91-102)

What runs where (forward + backward): everything on libleakgnn HIP kernels behind the
registered ops of models/library.py (leakgnn::encoder_trunk / gru_encoder / sensor_proj /
gnn_trunk / detector_heads) and models/loss.py (leakgnn::cross_entropy):
  * the GRU sensor encoder with the node init (sensor projection, mask column, ReLU,
    dropout) fused into its epilogue, and the projection's backward into the GRU backward;
  * every GCNConv + ReLU + dropout on the node-major trunk kernels over ONE device-resident
    single-graph CSR (the (2, B*E) batchified edge_index of the reference,
    detector.py:195-196, is never built);
  * the fused EdgeHead (endpoint gather -> MLP -> logit, the (B, P, 3D) features never
    materialised), the per-window mean pool with the NoLeakHead MLP, and their backward
    with the node scatter streamed per tile;
  * the loss (CrossEntropyLoss) and, in the training scripts, clip_grad_norm_ + AdamW
    (models/optim.py).
There is no CPU path: forward raises on CPU tensors.
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import library, ops
from .gcn import GCNConv, global_mean_pool  # noqa: F401  (re-exported PyG-compatible API)
from .utils import WDNGraph, build_wdn_graph_from_inp


class SharedSensorGRUEncoder(nn.Module):
    """One GRU shared by all sensors: (B, L, S) residuals (+ (B, L, 9) time features) -> (B, S, d)."""

    def __init__(self, time_dim: int = 9, hidden_size: int = 64, num_layers: int = 1, dropout: float = 0.0,
                 use_time: bool = True) -> None:
        super().__init__()
        self.use_time = bool(use_time)
        self.hidden_size = int(hidden_size)
        self.gru = nn.GRU(input_size=1 + (time_dim if self.use_time else 0), hidden_size=self.hidden_size,
                          num_layers=num_layers, batch_first=True, dropout=dropout if num_layers > 1 else 0.0)

    def forward(self, r: torch.Tensor, tfeat: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(B, L, S) residuals (+ (B, L, 9) time features) -> (B, S, hidden): h_L of the shared GRU
        over the B*S sensor sequences, on the fused HIP GRU (lg_gru_fwd / lg_gru_bwd)."""
        if self.use_time and tfeat is None:
            raise ValueError("tfeat required when use_time=True")
        if not r.is_cuda:
            raise RuntimeError("SharedSensorGRUEncoder runs on a ROCm GPU only (libleakgnn has no CPU path)")
        g = self.gru
        if g.num_layers != 1 or not 1 <= g.hidden_size <= 1024 or g.bidirectional or not g.bias:
            raise NotImplementedError("the HIP GRU kernels cover the reference encoder: 1 layer, hidden 1..1024 "
                                      "(32 / 64 tiled, others generic), bias")
        f = ops._f32
        ws = [f(t) for t in (g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0)]
        # contiguous once here: a strided tfeat (a slice of a longer segment) would otherwise be
        # saved as is and copied again in the backward
        tf = f(tfeat).contiguous() if self.use_time else None
        r = f(r)
        save = torch.is_grad_enabled() and any(t.requires_grad for t in [r, *ws] + ([tf] if tf is not None else []))
        return torch.ops.leakgnn.gru_encoder(r, tf, *ws, save)[0]


class EdgeHead(nn.Module):
    def __init__(self, node_dim: int, hidden_dim: int = 128, dropout: float = 0.1) -> None:
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(node_dim * 3, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, 1))

    def forward(self, h_u: torch.Tensor, h_v: torch.Tensor) -> torch.Tensor:
        return self.forward_feat(torch.cat([h_u, h_v, (h_u - h_v).abs()], dim=-1))

    def forward_feat(self, feat: torch.Tensor) -> torch.Tensor:
        """feat = cat[h_u, h_v, |h_u - h_v|] already built (by lg_pipe_gather_fwd)."""
        return self.mlp(feat).squeeze(-1)


class NoLeakHead(nn.Module):
    def __init__(self, node_dim: int, hidden_dim: int = 128, dropout: float = 0.1) -> None:
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(node_dim, hidden_dim), nn.ReLU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, 1))

    def forward(self, pooled: torch.Tensor) -> torch.Tensor:
        return self.mlp(pooled).squeeze(-1)


def _batchify_edge_index(edge_index_single: torch.Tensor, num_nodes: int, batch_size: int) -> torch.Tensor:
    """(2, E) -> (2, E*B) disjoint union, column b*E + e = edge e offset by b*N (detector.py:105-114).
    Runs on the device (lg_batchify_edge_index); bit-exact."""
    return ops.batchify_edge_index(edge_index_single, num_nodes, batch_size)


class LeakDetector(nn.Module):
    """residual (B, L_det, S), tfeat (B, L_det, 9) -> logits (B, num_pipes + 1); class P = no leak."""

    def __init__(self, inp_path: str | Path, sensor_node_ids: Sequence[str], pipe_ids_in_order: Sequence[str],
                 sensor_hidden: int = 64, node_hidden: int = 64, gnn_layers: int = 2, dropout: float = 0.1,
                 use_time: bool = True, include_links: Sequence[str] = ("PIPES", "PUMPS", "VALVES"),
                 mlp_dtype: str = "fp32") -> None:
        super().__init__()
        if mlp_dtype not in ("fp32", "bf16"):
            raise ValueError(f"mlp_dtype must be 'fp32' or 'bf16', got {mlp_dtype!r}")
        # "bf16": BASELINE configs[2]'s tier — the GCN transforms and the EdgeHead MLP as one
        # bf16 MFMA product with fp32 accumulate (LG_F_BF16); activations stay fp32.  Not an
        # fp32-parity mode (2e-2 relative on logits).  Not a state-dict entry.
        self.mlp_dtype = mlp_dtype
        self.graph: WDNGraph = build_wdn_graph_from_inp(inp_path=inp_path, sensor_node_ids=sensor_node_ids,
                                                        pipe_ids_in_order=pipe_ids_in_order,
                                                        include_links=include_links, add_self_loops=False,
                                                        make_undirected=True)
        self.node_names = self.graph.node_names
        self.node_to_idx = self.graph.node_to_idx
        self.pipe_ids = self.graph.pipe_ids
        self.pipe_to_idx = self.graph.pipe_to_idx
        self.pipe_ends = torch.tensor(self.graph.pipe_ends, dtype=torch.long)
        self.edge_index_single = self.graph.edge_index
        self.sensor_node_ids = list(sensor_node_ids)
        self.sensor_node_idx = torch.tensor([self.node_to_idx[n] for n in self.sensor_node_ids], dtype=torch.long)

        self.sensor_encoder = SharedSensorGRUEncoder(hidden_size=sensor_hidden, use_time=use_time)
        self.sensor_to_node = nn.Linear(sensor_hidden + 1, node_hidden)
        self.convs = nn.ModuleList(
            [GCNConv(node_hidden, node_hidden, add_self_loops=True, normalize=True) for _ in range(gnn_layers)])
        self.dropout = nn.Dropout(dropout)
        self.edge_head = EdgeHead(node_hidden, hidden_dim=128, dropout=dropout)
        self.noleak_head = NoLeakHead(node_hidden, hidden_dim=128, dropout=dropout)
        self._dev_state: Dict[torch.device, tuple] = {}
        # Test hook: a dict here receives the step's ReLU outputs as the kernels produced them
        # ("xs": node init + every GCN layer, "edge_hidden", "noleak_hidden"), so parity tests
        # can evaluate the fp64 truth on the same side of every ReLU kink.  None: nothing kept.
        self.capture: Optional[dict] = None
        # graph_step.CapturedTrainStep at world > 1: forward keeps the trunk output (the heads'
        # input) as `boundary` while keep_boundary is set, so the backward can stop there and
        # the heads' gradient all-reduce overlaps the trunk backward (overlap_split)
        self.keep_boundary = False
        # node-major trunk: keep the node init compressed (sensor rows + [x0 > 0] bits,
        # lg_node_init_bits_fwd) instead of materialising x_0 (43 MB at B = 256)
        self.compress_x0 = True
        # EdgeHead backward node sums: True = streamed per tile through the pipe schedule (each
        # node's incidences summed in schedule order); False = the reference's order (items
        # ascending, as index_add over pipe ids), per-window scatter.  Read when the device
        # state is first built.
        self.incidence_schedule = True
        # node-major training: the GRU encoder, node init and GCN layers as one op
        # (library.encoder_trunk: the node init formed in the GRU's epilogue, the projection's
        # backward in the GRU backward's); False: the encoder module, then library.gnn_trunk
        self.fuse_encoder = True
        self.boundary: Optional[torch.Tensor] = None
        self._batched_edges: Dict[tuple, torch.Tensor] = {}  # (B, device) -> (2, B*E): the general path's edge_index

    def overlap_split(self):
        """Parameters whose gradients are final once the backward reaches `boundary` (the
        heads: EdgeHead + NoLeakHead, detector.py:206-218 of the reference)."""
        return list(self.edge_head.parameters()) + list(self.noleak_head.parameters())

    # -- device-resident graph state (built once per device; not part of state_dict)
    def _device_state(self, device: torch.device):
        st = self._dev_state.get(device)
        if st is None:
            N = len(self.node_names)
            graph = ops.GCNGraph.build(self.edge_index_single, N, device, add_self_loops=True, normalize=True)
            inc = ops.Incidence.build(self.pipe_ends, N, device, schedule=self.incidence_schedule)
            slot = torch.full((N,), -1, dtype=torch.int32)
            for s, n in enumerate(self.sensor_node_idx.tolist()):
                slot[n] = s  # duplicate sensor ids: last write wins, as h0[:, idx] = h_s does
            live = torch.tensor([float(slot[n] == s) for s, n in enumerate(self.sensor_node_idx.tolist())])
            nonsensor = torch.nonzero(slot < 0).flatten()
            graph.x0marks = None  # built on the first node-major forward that compresses x_0 (_x0marks)
            st = (graph, inc, slot.to(device), self.sensor_node_idx.to(device),
                  None if bool(live.all()) else live.to(device), nonsensor.to(device))
            self._dev_state[device] = st
        return st

    def _x0marks(self, graph, slot: torch.Tensor):
        """The compressed layer-0 input's sensor-marked node tables (lg_nm_table_sensor_mark),
        built once per device on the first forward that uses them (window-major batches never
        do).  Its launches must run eagerly, not be recorded into a graph being captured."""
        if graph.x0marks is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("LeakDetector: run one eager node-major forward before capturing a graph "
                                   "(the compressed node init's tables are built on first use)")
            graph.x0marks = ops.SensorMarks.build(graph, slot)
        return graph.x0marks

    def _fused_encoder(self, residual: torch.Tensor, tfeat: Optional[torch.Tensor], B: int, N: int, D: int,
                       nm: bool) -> bool:
        """Whether this forward runs the encoder, node init and layers as ONE op
        (library.encoder_trunk): the node-major trunk with the compressed node init, the
        reference encoder (1 layer, bias) with node_hidden == sensor_hidden, and residual /
        tfeat as data (no gradient wanted for them: the fused backward forms no dx)."""
        g = self.sensor_encoder.gru
        if not (self.fuse_encoder and g.num_layers == 1 and g.bias and not g.bidirectional):
            return False
        if self.capture is not None:  # the capture reads h_s, which the fused op never forms
            return False
        if residual.requires_grad or (tfeat is not None and self.sensor_encoder.use_time and tfeat.requires_grad):
            return False
        return library.encoder_trunk_supported(B, N, g.hidden_size, D, len(self.convs), nm, self.compress_x0)

    def _widths_tiled(self) -> bool:
        """Whether the trunk and heads run the tiled kernels: sensor_hidden == node_hidden in
        {32, 64} (the reference's callers use 64 and 64, train_detector.py:250-254)."""
        return (self.sensor_encoder.hidden_size in ops.SUPPORTED_D
                and self.sensor_to_node.out_features == self.sensor_encoder.hidden_size)

    def _forward_general(self, residual: torch.Tensor, tfeat: Optional[torch.Tensor]) -> torch.Tensor:
        """Any sensor_hidden / node_hidden (detector.py:128-129): the reference's forward
        (:170-218) composed from the width-general pieces — the GRU encoder (lg_gru_fwd's generic
        kernel off 32 / 64), GCNConv's general path (lg_spmm_cols propagate, library GEMM
        transform) over the batchified edge_index, and library GEMMs / device indexing for the
        node init and the heads; dropout from torch's generator (the tiled path's counter RNG
        is a kernel feature).  A generality path: the bench's widths never take it."""
        B, L, S = residual.shape
        dev = residual.device
        graph, inc, slot, sensor_idx, slot_live, nonsensor = self._device_state(dev)
        N = len(self.node_names)
        h_s = self.sensor_encoder(residual, tfeat)                           # (B, S, Ds)
        # h0 rows: [h_s of the node's sensor, 1] for sensor nodes (last duplicate wins, as
        # h0[:, idx] = h_s), zeros for the rest (:178-187)
        has = (slot >= 0).to(h_s.dtype).view(1, N, 1)
        h0 = torch.cat([h_s.index_select(1, slot.clamp(min=0).long()) * has, has.expand(B, N, 1)], dim=-1)
        p = float(self.dropout.p)
        x = F.dropout(F.relu(self.sensor_to_node(h0)), p, self.training).reshape(B * N, -1)
        ei = self._batched_edges.get((B, dev))
        if ei is None:
            ei = _batchify_edge_index(self.edge_index_single.to(dev), N, B)
            self._batched_edges[(B, dev)] = ei
        for conv in self.convs:
            x = F.dropout(F.relu(conv(x, ei)), p, self.training)
        h_nodes = x.view(B, N, -1)
        ends = inc.ends.long()
        pipe_logits = self.edge_head(h_nodes[:, ends[:, 0]], h_nodes[:, ends[:, 1]])     # (B, P)
        pooled = global_mean_pool(x, torch.arange(B, device=dev).repeat_interleave(N), size=B)
        return torch.cat([pipe_logits, self.noleak_head(pooled).unsqueeze(-1)], dim=-1)

    def forward(self, residual: torch.Tensor, tfeat: Optional[torch.Tensor] = None) -> torch.Tensor:
        if not residual.is_cuda:
            raise RuntimeError("LeakDetector runs on a ROCm GPU only (libleakgnn has no CPU path)")
        if not self._widths_tiled():
            return self._forward_general(residual, tfeat)
        B, L, S = residual.shape
        graph, inc, slot, sensor_idx, slot_live, nonsensor = self._device_state(residual.device)
        f = ops._f32
        Wn, bn = f(self.sensor_to_node.weight), f(self.sensor_to_node.bias)  # (D, Ds+1), (D,)
        N, D = len(self.node_names), Wn.shape[0]
        nm = ops.use_node_major(B, N, D, bf16=self.mlp_dtype == "bf16")
        drop = self.training and float(self.dropout.p) > 0.0
        g = graph
        bf16 = self.mlp_dtype == "bf16"
        enc = self.sensor_encoder
        if enc.use_time and tfeat is None:
            raise ValueError("tfeat required when use_time=True")
        if self._fused_encoder(residual, tfeat, B, N, D, nm):
            # encoder + node init + layers as one op (library.encoder_trunk)
            mk = self._x0marks(g, slot)
            gw = [f(t) for t in (enc.gru.weight_ih_l0, enc.gru.weight_hh_l0, enc.gru.bias_ih_l0, enc.gru.bias_hh_l0)]
            cw, cb = [f(c.lin.weight) for c in self.convs], [f(c.bias) for c in self.convs]
            save = torch.is_grad_enabled() and any(t.requires_grad for t in gw + [Wn, bn] + cw + cb)
            tf = f(tfeat).contiguous() if enc.use_time else None
            out_t = torch.ops.leakgnn.encoder_trunk(
                f(residual), tf, *gw, Wn, bn, cw, cb, slot, sensor_idx, slot_live, g.nodetab, g.pairs, g.nodetab_t,
                g.pairs_t, mk.nodetab_s, mk.pairs_s, mk.pos_slot_t, float(self.dropout.p) if drop else 0.0,
                library.seed_tensor(residual.device) if drop else _NO_SEED, save, bf16=bf16)
            nl = len(self.convs)
            xs = [out_t[nl + 1]] + list(out_t[:nl])  # [x_0 (its sensor rows), x_1 .. x_L]
            x0bits = out_t[nl + 2]
        else:
            h_s = self.sensor_encoder(residual, tfeat)                        # (B, S, Ds)
            if self.capture is not None and torch.is_grad_enabled():
                if h_s.requires_grad:
                    h_s.retain_grad()
                self.capture["h_s"] = h_s
            # sensor_to_node (rows with a sensor: [h_s, 1] W^T + b; without: b) folded into node init
            mk = self._x0marks(g, slot) if (nm and self.compress_x0 and len(self.convs) > 1) else None
            out_t = torch.ops.leakgnn.gnn_trunk(
                h_s, Wn, bn, [f(c.lin.weight) for c in self.convs], [f(c.bias) for c in self.convs], slot, sensor_idx,
                nonsensor, slot_live, g.nodetab, g.pairs, g.rowptr, g.col, g.w, g.nodetab_t, g.pairs_t, g.rowptr_t,
                g.col_t, g.w_t, float(self.dropout.p) if drop else 0.0, nm,
                library.seed_tensor(residual.device) if drop else _NO_SEED,
                mk.nodetab_s if mk is not None else None, mk.pairs_s if mk is not None else None,
                mk.pos_slot_t if mk is not None else None, bf16=bf16)
            xs = out_t[:-2]                     # [x_0 .. x_L] (then x_L's mask bits and x_0's, when compressed)
            x0bits = out_t[-1]
        h_nodes = xs[-1]                                                   # (N, B, D) node-major, else (B, N, D)
        if self.keep_boundary:
            self.boundary = h_nodes
        mlp = self.edge_head.mlp     # Linear(3D,128), ReLU, Dropout, Linear(128,1)
        nmlp = self.noleak_head.mlp  # Linear(D,128), ReLU, Dropout, Linear(128,1)
        pe = float(mlp[2].p) if self.training else 0.0
        pn = float(nmlp[2].p) if self.training else 0.0
        hw = [f(t) for t in (mlp[0].weight, mlp[0].bias, mlp[3].weight, mlp[3].bias,
                             nmlp[0].weight, nmlp[0].bias, nmlp[3].weight, nmlp[3].bias)]
        keep = torch.is_grad_enabled() and (h_nodes.requires_grad or any(t.requires_grad for t in hw))
        seed = library.seed_tensor(residual.device) if (pe > 0.0 or pn > 0.0) else _NO_SEED
        # (B, P+1): pipe logits, then the no-leak logit of the mean-pooled window (:206-218)
        sched, sched_hdr = inc.schedule(D)
        out = torch.ops.leakgnn.detector_heads(h_nodes, *hw, inc.ends, inc.rowptr, inc.item, pe, pn, nm, keep, seed,
                                               sched, sched_hdr, bf16=bf16)
        if self.capture is not None:
            if x0bits.numel() > 0:  # x_0 compressed: materialise it for the diagnostics
                xs = [library.expand_x0(xs[0], x0bits, slot, bn, N, float(self.dropout.p) if drop else 0.0)] + xs[1:]
            self.capture.update(xs=xs, node_major=nm, edge_hidden=out[1], noleak_hidden=out[3])
        return out[0]


_NO_SEED = torch.zeros(1, dtype=torch.long)  # seed argument of an op that draws no dropout mask
