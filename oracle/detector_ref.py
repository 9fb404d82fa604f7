"""ORACLE (test infrastructure only) — LeakDetector forward restated on torch CPU.

Restates reference models/detector.py:28-218 step by step over the PyG
restatement in gcn_ref (scatter form) and the graph restatement in graph_ref.
Same state-dict keys as the reference module, so any LeakDetector state dict
loads into it.  Also the CPU baseline that bench.py times ("kind": "port").
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import gcn_ref, graph_ref


class _GRUEncoder(nn.Module):  # detector.py:28-73
    def __init__(self, hidden=64, time_dim=9, use_time=True):
        super().__init__()
        self.use_time = use_time
        self.gru = nn.GRU(1 + (time_dim if use_time else 0), hidden, num_layers=1, batch_first=True)

    def forward(self, r, tfeat):
        B, L, S = r.shape
        rr = r.transpose(1, 2).contiguous().view(B * S, L, 1)                        # :62
        if self.use_time:
            tf = tfeat.unsqueeze(1).repeat(1, S, 1, 1).contiguous().view(B * S, L, -1)  # :66
            rr = torch.cat([rr, tf], dim=-1)                                           # :67
        out, _ = self.gru(rr)                                                          # :71
        return out[:, -1, :].view(B, S, -1)                                            # :72-73


class _MLPHead(nn.Module):  # detector.py:76-102
    def __init__(self, d_in, hidden=128, dropout=0.1):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(d_in, hidden), nn.ReLU(), nn.Dropout(dropout), nn.Linear(hidden, 1))


class LeakDetectorRef(nn.Module):
    def __init__(self, inp_path, sensor_node_ids, pipe_ids_in_order, sensor_hidden=64, node_hidden=64,
                 gnn_layers=2, dropout=0.1, use_time=True, include_links=("PIPES", "PUMPS", "VALVES")):
        super().__init__()
        names, ei, ends = graph_ref.build_graph(inp_path, sensor_node_ids, pipe_ids_in_order, include_links,
                                                add_self_loops=False, make_undirected=True)    # :137-144
        self.node_names = names
        idx = {n: i for i, n in enumerate(names)}
        self.edge_index_single = torch.from_numpy(ei)
        self.pipe_ends = torch.from_numpy(ends)
        self.sensor_node_idx = torch.tensor([idx[n] for n in sensor_node_ids], dtype=torch.long)  # :155
        self.sensor_encoder = _GRUEncoder(sensor_hidden, use_time=use_time)
        self.sensor_to_node = nn.Linear(sensor_hidden + 1, node_hidden)                   # :160
        self.convs = nn.ModuleList([gcn_ref.GCNConvRef(node_hidden, node_hidden) for _ in range(gnn_layers)])
        self.dropout = nn.Dropout(dropout)
        self.edge_head = _MLPHead(3 * node_hidden, 128, dropout)
        self.noleak_head = _MLPHead(node_hidden, 128, dropout)
        self.trace = {}
        # Test hook: ReLU sites ("init", "conv0", "conv1", "edge", "noleak") -> 0/1 mask used
        # instead of the sign of this run's own pre-activation; "absdiff" -> the sign pattern
        # of h_u - h_v for the |h_u - h_v| features (-1 / 0 / 1).  Gradient parity of an fp32
        # path is checked against the fp64 truth on the SAME branch of every ReLU: a unit whose
        # pre-activation sits within fp32 rounding of 0 may land on either side.  The
        # pre-activations of every site are kept in trace["pre_<site>"].
        self.relu_masks = {}

    def _abs(self, site, d):  # |d|, or d * (the given sign pattern): abs has a kink at 0 too
        self.trace[f"pre_{site}"] = d
        sg = self.relu_masks.get(site)
        return d.abs() if sg is None else d * sg.to(d.dtype).to(d.device).reshape(d.shape)

    def _relu(self, site, z):
        self.trace[f"pre_{site}"] = z
        m = self.relu_masks.get(site)
        return F.relu(z) if m is None else z * m.to(z.dtype).to(z.device).reshape(z.shape)

    def forward(self, residual, tfeat=None):
        B, L, S = residual.shape
        N = len(self.node_names)
        h_s = self.sensor_encoder(residual, tfeat)                                      # :176
        dev = residual.device
        h0 = torch.zeros(B, N, h_s.shape[-1], dtype=residual.dtype, device=dev)         # :179
        idx = self.sensor_node_idx.to(dev)
        h0[:, idx, :] = h_s                                                             # :181
        mask = torch.zeros(N, 1, dtype=residual.dtype, device=dev)
        mask[idx, 0] = 1.0                                                              # :184-186
        h = torch.cat([h0, mask.unsqueeze(0).expand(B, -1, -1)], dim=-1)                # :188
        h = self.dropout(self._relu("init", self.sensor_to_node(h)))                     # :189-190
        self.trace["node_init"] = h
        x = h.reshape(B * N, -1)                                                        # :193
        ei = torch.from_numpy(graph_ref.batchify(self.edge_index_single.numpy(), N, B))  # :195-196
        for i, conv in enumerate(self.convs):                                            # :198-201
            x = self.dropout(self._relu(f"conv{i}", conv(x, ei)))
            self.trace[f"conv{i}"] = x
        h_nodes = x.view(B, N, -1)                                                      # :204
        u, v = self.pipe_ends[:, 0].to(dev), self.pipe_ends[:, 1].to(dev)               # :206-208
        h_u, h_v = h_nodes[:, u, :], h_nodes[:, v, :]                                   # :209-210
        feat = torch.cat([h_u, h_v, self._abs("absdiff", h_u - h_v)], dim=-1)             # :87
        mlp = self.edge_head.mlp                                                         # :88, 211
        pipe_logits = mlp[3](mlp[2](self._relu("edge", mlp[0](feat)))).squeeze(-1)
        batch = torch.arange(B, device=dev).repeat_interleave(N)                        # :214
        pooled = gcn_ref.global_mean_pool(x, batch, size=B)                              # :215
        nmlp = self.noleak_head.mlp                                                      # :216
        noleak = nmlp[3](nmlp[2](self._relu("noleak", nmlp[0](pooled)))).squeeze(-1).unsqueeze(-1)
        return torch.cat([pipe_logits, noleak], dim=-1)                                  # :218
