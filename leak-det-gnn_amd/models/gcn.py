"""Drop-in for the two PyG operators on the reference hot path.

Reference call sites: detector.py:23 (import), :163 (GCNConv ctor), :199 (forward),
:215 (global_mean_pool).  PyG is absent from the image and unpinned in the
reference; the semantics restated here are PyG 2.x's published ones:

  GCNConv(in, out, improved=False, cached=False, add_self_loops=True,
          normalize=True, bias=True)
     lin = Linear(in, out, bias=False, glorot init)  -> state key ``lin.weight`` [out, in]
     bias = zeros(out)                                -> state key ``bias``
     forward(x, edge_index) = propagate(gcn_norm(edge_index), lin(x)) + bias
  global_mean_pool(x, batch, size=None) = scatter(x, batch, reduce='mean', dim_size=size)

Here forward runs the registered op leakgnn::gcn_conv (models/library.py: one fused HIP
launch of (Ahat x) W^T + b — lg_gcn_fwd_rows, 16-node tiles off the node table, at D = 64;
lg_gcn_fwd at D = 32) and its autograd formula leakgnn::gcn_conv_backward
(lg_gcn_bwd_rows / lg_gcn_bwd).  Other widths (in != out, or not 32 / 64) take the general
path: leakgnn::spmm_cols (lg_spmm_cols, any column count, bias fused) for the propagate and a
library GEMM for the transform, on the narrower side.  The gcn_norm'ed CSR is built on the device
(lg_graph_build) and, unlike PyG with cached=False, re-used while an edge_index
with the SAME CONTENT is passed again — the graph is a pure function of edge_index,
so results are unchanged.  The same tensor object at the same version counter is a
hit with no device work (so a HIP-graph-captured step never syncs); any other tensor
is compared element-wise with a private copy.  Keying on the storage address alone
would reuse a stale CSR when the caching allocator hands a freed edge_index's
address to a different graph of the same shape.
"""
from __future__ import annotations

import math
import weakref
from typing import Optional

import torch
import torch.nn as nn

from . import library  # noqa: F401  (registers the leakgnn:: ops)
from .ops import SUPPORTED_D, GCNGraph, _f32


def _glorot_(t: torch.Tensor) -> None:
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class GCNConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, improved: bool = False, cached: bool = False,
                 add_self_loops: bool = True, normalize: bool = True, bias: bool = True, **kwargs) -> None:
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.improved = improved
        self.cached = cached
        self.add_self_loops = add_self_loops
        self.normalize = normalize
        self.lin = nn.Linear(in_channels, out_channels, bias=False)
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self._graph_key = None
        self._graph_ei: Optional[torch.Tensor] = None  # private copy of the edge_index the CSR was built from
        self._graph: Optional[GCNGraph] = None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        _glorot_(self.lin.weight)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()
        self._graph_key = None
        self._graph_ei = None
        self._graph = None
        self._graph_ref = None
        self._graph_ver = -1

    def graph_for(self, edge_index: torch.Tensor, num_nodes: int, device: torch.device) -> GCNGraph:
        """The cached CSR of `edge_index`.  Fast path (no device sync, capture-safe): the SAME
        tensor object as last time (a weak reference, so a new tensor at a recycled address
        never matches) at the same version counter.  Otherwise the content is compared with
        the cached copy (a sync) and the CSR rebuilt if it differs."""
        key = (tuple(edge_index.shape), edge_index.dtype, int(num_nodes), device)
        ref = self._graph_ref() if self._graph_ref is not None else None
        if (self._graph is not None and self._graph_key == key and ref is edge_index
                and edge_index._version == self._graph_ver):
            return self._graph
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("GCNConv: a new edge_index inside HIP graph capture; run one eager forward with it "
                               "first (the CSR is built and cached outside the capture)")
        ei = edge_index.to(device)
        if (self._graph is None or self._graph_key != key or self._graph_ei is None
                or not torch.equal(self._graph_ei, ei)):
            self._graph = GCNGraph.build(edge_index, num_nodes, device, add_self_loops=self.add_self_loops,
                                         normalize=self.normalize, improved=self.improved)
            self._graph_key = key
            self._graph_ei = ei.clone()
        self._graph_ref = weakref.ref(edge_index)
        self._graph_ver = edge_index._version
        return self._graph

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, edge_weight: Optional[torch.Tensor] = None):
        if edge_weight is not None:
            raise NotImplementedError("edge_weight is not used on the Leak-det-gnn path")
        g = self.graph_for(edge_index, x.size(0), x.device)
        if self.in_channels == self.out_channels and self.in_channels in SUPPORTED_D:
            return torch.ops.leakgnn.gcn_conv(_f32(x), _f32(self.lin.weight), _f32(self.bias), g.rowptr, g.col, g.w,
                                              g.rowptr_t, g.col_t, g.w_t, g.nodetab, g.pairs, g.nodetab_t, g.pairs_t)
        # general widths: propagate on lg_spmm_cols, transform on a library GEMM, on the narrower
        # side (PyG's order, lin then propagate, when the output is not wider than the input)
        x, W, b = _f32(x), _f32(self.lin.weight), _f32(self.bias)
        csr = (g.rowptr, g.col, g.w, g.rowptr_t, g.col_t, g.w_t)
        if self.out_channels <= self.in_channels:
            return torch.ops.leakgnn.spmm_cols(x @ W.t(), b, *csr)
        p = torch.ops.leakgnn.spmm_cols(x, None, *csr)
        return torch.addmm(b, p, W.t()) if b is not None else p @ W.t()

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


_WINDOW_BATCH: dict = {}  # id(batch) -> (weakref, version, B, N or None): its layout, checked once


def _window_layout(batch: torch.Tensor, B: int, rows: int) -> Optional[int]:
    """N when batch == arange(B).repeat_interleave(N) (equal windows, the detector's layout),
    else None.  Decided once per batch tensor (object and version counter, as GCNConv's CSR
    cache): later calls with the same tensor need no device sync."""
    ent = _WINDOW_BATCH.get(id(batch))
    if ent is not None and ent[0]() is batch and ent[1] == batch._version and ent[2] == B:
        return ent[3]
    N = None
    if rows % B == 0 and batch.numel() == rows:
        n = rows // B
        if torch.equal(batch, torch.arange(B, device=batch.device).repeat_interleave(n)):
            N = n
    if len(_WINDOW_BATCH) > 64:
        _WINDOW_BATCH.clear()
    _WINDOW_BATCH[id(batch)] = (weakref.ref(batch), batch._version, B, N)
    return N


def global_mean_pool(x: torch.Tensor, batch: Optional[torch.Tensor], size: Optional[int] = None) -> torch.Tensor:
    """PyG global_mean_pool(x, batch, size): per-graph mean of the rows of x, graph ids in
    `batch` (any order, any sizes; a graph with no rows pools to 0, as PyG's scatter mean).
    Equal windows in order (the detector's batch vector, detector.py:214) at D = 32 / 64 run
    the HIP kernel (lg_mean_pool_fwd); other batches a device scatter-sum and count.  Pass
    ``size`` to skip the max() sync; the layout check syncs once per batch tensor."""
    if not x.is_cuda:
        raise RuntimeError("global_mean_pool runs on a ROCm GPU only (libleakgnn has no CPU path)")
    if batch is None:
        return x.mean(dim=0, keepdim=True)
    B = int(size) if size is not None else int(batch.max().item()) + 1
    if x.size(-1) in SUPPORTED_D and x.dim() == 2:
        N = _window_layout(batch, B, x.size(0))
        if N is not None:
            return torch.ops.leakgnn.mean_pool(_f32(x), B, N)
    idx = batch.to(device=x.device, dtype=torch.long)
    sums = x.new_zeros((B,) + tuple(x.shape[1:])).index_add(0, idx, x)
    cnt = torch.bincount(idx, minlength=B).clamp(min=1).to(x.dtype)
    return sums / cnt.view((B,) + (1,) * (x.dim() - 1))
