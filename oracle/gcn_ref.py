"""ORACLE (test infrastructure only) — PyG GCNConv / global_mean_pool on torch CPU.

PyG (torch_geometric) is not installed in the image and the reference does not pin
a version.  This restates the published PyG 2.x algorithm that the
reference calls at detector.py:23 / :163 / :199 / :215:

  gcn_norm (torch_geometric/nn/conv/gcn_conv.py):
      add_remaining_self_loops(edge_index, fill_value=1) ->
      deg = scatter_add(edge_weight, col); dis = deg^-1/2 (inf -> 0);
      edge_weight = dis[row] * edge_weight * dis[col]
  GCNConv.forward: x = lin(x) (no bias); out = propagate(edge_index, x, edge_weight)
      = scatter_add(edge_weight[:, None] * x[row], col); out += bias
  global_mean_pool: scatter(x, batch, dim=0, reduce='mean') = sum / count

Scatter sums are accumulated in ascending edge order (index_add_ on CPU).  The functions
follow the device of their inputs, so the tests can also time the reference arithmetic as
plain torch on the GPU (as an error yardstick, never as the product).
"""
from __future__ import annotations

import torch


def gcn_norm(edge_index: torch.Tensor, num_nodes: int, add_self_loops: bool = True, fill: float = 1.0,
             dtype=torch.float32):
    row, col = edge_index[0], edge_index[1]
    dev = edge_index.device
    w = torch.ones(row.numel(), dtype=dtype, device=dev)
    if add_self_loops:
        keep = row != col
        loops = torch.arange(num_nodes, dtype=torch.long, device=dev)
        row = torch.cat([row[keep], loops])
        col = torch.cat([col[keep], loops])
        w = torch.cat([w[keep], torch.full((num_nodes,), fill, dtype=dtype, device=dev)])
    deg = torch.zeros(num_nodes, dtype=dtype, device=dev).index_add_(0, col, w)
    dis = deg.pow(-0.5)
    dis = dis.masked_fill(torch.isinf(dis), 0.0)
    return row, col, dis[row] * w * dis[col]


def gcn_conv(x: torch.Tensor, edge_index: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None,
             add_self_loops: bool = True, normalize: bool = True) -> torch.Tensor:
    """GCNConv.forward: weight is lin.weight [out, in]."""
    N = x.size(0)
    edge_index = edge_index.to(x.device)
    if normalize:
        row, col, w = gcn_norm(edge_index, N, add_self_loops)
    else:
        row, col = edge_index[0], edge_index[1]
        w = torch.ones(row.numel(), dtype=x.dtype, device=x.device)
    h = x @ weight.t()
    msg = w.view(-1, 1) * h.index_select(0, row)  # PyG message(): edge_weight * x_j (type-promoted)
    out = torch.zeros(N, h.size(1), dtype=msg.dtype, device=x.device).index_add_(0, col, msg)
    if bias is not None:
        out = out + bias
    return out


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor, size: int | None = None) -> torch.Tensor:
    B = int(batch.max()) + 1 if size is None else int(size)
    batch = batch.to(x.device)
    s = torch.zeros(B, x.size(1), dtype=x.dtype, device=x.device).index_add_(0, batch, x)
    cnt = torch.zeros(B, dtype=x.dtype, device=x.device).index_add_(
        0, batch, torch.ones(batch.numel(), dtype=x.dtype, device=x.device))
    return s / cnt.clamp(min=1).view(-1, 1)


class GCNConvRef(torch.nn.Module):
    """Module form with PyG's state-dict keys (lin.weight, bias)."""

    def __init__(self, in_channels: int, out_channels: int, add_self_loops: bool = True, normalize: bool = True,
                 bias: bool = True, **_):
        super().__init__()
        self.add_self_loops, self.normalize = add_self_loops, normalize
        self.lin = torch.nn.Linear(in_channels, out_channels, bias=False)
        self.bias = torch.nn.Parameter(torch.zeros(out_channels)) if bias else None
        a = (6.0 / (in_channels + out_channels)) ** 0.5
        with torch.no_grad():
            self.lin.weight.uniform_(-a, a)

    def forward(self, x, edge_index):
        return gcn_conv(x, edge_index, self.lin.weight, self.bias, self.add_self_loops, self.normalize)
