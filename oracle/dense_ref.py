"""ORACLE (test infrastructure only) — an INDEPENDENT dense formulation of the PyG ops.

Used (a) as a second anchor for gcn_ref (scatter form) and (b) as the
``torch_geometric.nn`` the reference detector.py is run with when the golden
fixtures are generated (oracle/make_golden.py), because PyG itself is absent.

  GCNConv:  Ahat = D^-1/2 (A + I) D^-1/2 as a dense (N, N) matrix built by
            counting edges (multi-edges add up; existing loops replaced by one
            unit loop), out = Ahat @ (x W^T) + b
  global_mean_pool: one-hot (B, N) matrix / counts, times x
"""
from __future__ import annotations

import torch


def dense_ahat(edge_index: torch.Tensor, num_nodes: int, dtype=torch.float64) -> torch.Tensor:
    A = torch.zeros(num_nodes, num_nodes, dtype=dtype)
    src, dst = edge_index[0].tolist(), edge_index[1].tolist()
    for s, d in zip(src, dst):
        if s != d:
            A[d, s] += 1.0          # message s -> d lands in row d
    A += torch.eye(num_nodes, dtype=dtype)
    deg = A.sum(dim=1)
    dis = torch.where(deg > 0, deg.rsqrt(), torch.zeros_like(deg))
    return dis.view(-1, 1) * A * dis.view(1, -1)


class GCNConv(torch.nn.Module):
    """Dense stand-in with PyG's constructor, state keys and forward signature."""

    def __init__(self, in_channels: int, out_channels: int, add_self_loops: bool = True, normalize: bool = True,
                 bias: bool = True, **_):
        super().__init__()
        assert add_self_loops and normalize
        self.lin = torch.nn.Linear(in_channels, out_channels, bias=False)
        self.bias = torch.nn.Parameter(torch.zeros(out_channels)) if bias else None
        a = (6.0 / (in_channels + out_channels)) ** 0.5
        with torch.no_grad():
            self.lin.weight.uniform_(-a, a)
        self._cache = None

    def forward(self, x, edge_index):
        key = (edge_index.data_ptr(), edge_index.shape, x.size(0))
        if self._cache is None or self._cache[0] != key:
            self._cache = (key, dense_ahat(edge_index, x.size(0), dtype=torch.float64))
        ahat = self._cache[1]
        h = (x @ self.lin.weight.t()).double()
        out = (ahat @ h).to(x.dtype)
        return out + self.bias if self.bias is not None else out


def global_mean_pool(x, batch, size=None):
    B = int(batch.max()) + 1 if size is None else int(size)
    onehot = torch.zeros(B, x.size(0), dtype=x.dtype)
    onehot[batch, torch.arange(x.size(0))] = 1.0
    return (onehot @ x) / onehot.sum(dim=1, keepdim=True).clamp(min=1)
