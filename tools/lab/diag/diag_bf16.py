"""Diagnostic (GPU box): bf16-tier kernels against their fp32 (split) versions on the same
inputs — EdgeHead forward/backward outputs one by one, and the node-major GCN layer."""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[3]
for p in (ROOT, ROOT / "leak-det-gnn_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
from helpers import LTA_INP, lta_ids  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def main():
    from models import library  # noqa: F401
    from models.detector import LeakDetector
    dev = torch.device("cuda:0")
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, sensors, pipes).to(dev).eval()
    graph, inc, slot, sidx, live, nons = m._device_state(dev)
    B, N, D = 256, len(m.node_names), 64
    h = torch.randn(N, B, D, device=dev).relu_()
    mlp, nmlp = m.edge_head.mlp, m.noleak_head.mlp
    hw = [t.detach() for t in (mlp[0].weight, mlp[0].bias, mlp[3].weight, mlp[3].bias, nmlp[0].weight, nmlp[0].bias,
                                nmlp[3].weight, nmlp[3].bias)]
    seed = torch.zeros(1, dtype=torch.long)
    outs = {}
    for bf in (False, True):
        o = torch.ops.leakgnn.detector_heads(h, *hw, inc.ends, inc.rowptr, inc.item, 0.0, 0.0, True, True, seed, bf16=bf)
        dl = torch.randn_like(o[0]) / B
        g = torch.ops.leakgnn.detector_heads_backward(dl if not bf else outs[False][2], h, hw[0], hw[2], o[1], o[2],
                                                      o[3], hw[4], hw[6], inc.ends, inc.rowptr, inc.item, 0.0, 0.0,
                                                      True, bf16=bf)
        outs[bf] = (o, g, dl if not bf else outs[False][2])
    (o0, g0, _), (o1, g1, _) = outs[False], outs[True]
    for i, n in enumerate(("logits", "ehid", "pooled", "hid")):
        print(f"fwd {n:8s} rel {rel(o1[i], o0[i]):.3e}")
    for i, n in enumerate(("dh", "dW1", "db1", "dW2", "db2", "ndW1", "ndb1", "ndW2", "ndb2")):
        print(f"bwd {n:8s} rel {rel(g1[i], g0[i]):.3e}")
    # bwd alone in bf16 on the fp32 forward's hidden layer
    g2 = torch.ops.leakgnn.detector_heads_backward(outs[False][2], h, hw[0], hw[2], o0[1], o0[2], o0[3], hw[4], hw[6],
                                                   inc.ends, inc.rowptr, inc.item, 0.0, 0.0, True, bf16=True)
    for i, n in enumerate(("dh", "dW1", "db1", "dW2")):
        print(f"bwd-only-bf16 {n:8s} rel {rel(g2[i], g0[i]):.3e}")


if __name__ == "__main__":
    main()
