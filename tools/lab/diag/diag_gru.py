"""Diagnostic (GPU box): precision of the fused GRU encoder backward alone at the bench
shape (B = 256 windows x 29 sensors, L = 36), against torch nn.GRU in fp64 (truth) and
fp32 on the CPU and the GPU, for a random dh_L of the size the detector feeds it; and
with dh_L taken from the train-mode B = 256 test (upstream error included)."""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[3]
for p in (ROOT, ROOT / "leak-det-gnn_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))


def run_torch(gru_sd, r, tf, dh, dt, dev):
    g = torch.nn.GRU(10, 64, batch_first=True).to(dt).to(dev)
    g.load_state_dict({k: v.to(dt) for k, v in gru_sd.items()})
    B, L, S = r.shape
    x = torch.cat([r.transpose(1, 2).reshape(B * S, L, 1), tf.unsqueeze(1).expand(B, S, L, 9).reshape(B * S, L, 9)], -1)
    x = x.to(dt).to(dev)
    out, _ = g(x)
    out[:, -1, :].backward(dh.reshape(B * S, 64).to(dt).to(dev))
    return {n: p.grad.detach().cpu().double() for n, p in g.named_parameters()}


def main():
    from models import library  # noqa: F401
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    g = torch.nn.GRU(10, 64, batch_first=True)
    sd = {k: v.detach().clone() for k, v in g.state_dict().items()}
    B, L, S = 256, 36, 29
    gen = torch.Generator().manual_seed(4)
    r = torch.randn(B, L, S, generator=gen)
    tf = torch.randn(B, L, 9, generator=gen)
    dh = torch.randn(B, S, 64, generator=gen) * 1e-4
    g64 = run_torch(sd, r, tf, dh, torch.float64, "cpu")
    g32 = run_torch(sd, r, tf, dh, torch.float32, "cpu")
    g32d = run_torch(sd, r, tf, dh, torch.float32, dev)
    ws = [sd[k].to(dev).requires_grad_(True) for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    h = torch.ops.leakgnn.gru_encoder(r.to(dev), tf.to(dev), *ws, True)[0]
    h.backward(dh.to(dev))
    names = ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")
    for n, w in zip(names, ws):
        t = g64[n]
        s = t.abs().max().item()
        e = lambda a: (a.double().cpu() - t).abs().max().item() / s  # noqa: E731
        print(f"{n:14s} scale {s:.2e}  hip {e(w.grad):.2e}  cpu32 {e(g32[n]):.2e}  gpu32 {e(g32d[n]):.2e}")


if __name__ == "__main__":
    main()
