"""Diagnostic (GPU box): the train-mode B = 256 case of tests/test_gpu_configs.py, with the
gradient at the GRU output (h_s) and at the trunk input (the sensor rows' node-init
pre-activation) of the HIP path compared with the fp32 / fp64 replays, to place the GRU
weight-gradient error between the GRU kernel and the layers above it."""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[3]
for p in (ROOT, ROOT / "leak-det-gnn_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

import test_gpu_configs as T  # noqa: E402
from helpers import LTA_INP, check_relu_ties, hip_relu_masks, lta_ids  # noqa: E402


def main():
    from models.detector import LeakDetector
    dev = torch.device("cuda:0")
    sensors, pipes = lta_ids()
    sd = T._random_ref(51)
    B = 256
    gen = torch.Generator().manual_seed(52)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    up = torch.randn(B, len(pipes) + 1, generator=gen) / B
    m = LeakDetector(LTA_INP, sensors, pipes).to(dev).train()
    m.load_state_dict(sd)
    torch.manual_seed(53)
    m.capture = {}
    lg = m(r.to(dev), tf.to(dev))
    lg.backward(up.to(dev))
    cap = m.capture
    masks = hip_relu_masks(cap, B, len(m.node_names), len(pipes), m.pipe_ends)
    torch.manual_seed(53)
    seeds = tuple(int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item()) for _ in range(2))
    a32, a64, a32d = {}, {}, {}
    _, g64, pre64, keep = T._replay_train_cpu(sd, r, tf, seeds, torch.float64, up, aux=a64)
    ties = check_relu_ties(pre64, masks, keep)
    print("ties", ties)
    for site, mk in masks.items():
        z = pre64[site].double().cpu().reshape(mk.shape)
        flip = mk != (z > 0) if mk.dtype == torch.bool else mk != torch.sign(z)
        if site in keep:
            flip &= keep[site].cpu().reshape(mk.shape) != 0
        print(f"  {site}: {int(flip.sum())} decisions differ")
        if flip.any():
            idx = flip.nonzero()[:4].tolist()
            print(f"  tie at {site} {idx} pre64 {z[flip][:4].tolist()}")
    nat = a64
    if ties:
        a64 = {}
        _, g64, _, _ = T._replay_train_cpu(sd, r, tf, seeds, torch.float64, up, masks=masks, aux=a64)
    tn, tm = nat["h_s"].grad.double().cpu(), a64["h_s"].grad.double().cpu()
    print(f"d h_s natural vs HIP-branch fp64: {(tn - tm).abs().max().item() / tn.abs().max().item():.2e}")
    _, g32, _, _ = T._replay_train_cpu(sd, r, tf, seeds, torch.float32, up, aux=a32)
    _, g32d, _, _ = T._replay_train_cpu(sd, r, tf, seeds, torch.float32, up, dev=dev, aux=a32d)
    sidx = m.sensor_node_idx
    t = a64["h_s"].grad.double().cpu()
    s = t.abs().max().item()
    e = lambda x: (x.double().cpu() - t).abs().max().item() / s  # noqa: E731
    print(f"d h_s   scale {s:.2e}  hip {e(cap['h_s'].grad):.2e}  cpu32 {e(a32['h_s'].grad):.2e}  gpu32 {e(a32d['h_s'].grad):.2e}")
    for n, p in m.named_parameters():
        t = g64[n].double()
        s = t.abs().max().item()
        e = lambda x: (x.double().cpu() - t).abs().max().item() / s  # noqa: E731
        print(f"{n:40s} scale {s:.2e}  hip {e(p.grad):.2e}  cpu32 {e(g32[n]):.2e}  gpu32 {e(g32d[n]):.2e}")


if __name__ == "__main__":
    main()
