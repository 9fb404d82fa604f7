"""Diagnostic (GPU box): where do the B = 256 gradient errors of the HIP path come from?

Runs the test_detector_b256_eval_vs_oracle case and compares, at every ReLU of the
detector (node init, each GCN layer, EdgeHead hidden), the sign pattern the HIP path used
with the sign of the fp64 oracle's pre-activation; the same for torch fp32 on the CPU and
on the GPU.  A flipped ReLU mask changes the gradient by a whole term, independent of the
summation order, so it separates "kink flips" from accumulation error.  Then predicts the
EdgeHead db1 error from the HIP path's flips alone and prints it beside the measured one.
"""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[3]
for p in (ROOT, ROOT / "leak-det-gnn_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))

from helpers import LTA_INP, lta_ids  # noqa: E402


def random_ref(seed):
    from oracle.detector_ref import LeakDetectorRef
    sensors, pipes = lta_ids()
    torch.manual_seed(seed)
    ref = LeakDetectorRef(LTA_INP, sensors, pipes).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    return {k: v.clone() for k, v in ref.state_dict().items()}


def run_ref(sd, r, tf, dt, dev, up=None, lab=None):
    from oracle.detector_ref import LeakDetectorRef
    sensors, pipes = lta_ids()
    mr = LeakDetectorRef(LTA_INP, sensors, pipes).eval()
    mr.load_state_dict(sd)
    mr = mr.to(dt).to(dev)
    mr.sensor_encoder.gru.train()
    pre = {}
    mr.sensor_to_node.register_forward_hook(lambda m, i, o: pre.__setitem__("init", o.detach().cpu().double()))
    for l, c in enumerate(mr.convs):
        c.register_forward_hook(lambda m, i, o, l=l: pre.__setitem__(f"conv{l}", o.detach().cpu().double()))
    mr.edge_head.mlp[0].register_forward_hook(lambda m, i, o: pre.__setitem__("edge", o.detach().cpu().double()))
    mr.noleak_head.mlp[0].register_forward_hook(lambda m, i, o: pre.__setitem__("noleak", o.detach().cpu().double()))
    out = mr(r.to(dt).to(dev), tf.to(dt).to(dev))
    if up is None:
        l64 = out.detach().requires_grad_(True)
        torch.nn.functional.cross_entropy(l64, lab).backward()
        up = l64.grad.clone()
    out.backward(up.to(dt).to(dev))
    grads = {n: p.grad.detach().cpu().double() for n, p in mr.named_parameters()}
    return pre, grads, up


def main():
    from models import library, ops  # noqa: F401
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    dev = torch.device("cuda:0")
    sd = random_ref(41)
    B = 256
    gen = torch.Generator().manual_seed(42)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen)
    pre64, g64, up = run_ref(sd, r, tf, torch.float64, "cpu", lab=lab)
    pre32, g32, _ = run_ref(sd, r, tf, torch.float32, "cpu", up=up)
    pre32g, g32g, _ = run_ref(sd, r, tf, torch.float32, dev, up=up)

    m = LeakDetector(LTA_INP, sensors, pipes).to(dev).eval()
    m.load_state_dict(sd)
    # the HIP path's ReLU outputs: trunk layer outputs and the kept EdgeHead hidden
    cap = {}
    trunk, heads = torch.ops.leakgnn.gnn_trunk, torch.ops.leakgnn.detector_heads

    class Spy:
        def __getattr__(self, name):
            real = getattr(torch.ops.leakgnn, name)
            if name == "gnn_trunk":
                def f(*a):
                    xs = real(*a)
                    cap["xs"] = [x.detach().clone() for x in xs]
                    cap["nm"] = a[19]
                    return xs
                return f
            if name == "detector_heads":
                def f(*a):
                    out = real(*a)
                    cap["ehid"] = out[1].detach().clone()
                    return out
                return f
            return real
    import models.detector as det
    real_ops = det.torch.ops
    det_torch = det.torch

    class OpsNS:
        leakgnn = Spy()

        def __getattr__(self, name):
            return getattr(real_ops, name)

    class TorchNS:
        ops = OpsNS()

        def __getattr__(self, name):
            return getattr(det_torch, name)
    det.torch = TorchNS()
    try:
        lg = m(r.to(dev), tf.to(dev))
        lg.backward(up.float().to(dev))
    finally:
        det.torch = det_torch
    del trunk, heads
    gg = {n: p.grad.detach().cpu().double() for n, p in m.named_parameters()}
    N = len(m.node_names)
    P = len(pipes)
    xs = cap["xs"]
    nm = cap["nm"]
    print(f"node_major={nm}, trunk outputs {[tuple(x.shape) for x in xs]}, ehid {tuple(cap['ehid'].shape)}")

    def to_bn(x):  # -> (B*N, D)
        x = x.detach().cpu().double()
        if x.dim() == 3 and nm:
            x = x.permute(1, 0, 2)
        return x.reshape(B * N, -1)

    sites = []
    if len(xs) == len(m.convs) + 1:
        sites.append(("init", to_bn(xs[0]), pre64["init"].reshape(B * N, -1)))
        conv_x = xs[1:]
    else:
        conv_x = xs
    for l, x in enumerate(conv_x):
        sites.append((f"conv{l}", to_bn(x), pre64[f"conv{l}"].reshape(B * N, -1)))
    sites.append(("edge", cap["ehid"].cpu().double().reshape(B * P, -1), pre64["edge"].reshape(B * P, -1)))
    for name, hip_out, p64 in sites:
        hm = hip_out > 0
        rm = p64 > 0
        bad = (hm != rm)
        nb = int(bad.sum())
        msg = f"{name:7s} HIP flips {nb:4d}"
        if nb:
            msg += f" (|pre64| max {p64[bad].abs().max().item():.2e})"
        for tag, pp in (("cpu32", pre32), ("gpu32", pre32g)):
            q = pp[name].reshape(p64.shape) > 0
            msg += f"  {tag} flips {int((q != rm).sum()):4d}"
        print(msg)
    # EdgeHead db1 predicted from the HIP flips alone: dl[b, p] * w2[n] * (hip_mask - ref_mask)
    ehid = cap["ehid"].cpu().double().reshape(B, P, -1)
    d = (ehid > 0).double() - (pre64["edge"].reshape(B, P, -1) > 0).double()
    w2 = sd["edge_head.mlp.3.weight"].double().reshape(-1)
    dl = up[:, :P].double()
    pred = torch.einsum("bp,bpn->n", dl, d) * w2
    act = gg["edge_head.mlp.0.bias"] - g64["edge_head.mlp.0.bias"]
    print(f"db1: measured err {act.abs().max().item():.3e}, flip-predicted {pred.abs().max().item():.3e}, "
          f"residual after removing flips {(act - pred).abs().max().item():.3e}, "
          f"cpu32 err {(g32['edge_head.mlp.0.bias'] - g64['edge_head.mlp.0.bias']).abs().max().item():.3e}, "
          f"gpu32 err {(g32g['edge_head.mlp.0.bias'] - g64['edge_head.mlp.0.bias']).abs().max().item():.3e}")
    for n in g64:
        s = g64[n].abs().max().item()
        print(f"{n:40s} scale {s:.2e}  hip {((gg[n] - g64[n]).abs().max().item()) / s:.2e}  "
              f"cpu32 {((g32[n] - g64[n]).abs().max().item()) / s:.2e}  gpu32 {((g32g[n] - g64[n]).abs().max().item()) / s:.2e}")


if __name__ == "__main__":
    main()
