"""Shared test helpers: fixture loading and the tolerance rules used everywhere."""
from __future__ import annotations

import numpy as np
import torch

from conftest import GOLD, LTA_INP  # noqa: F401

# fp32 tolerance (north star: "within 1e-5 relative fp32"): an output matches when
#   max|a - b| <= RTOL * max|b| + ATOL
# i.e. relative to the tensor's own scale, so near-zero entries do not make the
# element-wise ratio meaningless.  Integer/index outputs are compared bit-exactly.
RTOL = 1e-5
ATOL = 1e-7


def load(name: str) -> dict:
    with np.load(GOLD / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def rel_err(a, b) -> float:
    a = torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a.detach().cpu()).double()
    b = torch.as_tensor(np.asarray(b) if not torch.is_tensor(b) else b.detach().cpu()).double()
    scale = b.abs().max().item()
    return (a - b).abs().max().item() / max(scale, 1e-30)


def assert_close(a, b, rtol: float = RTOL, atol: float = ATOL, what: str = "") -> None:
    a = a.detach().cpu().double() if torch.is_tensor(a) else torch.as_tensor(np.asarray(a)).double()
    b = b.detach().cpu().double() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b)).double()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs().max().item() if a.numel() else 0.0
    lim = rtol * (b.abs().max().item() if b.numel() else 0.0) + atol
    assert err <= lim, f"{what}: max abs err {err:.3e} > {lim:.3e} (rtol {rtol}, atol {atol})"


def lta_ids():
    g = load("graph_ltown_a.npz")
    return [str(s) for s in g["sensor_ids"]], [str(p) for p in g["pipe_ids"]]


def assert_grads_close(named_grads, ref_grads: dict, rtol: float = RTOL, rtol_inf: float = 1e-4,
                       prefix: str = "grad ") -> None:
    """Parameter gradients are judged as ONE vector (the thing the optimizer consumes):
      ||g - g_ref||_2   <= rtol     * ||g_ref||_2      (1e-5, the north-star fp32 bar)
      ||g_t - g_ref_t||_inf <= rtol_inf * ||g_ref||_inf  for every tensor t (localised-bug net)
    A per-tensor bound relative to the tensor's own size is meaningless for sums with
    heavy cancellation: the last EdgeHead bias grad is the sum over every (window, pipe)
    of softmax - onehot, ~1e-2 while its terms are ~1, and torch's GPU vs CPU reduction
    order alone moves it by ~1e-6 relative to the gradient scale."""
    refs = {n: (torch.as_tensor(np.asarray(v)) if not torch.is_tensor(v) else v.detach().cpu()).double()
            for n, v in ref_grads.items()}
    gs = {n: g.detach().cpu().double() for n, g in named_grads}
    assert set(gs) == set(refs), sorted(set(gs) ^ set(refs))
    num = sum(((gs[n] - refs[n]) ** 2).sum().item() for n in refs) ** 0.5
    den = sum((refs[n] ** 2).sum().item() for n in refs) ** 0.5
    assert num <= rtol * den + ATOL, f"{prefix}vector: ||g - ref||_2 = {num:.3e} > {rtol} * {den:.3e}"
    scale = max(r.abs().max().item() for r in refs.values())
    for n, r in refs.items():
        assert gs[n].shape == r.shape, n
        err = (gs[n] - r).abs().max().item()
        assert err <= rtol_inf * scale + ATOL, f"{prefix}{n}: max abs err {err:.3e} > {rtol_inf * scale:.3e}"


def oracle_grads(state: dict, residual, tfeat, label, dtype) -> tuple:
    """CPU oracle (oracle/detector_ref.py) logits and parameter grads in `dtype` on the given inputs."""
    from oracle.detector_ref import LeakDetectorRef
    sensors, pipes = lta_ids()
    m = LeakDetectorRef(LTA_INP, sensors, pipes).eval()
    m.load_state_dict(state)
    m = m.to(dtype)
    out = m(torch.as_tensor(residual).to(dtype), torch.as_tensor(tfeat).to(dtype))
    torch.nn.functional.cross_entropy(out, torch.as_tensor(label)).backward()
    return out.detach(), {n: p.grad.detach() for n, p in m.named_parameters()}


def assert_grads_match_truth(gpu: dict, cpu32: dict, cpu64: dict, slack: float = 4.0, rtol: float = RTOL,
                             rtol_tensor: float | None = None, ref32: dict | None = None) -> None:
    """Backward bar (the north star bounds the fp32 FORWARD at 1e-5; for gradients the
    reference's own fp32 CPU path is itself ~1e-5 off in norm because some parameter
    grads are sums with heavy cancellation).  Against an fp64 run of the oracle, every
    tensor's GPU error must be within `slack` x the CPU fp32 error or within rtol of the
    tensor's scale (rtol_tensor, default rtol), and likewise for the whole-vector 2-norm
    (always rtol).  ref32: the same reference arithmetic as plain torch fp32 on the GPU
    (its GEMM / scatter accumulation order); when given, its error vs fp64 also sets the
    fp32 yardstick, so a sum over ~10^5 rows is not held to torch-CPU's cascaded summation."""
    rt = rtol if rtol_tensor is None else rtol_tensor
    g64 = {n: v.double().cpu() for n, v in cpu64.items()}
    e_gpu2 = e_cpu2 = n2 = 0.0
    bad = []
    for n, t in g64.items():
        g = gpu[n].detach().double().cpu()
        c = cpu32[n].detach().double().cpu()
        eg = (g - t).abs().max().item()
        ec = (c - t).abs().max().item()
        if ref32 is not None:
            ec = max(ec, (ref32[n].detach().double().cpu() - t).abs().max().item())
        lim = max(slack * ec, rt * t.abs().max().item()) + 1e-12
        if eg > lim:
            bad.append(f"grad {n}: gpu err {eg:.3e} > {lim:.3e} (fp32 reference err {ec:.3e}, "
                       f"scale {t.abs().max().item():.3e})")
        e_gpu2 += ((g - t) ** 2).sum().item()
        e_ref = ((c - t) ** 2).sum().item()
        if ref32 is not None:
            e_ref = max(e_ref, ((ref32[n].detach().double().cpu() - t) ** 2).sum().item())
        e_cpu2 += e_ref
        n2 += (t ** 2).sum().item()
    assert not bad, "; ".join(bad)
    e_gpu2, e_cpu2, n2 = e_gpu2 ** 0.5, e_cpu2 ** 0.5, n2 ** 0.5
    assert e_gpu2 <= max(slack * e_cpu2, rtol * n2), f"grad vector: gpu {e_gpu2:.3e}, cpu32 {e_cpu2:.3e}, |g| {n2:.3e}"


def hip_relu_masks(cap: dict, B: int, N: int, P: int, ends) -> dict:
    """The kink decisions the HIP path took, from LeakDetector.capture, in the shapes of the
    oracle's sites (oracle/detector_ref.py relu_masks): every ReLU (its stored
    post-ReLU/dropout activations: x > 0 <=> unit active and kept) and the sign of
    h_u - h_v behind the EdgeHead's |h_u - h_v| features (pipe ends `ends` (P, 2)), taken
    from the same fp32 node features the edge kernels read."""
    xs = cap["xs"]
    hn = xs[-1].detach()
    hn = hn.permute(1, 0, 2) if cap["node_major"] else hn  # (B, N, D)
    ends = ends.to(hn.device).long()
    sign = torch.sign(hn[:, ends[:, 0]] - hn[:, ends[:, 1]]).cpu()

    def bnd(x):
        x = x.detach()
        return (x.permute(1, 0, 2) if cap["node_major"] else x).reshape(B, N, -1).cpu() > 0
    out = {"init": bnd(xs[0])}
    for l, x in enumerate(xs[1:]):
        out[f"conv{l}"] = bnd(x)
    out["edge"] = cap["edge_hidden"].detach().reshape(B, P, -1).cpu() > 0
    out["noleak"] = cap["noleak_hidden"].detach().reshape(B, -1).cpu() > 0
    out["absdiff"] = sign
    return out


def check_relu_ties(pre64: dict, masks: dict, keep: dict | None = None, rel: float = 1e-5) -> int:
    """Every kink (ReLU, or the sign behind |h_u - h_v|) where the HIP path and the fp64
    oracle took different sides must be a tie: |fp64 pre-activation| <= rel x the site's
    largest.  Units dropped by dropout (keep == 0)
    are not decisions.  Returns the number of such ties (each then enters the fp64 truth
    through relu_masks, so gradients are compared on the same branch)."""
    ties = 0
    for site, m in masks.items():
        z = pre64[site].detach().double().cpu().reshape(m.shape)
        flip = m != (z > 0) if m.dtype == torch.bool else m != torch.sign(z)
        if keep is not None and site in keep:
            flip &= keep[site].cpu().reshape(m.shape) != 0
        n = int(flip.sum())
        if n:
            worst = z[flip].abs().max().item()
            lim = rel * z.abs().max().item()
            assert worst <= lim, f"ReLU site {site}: {n} HIP decisions differ from fp64, |pre| up to {worst:.3e} > {lim:.3e}"
            ties += n
    return ties


def oracle_run(sd: dict, r, tf, dt, dev, up=None, lab=None, masks=None, autocast=False, net=None):
    """The oracle detector (oracle/detector_ref.py) in eval mode: (logits, grads, fp64-comparable ReLU
    pre-activations, upstream gradient) for `up`, or for the CE gradient of `lab` in this
    run's own precision when up is None.  masks: ReLU decisions to use (relu_masks).
    net: (inp_path, sensors, pipes, constructor kwargs); default L-TOWN-A."""
    from oracle.detector_ref import LeakDetectorRef
    if net is None:
        sensors, pipes = lta_ids()
        net = (LTA_INP, sensors, pipes, {})
    mr = LeakDetectorRef(net[0], net[1], net[2], **net[3]).eval()
    mr.load_state_dict(sd)
    mr = mr.to(dt).to(dev)
    mr.sensor_encoder.gru.train()  # MIOpen's RNN backward needs training mode (1 layer: no dropout)
    mr.relu_masks = masks or {}
    if autocast:  # the tier keeps the GRU encoder fp32: so does the yardstick
        enc_fwd = mr.sensor_encoder.forward

        def enc_fp32(*a):
            with torch.autocast("cuda", enabled=False):
                return enc_fwd(*a)
        mr.sensor_encoder.forward = enc_fp32
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        out = mr(r.to(dt).to(dev), tf.to(dt).to(dev)).float() if autocast else mr(r.to(dt).to(dev), tf.to(dt).to(dev))
    if up is None:
        lo = out.detach().requires_grad_(True)
        torch.nn.functional.cross_entropy(lo, lab).backward()
        up = lo.grad.clone()
    out.backward(up.to(dt).to(dev))
    pre = {k[len("pre_"):]: v.detach() for k, v in mr.trace.items() if k.startswith("pre_")}
    return out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in mr.named_parameters()}, pre, up
