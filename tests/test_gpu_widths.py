"""Widths other than the reference callers' 64 (VERDICT r05 missing #1, #2): the GRU encoder
at any hidden size (lg_gru_fwd / lg_gru_bwd's generic kernel, ABI 26), LeakDetector at any
sensor_hidden / node_hidden (detector.py:128-129; models/detector.py _forward_general) and
global_mean_pool over a ragged, unordered batch vector (PyG's scatter mean).  Each against the
fp64 oracle (oracle/detector_ref.py) or torch's CPU modules in fp64."""
import numpy as np
import pytest
import torch

from conftest import LTA_INP
from helpers import assert_close, assert_grads_match_truth, lta_ids, oracle_run

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("H,use_time", [(48, True), (17, False), (96, True)])
def test_gru_generic_width_matches_torch(H, use_time):
    """h_L and every gradient (weights, residual, tfeat) of the shared GRU at widths the tiled
    kernels do not cover, against torch.nn.GRU on the CPU in fp64 (fp32 bar: 1e-5 of scale for
    h_L, the whole gradient vector within 4x torch fp32's own error or 1e-5)."""
    from models.detector import SharedSensorGRUEncoder
    torch.manual_seed(3)
    enc = SharedSensorGRUEncoder(hidden_size=H, use_time=use_time)
    B, L, S = 3, 36, 5
    r = torch.randn(B, L, S)
    tf = torch.randn(B, L, 9) if use_time else None

    def run(mod, dt, dev):
        m = SharedSensorGRUEncoder(hidden_size=H, use_time=use_time)
        m.load_state_dict(mod.state_dict())
        m = m.to(dt).to(dev)
        ri = r.to(dt).to(dev).requires_grad_(True)
        ti = tf.to(dt).to(dev).requires_grad_(True) if use_time else None
        if dev == "cpu":  # torch's own module: x_t = [r[b, t, s], tfeat[b, t]] per sequence b*S + s
            x = ri.permute(0, 2, 1).reshape(B * S, L, 1)
            if use_time:
                x = torch.cat([x, ti[:, None].expand(B, S, L, 9).reshape(B * S, L, 9)], dim=-1)
            _, hl = m.gru(x)
            out = hl[0].view(B, S, H)
        else:
            out = m(ri, ti)
        g = torch.Generator().manual_seed(5)
        out.backward(torch.randn(out.shape, generator=g, dtype=torch.float64).to(dt).to(dev))
        grads = {n: p.grad for n, p in m.gru.named_parameters()}
        grads["residual"] = ri.grad
        if use_time:
            grads["tfeat"] = ti.grad
        return out.detach().cpu(), grads

    hg, gg = run(enc, torch.float32, DEV)
    h64, g64 = run(enc, torch.float64, "cpu")
    _, g32 = run(enc, torch.float32, "cpu")
    assert_close(hg, h64, what=f"GRU h_L (H={H})")
    assert_grads_match_truth(gg, g32, g64)


@pytest.mark.parametrize("ds,dn", [(48, 40), (64, 96), (32, 64)])
def test_detector_general_widths_vs_oracle(ds, dn):
    """LeakDetector(sensor_hidden=ds, node_hidden=dn) on L-TOWN-A, B = 4, eval mode, random
    weights: logits within 1e-5 of the oracle (fp32 CPU) and parameter gradients for the oracle's
    fp64 CE gradient against the fp64 truth (4x the fp32 reference's own error, or 1e-5).  The
    (32, 64) case has both widths in {32, 64} but unequal (the tiled node init needs them equal):
    the general path with the tiled GRU (H = 32) and the tiled GCNConv (D = 64)."""
    from models.detector import LeakDetector
    from oracle.detector_ref import LeakDetectorRef
    sensors, pipes = lta_ids()
    kw = dict(sensor_hidden=ds, node_hidden=dn)
    torch.manual_seed(11)
    ref = LeakDetectorRef(LTA_INP, sensors, pipes, **kw).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    net = (LTA_INP, sensors, pipes, kw)
    B = 4
    gen = torch.Generator().manual_seed(12)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen)
    _, g64, _, up = oracle_run(sd, r, tf, torch.float64, "cpu", lab=lab, net=net)
    o32, g32, _, _ = oracle_run(sd, r, tf, torch.float32, "cpu", up=up, net=net)
    m = LeakDetector(LTA_INP, sensors, pipes, **kw).to(DEV).eval()
    m.load_state_dict(sd)
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(up.float().to(DEV))
    assert lg.shape == (B, len(pipes) + 1)
    assert_close(lg, o32, what=f"logits ({ds}, {dn})")
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64)


def test_detector_general_widths_train_step():
    """Train mode at a general width (dropout from torch's generator): a finite step whose
    gradients reach every parameter."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes, sensor_hidden=24, node_hidden=40).to(DEV).train()
    r, tf = torch.randn(8, 36, 29, device=DEV), torch.randn(8, 36, 9, device=DEV)
    lab = torch.randint(0, len(pipes) + 1, (8,), device=DEV)
    loss = torch.nn.functional.cross_entropy(m(r, tf), lab)
    loss.backward()
    assert torch.isfinite(loss)
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n


@pytest.mark.parametrize("D", [64, 20])
def test_global_mean_pool_ragged(D):
    """PyG's scatter mean over an unordered batch vector with unequal graphs and one empty graph
    (pools to 0); then the equal-window layout (the HIP kernel at D = 64) twice with the same
    batch tensor, against numpy in fp64."""
    from models.gcn import global_mean_pool
    rng = np.random.default_rng(7)
    G, rows = 6, 50
    batch = rng.integers(0, G, rows)
    batch[batch == 3] = 4  # graph 3 empty
    x = rng.standard_normal((rows, D)).astype(np.float32)
    want = np.zeros((G, D))
    for g in range(G):
        if (batch == g).any():
            want[g] = x[batch == g].astype(np.float64).mean(0)
    xt = torch.from_numpy(x).to(DEV).requires_grad_(True)
    out = global_mean_pool(xt, torch.from_numpy(batch).to(DEV), size=G)
    assert_close(out, want, what="ragged mean pool")
    out.sum().backward()
    cnt = np.bincount(batch, minlength=G)
    assert_close(xt.grad, np.repeat((1.0 / cnt[batch])[:, None], D, 1), what="ragged mean pool grad")
    B, N = 4, 13
    xe = torch.randn(B * N, D, device=DEV)
    be = torch.arange(B, device=DEV).repeat_interleave(N)
    for _ in range(2):  # the second call reuses the cached layout decision
        assert_close(global_mean_pool(xe, be), xe.view(B, N, D).double().mean(1), what="window mean pool")
