"""The compressed node init (ABI 21) on MI355X: x_0 kept as its sensor rows plus [x_0 > 0]
bits (lg_node_init_bits_fwd) and read by layer 0 through the sensor-marked node table
(lg_gcn_fwd_nm_x0, lg_gcn_bwd_nm_x0).  The reference materialises x_0 = dropout(relu(
sensor_to_node([h0, mask]))) (detector.py:179-190).  Checked against the dense path
(lg_node_init_proj_fwd + lg_gcn_fwd_nm_bits / lg_gcn_bwd_nm_bits), which the oracle tests pin
to the reference: the node init and the layer-0 backward bit for bit; the layer-0 forward
within 1e-6 of its output scale (ABI 22: the sensor neighbours' terms are added after the
others, by the consumer waves) with the same ReLU/dropout pattern wherever |y| clears that."""
from __future__ import annotations

import pytest
import torch

from helpers import LTA_INP, lta_ids

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def state():
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
    graph, inc, slot, sidx, live, nons = m._device_state(DEV)
    return m, graph, slot, sidx


def _expected_bits(x0, B, D):
    """[x0 > 0] of node-major x0 (N, B, D) in the ymask layout: per (node, window group) 64
    lanes, bit 4k + i of lane l = row RPI k + l // LPR of the group, channel 4 (l % LPR) + i."""
    N = x0.shape[0]
    LPR = D // 4
    RPI = 64 // LPR
    K = 16 // RPI
    G = (B + 15) // 16
    pad = torch.zeros(N, G * 16, D, device=x0.device, dtype=torch.bool)
    pad[:, :B] = x0 > 0
    t = pad.view(N, G, K, RPI, LPR, 4)                         # n, g, k, rl, fg, i
    t = t.permute(0, 1, 3, 4, 2, 5).reshape(N, G, 64, 4 * K)   # lane = rl * LPR + fg, bit 4k + i
    w = (t.to(torch.int32) << torch.arange(4 * K, device=x0.device, dtype=torch.int32)).sum(-1)
    return w.to(torch.int16).reshape(-1)


def _node_init(lib, ops, nat, slot, sidx, h_s, Wp, bias, B, N, S, D, flags, p, seed):
    st = ops.stream_of(h_s)
    x0 = torch.full((N, B, D), float("nan"), device=DEV)
    ops.check(lib.lg_node_init_proj_fwd(ops.ptr(slot), ops.ptr(sidx), ops.ptr(h_s), ops.ptr(Wp), ops.ptr(bias),
                                        ops.ptr(x0), B, N, S, D, D, flags | nat.LG_F_NODE_MAJOR, p, seed, 0, st),
              "node init dense")
    xs0 = torch.zeros(S, B, D, device=DEV)
    bits = torch.full((N * ((B + 15) // 16) * 64,), -1, device=DEV, dtype=torch.int16)
    ops.check(lib.lg_node_init_bits_fwd(ops.ptr(slot), ops.ptr(sidx), ops.ptr(h_s), ops.ptr(Wp), ops.ptr(bias),
                                        ops.ptr(xs0), ops.ptr(bits), B, N, S, D, D, flags, p, seed, 0, st),
              "node init bits")
    return x0, xs0, bits


@pytest.mark.parametrize("B,D,p", [(256, 64, 0.1), (37, 64, 0.0), (37, 64, 0.3), (64, 32, 0.1)])
def test_node_init_bits_equal_dense(state, B, D, p):
    from models import _native as nat
    from models import ops
    from models.library import expand_x0
    m, g, slot, sidx = state
    lib = nat.load_library()
    N, S = 661, sidx.numel()
    gen = torch.Generator().manual_seed(B * 7 + D)
    h_s = torch.randn(B, S, D, generator=gen).to(DEV)
    Wp = (torch.randn(D, D + 1, generator=gen) / 8).to(DEV)
    bias = torch.randn(D, generator=gen).to(DEV)  # about half the channels relu to 0
    flags = nat.LG_F_DROPOUT if p > 0 else 0
    x0, xs0, bits = _node_init(lib, ops, nat, slot, sidx, h_s, Wp, bias, B, N, S, D, flags, p, 424242)
    assert torch.equal(bits, _expected_bits(x0, B, D)), "[x0 > 0] bits differ from the dense node init"
    for s, n in enumerate(sidx.tolist()):
        if int(slot[n]) == s:
            assert torch.equal(xs0[s], x0[n]), f"sensor row of slot {s} differs"
    assert torch.equal(expand_x0(xs0, bits, slot, bias, N, p), x0), "expanded x0 differs from the dense node init"


@pytest.mark.parametrize("B,D,extra", [(256, 64, 0), (256, 64, "x3"), (37, 64, 0), (64, 32, 0), (48, 64, "bf16")])
def test_layer0_x0_forward_and_backward_equal_dense(state, B, D, extra):
    """lg_gcn_fwd_nm_x0 == lg_gcn_fwd_nm_bits on the dense x0, and lg_gcn_bwd_nm_x0 ==
    lg_gcn_bwd_nm_bits (dW, db, the node-bias sum, the sensor rows of dx), bit for bit."""
    from models import _native as nat
    from models import ops
    m, g, slot, sidx = state
    lib = nat.load_library()
    N, S = 661, sidx.numel()
    p = 0.1
    gen = torch.Generator().manual_seed(B + D)
    h_s = torch.randn(B, S, D, generator=gen).to(DEV)
    Wp = (torch.randn(D, D + 1, generator=gen) / 8).to(DEV)
    nbias = torch.randn(D, generator=gen).to(DEV)
    x0, xs0, bits = _node_init(lib, ops, nat, slot, sidx, h_s, Wp, nbias, B, N, S, D, nat.LG_F_DROPOUT, p, 99)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    xf = {0: 0, "x3": nat.LG_F_BF16X3, "bf16": nat.LG_F_BF16 | nat.LG_F_PC}[extra]
    flags = nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT | xf
    st = ops.stream_of(x0)
    mk = m._x0marks(g, slot)  # graph-level: the same tables at any D
    y_d = torch.empty(N, B, D, device=DEV)
    y_x = torch.empty(N, B, D, device=DEV)
    ops.check(lib.lg_gcn_fwd_nm_bits(ops.ptr(g.nodetab), ops.ptr(g.pairs), ops.ptr(x0), ops.ptr(W), ops.ptr(b),
                                     ops.ptr(y_d), B, N, D, g.nnz_cap, flags, p, 7, 1, st, None), "fwd dense")
    ops.check(lib.lg_gcn_fwd_nm_x0(ops.ptr(mk.nodetab_s), ops.ptr(mk.pairs_s), ops.ptr(xs0), ops.ptr(bits),
                                   ops.ptr(nbias), ops.ptr(W), ops.ptr(b), ops.ptr(y_x), B, N, S, D, flags, p, 7, 1, st),
              "fwd x0")
    # the nm3 / exact-fp32 forms have no compressed-input variant: refused, not silently replaced
    for bad in (nat.LG_F_NM3, nat.LG_F_F32_MFMA):
        rc = lib.lg_gcn_fwd_nm_x0(ops.ptr(mk.nodetab_s), ops.ptr(mk.pairs_s), ops.ptr(xs0), ops.ptr(bits),
                                  ops.ptr(nbias), ops.ptr(W), ops.ptr(b), ops.ptr(y_x), B, N, S, D, flags | bad, p, 7, 1,
                                  st)
        assert rc == -2, f"flag {bad:#x} on the x0 layer: rc {rc} (LG_EUNSUPPORTED expected)"
    # the sums' order differs (sensor terms last): fp32 tier within 1e-6 of scale; the bf16
    # tier rounds z to bf16 before its single product, so one bf16 ulp (2^-8) of z can differ
    tol = 1e-3 if extra == "bf16" else 1e-6
    scale = y_d.abs().max().item()
    err = (y_x - y_d).abs().max().item()
    assert err <= tol * scale, f"layer-0 forward on the compressed x0: err {err:.3e} of scale {scale:.3e}"
    # same relu / dropout decisions except where the pre-activation is within rounding of 0
    flip = (y_x > 0) != (y_d > 0)
    assert (torch.maximum(y_x.abs(), y_d.abs())[flip] <= tol * scale).all()

    dy = torch.randn(N, B, D, generator=gen).to(DEV)
    scale = 1.0 / (1.0 - p)
    bflags = nat.LG_F_MASK_OUT | nat.LG_F_DX_SENSOR_ROWS | (nat.LG_F_BF16 if extra == "bf16" else 0)
    outs = []
    for x0c in (False, True):
        dx = torch.zeros(N, B, D, device=DEV)
        dW, db, dnb = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
        if x0c:
            ops.check(lib.lg_gcn_bwd_nm_x0(ops.ptr(g.nodetab_t), ops.ptr(g.pairs_t), ops.ptr(mk.pos_slot_t),
                                           ops.ptr(dy), ops.ptr(xs0), ops.ptr(bits), ops.ptr(nbias), ops.ptr(W),
                                           ops.ptr(dx), ops.ptr(dW), ops.ptr(db), ops.ptr(slot), ops.ptr(dnb), B, N, S,
                                           D, bflags | nat.LG_F_DROPOUT, p, scale, ops.ptr(ws), ws.numel(), st),
                      "bwd x0")
        else:
            ops.check(lib.lg_gcn_bwd_nm_bits(ops.ptr(g.nodetab_t), ops.ptr(g.pairs_t), ops.ptr(dy), None, ops.ptr(x0),
                                             ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db), ops.ptr(slot),
                                             ops.ptr(dnb), B, N, D, bflags, 1.0, scale, ops.ptr(ws), ws.numel(), st,
                                             None), "bwd dense")
        outs.append((dx, dW, db, dnb))
    for name, a, c in zip(("dx", "dW", "db", "dnode_bias"), outs[0], outs[1]):
        assert torch.equal(a, c), f"layer-0 backward on the compressed x0: {name} differs from the dense backward"


@pytest.mark.parametrize("train", [False, True])
def test_detector_compressed_x0_equals_dense(train):
    """The whole detector step with the node init compressed (the default) equals the dense node
    init: logits and every parameter gradient within 1e-5 of their scale (train mode: the same
    dropout draws from the same seed; the layer-0 forward sums its sensor terms last)."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train(train)
    gen = torch.Generator().manual_seed(5)
    B = 48
    r = torch.randn(B, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(B, 36, 9, generator=gen).to(DEV)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(DEV)
    res = []
    for comp in (False, True):
        m.compress_x0 = comp
        m.zero_grad(set_to_none=True)
        torch.manual_seed(11)
        logits = m(r, tf)
        loss = torch.nn.functional.cross_entropy(logits, lab)
        loss.backward()
        res.append((logits.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    from helpers import assert_close
    assert_close(res[1][0], res[0][0], rtol=1e-5, what="logits")
    for k in res[0][1]:
        assert_close(res[1][1][k], res[0][1][k], rtol=1e-5, atol=0.0, what=f"grad {k}")


@pytest.mark.parametrize("layers", [1, 3])
def test_detector_gnn_layers_train_step(layers):
    """gnn_layers is a public constructor argument (reference detector.py:128,162-164).  At 1
    layer, layer 0 is also the last: its backward needs the input mask (LG_F_MASK_IN), which
    only the dense node init provides, so x_0 is not compressed there.  A train-mode step at
    B = 32 (node-major) must run and equal the dense node init's step at any depth."""
    from models.detector import LeakDetector
    from helpers import assert_close
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, sensors, pipes, gnn_layers=layers).to(DEV).train()
    gen = torch.Generator().manual_seed(6)
    B = 32
    r = torch.randn(B, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(B, 36, 9, generator=gen).to(DEV)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(DEV)
    res = []
    for comp in (False, True):
        m.compress_x0 = comp
        m.zero_grad(set_to_none=True)
        torch.manual_seed(12)
        logits = m(r, tf)
        torch.nn.functional.cross_entropy(logits, lab).backward()
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
        res.append((logits.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    assert_close(res[1][0], res[0][0], rtol=1e-5, what="logits")
    for k in res[0][1]:
        assert_close(res[1][1][k], res[0][1][k], rtol=1e-5, atol=0.0, what=f"grad {k}")


@pytest.mark.parametrize("train,B", [(True, 48), (False, 48), (True, 256), (True, 37)])
def test_encoder_trunk_equals_separate_ops(train, B):
    """library.encoder_trunk (the GRU, node init and layers as one op: the node init in the GRU
    forward's epilogue, the projection's backward in the GRU backward's prologue / epilogue)
    equals gru_encoder + gnn_trunk bit for bit: logits and every parameter gradient (same
    arithmetic, same dropout draws, the reductions over the same partials in the same order)."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train(train)
    with torch.no_grad():
        for c in m.convs:
            c.bias.normal_(0, 0.1)
    gen = torch.Generator().manual_seed(7)
    r = torch.randn(B, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(B, 36, 9, generator=gen).to(DEV)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(DEV)
    res = []
    for fused in (False, True):
        m.fuse_encoder = fused
        m.zero_grad(set_to_none=True)
        torch.manual_seed(13)
        logits = m(r, tf)
        torch.nn.functional.cross_entropy(logits, lab).backward()
        res.append((logits.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    assert torch.equal(res[1][0], res[0][0]), "logits differ"
    for k in res[0][1]:
        assert torch.equal(res[1][1][k], res[0][1][k]), f"grad {k} differs: {(res[1][1][k] - res[0][1][k]).abs().max():.3e}"


def test_encoder_trunk_eval_no_grad_and_fallbacks():
    """Eval under no_grad takes the fused op without saving the GRU steps; a residual that wants
    a gradient, or the window-major layout (B < 16), takes the separate ops."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    gen = torch.Generator().manual_seed(8)
    r = torch.randn(32, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(32, 36, 9, generator=gen).to(DEV)
    with torch.no_grad():
        m.fuse_encoder = True
        a = m(r, tf)
        m.fuse_encoder = False
        b = m(r, tf)
    assert torch.equal(a, b)
    m.fuse_encoder = True
    rg = r.clone().requires_grad_(True)
    assert not m._fused_encoder(rg, tf, 32, 661, 64, True)
    m(rg, tf).sum().backward()
    assert rg.grad is not None and torch.isfinite(rg.grad).all()
    assert not m._fused_encoder(r[:8], tf[:8], 8, 661, 64, False)
