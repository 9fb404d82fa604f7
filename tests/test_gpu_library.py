"""The torch.library registration of the hot-path ops (models/library.py, SURVEY §8 b):
torch.library.opcheck (schema, fake-tensor shapes, autograd registration and the
AOTAutograd dynamic-shape dispatch of forward + backward) on every differentiable op, and
one LeakDetector step traced by torch.compile (aot_eager) against the eager step."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import LTA_INP, assert_close, load, lta_ids
from models import library  # noqa: F401  (registers the torch.ops.leakgnn ops)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph(N=300, E=1500, seed=1):
    from models.ops import GCNGraph
    gen = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, N, (2, E), generator=gen)
    return GCNGraph.build(ei, N, DEV)


def _check(op, args, kwargs=None):
    torch.library.opcheck(op, args, kwargs, test_utils=("test_schema", "test_autograd_registration",
                                                        "test_faketensor", "test_aot_dispatch_dynamic"))


def test_opcheck_gcn_conv_and_mean_pool():
    g = _graph()
    x = torch.randn(300, 64, device=DEV, requires_grad=True)
    W = torch.randn(64, 64, device=DEV, requires_grad=True)
    b = torch.randn(64, device=DEV, requires_grad=True)
    _check(torch.ops.leakgnn.gcn_conv.default, (x, W, b, g.rowptr, g.col, g.w, g.rowptr_t, g.col_t, g.w_t, g.nodetab,
                                                g.pairs, g.nodetab_t, g.pairs_t))
    _check(torch.ops.leakgnn.mean_pool.default, (torch.randn(4 * 50, 64, device=DEV, requires_grad=True), 4, 50))


@pytest.mark.parametrize("N,E,seed", [(661, 1532, 3), (300, 1500, 1), (1000, 400, 2), (17, 0, 4)])
def test_rows_kernels_match_window_major(N, E, seed):
    """lg_gcn_fwd_rows / lg_gcn_bwd_rows (the B = 1 GCNConv path at D = 64: 16-node tiles off
    the node table, 3-way bf16 split) against lg_gcn_fwd / lg_gcn_bwd (exact fp32 MFMA) on
    the same graph: y, dx, dW, db within 1e-6 of scale.  Random graphs up to degree ~20
    (entries past the six inline pairs), isolated nodes (E = 400 on 1000 nodes), an edgeless
    17-node graph (a ragged last tile of one row, self loops only)."""
    from models import _native as nat
    from models.ops import GCNGraph, check, ptr, stream_of
    lib = nat.load_library()
    gen = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, N, (2, E), generator=gen)
    g = GCNGraph.build(ei, N, DEV)
    D = 64
    x = torch.randn(N, D, generator=gen).to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = torch.randn(D, generator=gen).to(DEV)
    dy = torch.randn(N, D, generator=gen).to(DEV)
    st = stream_of(x)
    for flags in (0, nat.LG_F_BIAS):
        y0, y1 = torch.empty_like(x), torch.full_like(x, float("nan"))
        check(lib.lg_gcn_fwd(ptr(g.rowptr), ptr(g.col), ptr(g.w), ptr(x), ptr(W), ptr(b), ptr(y0), 1, N, D,
                             g.col.numel(), flags, 0.0, 0, 0, st), "fwd")
        check(lib.lg_gcn_fwd_rows(ptr(g.nodetab), ptr(g.pairs), ptr(x), ptr(W), ptr(b), ptr(y1), N, D, flags, st),
              "fwd rows")
        assert_close(y1, y0, rtol=1e-6, atol=0.0, what=f"fwd rows flags={flags}")
    outs = []
    for rows in (False, True):
        dx, dW, db = torch.full_like(x, float("nan")), torch.empty(D, D, device=DEV), torch.empty(D, device=DEV)
        if rows:
            ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            check(lib.lg_gcn_bwd_rows(ptr(g.nodetab_t), ptr(g.pairs_t), ptr(dy), ptr(x), ptr(W), ptr(dx), ptr(dW),
                                      ptr(db), N, D, ptr(ws), ws.numel(), st), "bwd rows")
        else:
            ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            check(lib.lg_gcn_bwd(ptr(g.rowptr_t), ptr(g.col_t), ptr(g.w_t), ptr(dy), None, ptr(x), ptr(W), ptr(dx),
                                 ptr(dW), ptr(db), None, None, 1, N, D, g.col_t.numel(), 0, 1.0, 1.0, ptr(ws), ws.numel(), st),
                  "bwd")
        outs.append((dx, dW, db))
    for i, what in enumerate(("dx", "dW", "db")):
        assert_close(outs[1][i], outs[0][i], rtol=1e-6, atol=0.0, what=f"bwd rows {what}")
    # D = 32 and extra flags are refused (the caller falls back to lg_gcn_fwd)
    LG_EUNSUPPORTED = -2  # include/leakgnn.h
    assert lib.lg_gcn_fwd_rows(ptr(g.nodetab), ptr(g.pairs), ptr(x), ptr(W), ptr(b), ptr(y0), N, 32, 0, st) == \
        LG_EUNSUPPORTED
    assert lib.lg_gcn_fwd_rows(ptr(g.nodetab), ptr(g.pairs), ptr(x), ptr(W), ptr(b), ptr(y0), N, D,
                               nat.LG_F_RELU, st) == LG_EUNSUPPORTED


def test_opcheck_sensor_proj_and_gru():
    h = torch.randn(3, 29, 64, device=DEV, requires_grad=True)
    Wn = torch.randn(64, 65, device=DEV, requires_grad=True)
    bn = torch.randn(64, device=DEV, requires_grad=True)
    _check(torch.ops.leakgnn.sensor_proj.default, (h, Wn, bn))
    r = torch.randn(3, 36, 29, device=DEV, requires_grad=True)
    tf = torch.randn(3, 36, 9, device=DEV)
    ws = [torch.randn(*s, device=DEV).div_(8).requires_grad_(True) for s in ((192, 10), (192, 64), (192,), (192,))]
    _check(torch.ops.leakgnn.gru_encoder.default, (r, tf, *ws, True))


@pytest.mark.parametrize("B,p", [(3, 0.0), (16, 0.1)])
def test_opcheck_trunk_and_heads(B, p):
    """gnn_trunk (window-major at B = 3, node-major with dropout and the bf16 tier at B = 16) and
    detector_heads on L-TOWN-A, with the detector's own graph state."""
    from models import ops
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
    graph, inc, slot, sidx, live, nons = m._device_state(DEV)
    nm = ops.use_node_major(B, 661, 64)
    seed = torch.tensor([12345], dtype=torch.long)
    h_s = torch.randn(B, 29, 64, device=DEV, requires_grad=True)
    Wn = torch.randn(64, 65, device=DEV).div_(8).requires_grad_(True)
    wts = [c.lin.weight.detach().clone().requires_grad_(True) for c in m.convs]
    bs = [c.bias.detach().clone().normal_(0, 0.1).requires_grad_(True) for c in m.convs]
    nb = torch.randn(64, device=DEV, requires_grad=True)
    g = graph
    mk = m._x0marks(g, slot)  # node-major: the compressed node init (lg_node_init_bits_fwd, lg_gcn_*_nm_x0)
    marks = (mk.nodetab_s, mk.pairs_s, mk.pos_slot_t) if nm else (None, None, None)
    _check(torch.ops.leakgnn.gnn_trunk.default,
           (h_s, Wn, nb, wts, bs, slot, sidx, nons, live, g.nodetab, g.pairs, g.rowptr, g.col, g.w, g.nodetab_t,
            g.pairs_t, g.rowptr_t, g.col_t, g.w_t, p, nm, seed, *marks), {"bf16": B == 16})
    h = torch.randn((661, B, 64) if nm else (B, 661, 64), device=DEV).relu_().requires_grad_(True)
    mlp, nmlp = m.edge_head.mlp, m.noleak_head.mlp
    hw = [t.detach().clone().requires_grad_(True) for t in (mlp[0].weight, mlp[0].bias, mlp[3].weight, mlp[3].bias,
                                                              nmlp[0].weight, nmlp[0].bias, nmlp[3].weight,
                                                              nmlp[3].bias)]
    _check(torch.ops.leakgnn.detector_heads.default, (h, *hw, inc.ends, inc.rowptr, inc.item, p, p, nm, True, seed),
           {"bf16": B == 16})


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_opcheck_encoder_trunk(p):
    """leakgnn::encoder_trunk (the GRU, node init and layers as one op) at B = 16, node-major,
    with the detector's own graph state and marks."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
    graph, inc, slot, sidx, live, nons = m._device_state(DEV)
    mk = m._x0marks(graph, slot)
    B = 16
    seed = torch.tensor([4242], dtype=torch.long)
    r, tf = torch.randn(B, 36, 29, device=DEV), torch.randn(B, 36, 9, device=DEV)
    gw = [t.detach().clone().requires_grad_(True) for t in (m.sensor_encoder.gru.weight_ih_l0,
                                                              m.sensor_encoder.gru.weight_hh_l0,
                                                              m.sensor_encoder.gru.bias_ih_l0,
                                                              m.sensor_encoder.gru.bias_hh_l0)]
    Wn = torch.randn(64, 65, device=DEV).div_(8).requires_grad_(True)
    nb = torch.randn(64, device=DEV, requires_grad=True)
    wts = [c.lin.weight.detach().clone().requires_grad_(True) for c in m.convs]
    bs = [c.bias.detach().clone().normal_(0, 0.1).requires_grad_(True) for c in m.convs]
    g = graph
    _check(torch.ops.leakgnn.encoder_trunk.default,
           (r, tf, *gw, Wn, nb, wts, bs, slot, sidx, live, g.nodetab, g.pairs, g.nodetab_t, g.pairs_t, mk.nodetab_s,
            mk.pairs_s, mk.pos_slot_t, p, seed, True), {"bf16": False})


@pytest.mark.parametrize("fullgraph", [False, True])
def test_torch_compile_aot_eager_matches_eager(fullgraph):
    """The detector forward + backward traced by torch.compile (aot_eager: every
    leakgnn:: op stays an opaque registered op) equals the eager run.  Dynamo refuses to
    wrap an nn.GRU module by default (torch._dynamo.config.allow_rnn), and the encoder
    reads its weights off the reference's nn.GRU (state-dict compatibility): plain
    torch.compile graph-breaks there; with allow_rnn the whole step is ONE graph."""
    from models.detector import LeakDetector
    state = load("detector_b2.npz")
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    m.load_state_dict({k[len("param."):]: torch.from_numpy(v) for k, v in state.items() if k.startswith("param.")})
    r = torch.randn(20, 36, 29, device=DEV)
    tf = torch.randn(20, 36, 9, device=DEV)
    lab = torch.randint(0, len(pipes) + 1, (20,), device=DEV)

    def step(model):
        model.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(model(r, tf), lab)
        loss.backward()
        return loss.detach(), [p.grad.clone() for p in model.parameters()]

    l0, g0 = step(m)
    torch._dynamo.reset()
    mc = torch.compile(m, backend="aot_eager", fullgraph=fullgraph)
    with torch._dynamo.config.patch(allow_rnn=fullgraph):
        l1, g1 = step(mc)
    assert_close(l1, l0, rtol=1e-6, what="compiled loss")
    for a, b in zip(g1, g0):
        assert_close(a, b, rtol=1e-6, what="compiled grad")
    assert np.isfinite(l1.item())


def test_kernel_timer_times_the_kernel():
    """bench.py's KernelTimer: every named call arms one library event pair
    (lg_timing_arm) that its main kernel consumes (hipExtLaunchKernelGGL); the mean is a
    positive kernel duration, no longer than a pair of stream events around the call."""
    from models import ops
    g = _graph(N=20000, E=100000)
    x = torch.randn(20000, 64, device=DEV)
    W = torch.randn(64, 64, device=DEV)
    b = torch.randn(64, device=DEV)
    args = (x, W, b, g.rowptr, g.col, g.w, g.rowptr_t, g.col_t, g.w_t, g.nodetab, g.pairs, g.nodetab_t, g.pairs_t)
    torch.ops.leakgnn.gcn_conv(*args)
    timer = ops.KernelTimer(["gcn_fwd"])
    ops.set_kernel_timer(timer)
    timer.enabled = True
    try:
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            torch.ops.leakgnn.gcn_conv(*args)
        z.record()
    finally:
        timer.enabled = False
        ops.set_kernel_timer(None)
    ms = timer.mean_ms("gcn_fwd")
    assert timer.count("gcn_fwd") == 5
    assert 0.0 < ms <= a.elapsed_time(z) / 5
    from models import _native
    assert _native.load_library().lg_timing_disarm() == 0  # nothing left armed


def test_clip_adamw_matches_torch():
    """models/optim.py ClipAdamW == torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW
    (fused) over three steps on the detector's parameter set: clipped gradients, the
    returned total norm, and the updated parameters, to fp32 rounding (the norm is summed in
    a different order)."""
    from models.detector import LeakDetector
    from models.optim import ClipAdamW
    sensors, pipes = lta_ids()
    torch.manual_seed(5)
    ma = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
    mb = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
    mb.load_state_dict(ma.state_dict())
    oa = torch.optim.AdamW(ma.parameters(), lr=1e-2, weight_decay=1e-2, fused=True)
    ob = ClipAdamW(mb.parameters(), lr=1e-2, weight_decay=1e-2, max_norm=1.0)
    for it in range(3):
        for pa, pb in zip(ma.parameters(), mb.parameters()):
            g = torch.randn_like(pa) * (0.05 if it == 1 else 1.0)  # step 1: under the clip threshold
            pa.grad, pb.grad = g.clone(), g.clone()
        na = torch.nn.utils.clip_grad_norm_(ma.parameters(), 1.0)
        oa.step()
        ob.step()
        assert_close(ob.last_grad_norm[0], na, rtol=1e-6, what="total norm")
        for (n, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            assert_close(pb.grad, pa.grad, rtol=1e-6, what=f"clipped grad {n}")
            assert_close(pb, pa, rtol=1e-6, what=f"param {n} after step {it}")
        # the device step counter is committed by the launch's last workgroup, whose ticket
        # counter (word 1, uint32) is back at 0 between launches
        st = ob.param_groups[0]["step_t"]
        assert st[0].item() == it + 1 and st[1:3].view(torch.int32).tolist() == [0, 0]


def _adam_trajectory(shapes, steps=3, seed=11, max_norm=1.0, env=None, monkeypatch=None):
    """ClipAdamW over `steps` steps on fresh parameters of `shapes` (seeded), gradients drawn
    per step (step 1 under the clip threshold); returns the final parameters, the last
    clipped gradients, the norms and the step word."""
    from models.optim import ClipAdamW
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    try:
        gen = torch.Generator(device=DEV).manual_seed(seed)
        ps = [torch.randn(s, device=DEV, generator=gen).requires_grad_(True) for s in shapes]
        opt = ClipAdamW(ps, lr=1e-2, weight_decay=1e-2, max_norm=max_norm)
        norms = []
        for it in range(steps):
            for p in ps:
                p.grad = torch.randn(p.shape, device=DEV, generator=gen) * (0.05 if it == 1 else 1.0)
            opt.step()
            norms.append(opt.last_grad_norm.clone())
        torch.cuda.synchronize()
        return ([p.detach().clone() for p in ps], [p.grad.clone() for p in ps], torch.cat(norms),
                opt.param_groups[0]["step_t"].clone())
    finally:
        for k in (env or {}):
            monkeypatch.delenv(k, raising=False)


def test_clip_adamw_barrier_under_skew_and_two_launch_form(monkeypatch):
    """the one-launch clip + AdamW must not let any workgroup see another's
    clipped gradients or a partial norm.  The odd slices are held back ~0.2 ms before their
    partial sums (LEAKGNN_LAB_ADAM_SKEW: s_sleep rounds), so without a working grid barrier the
    even slices would clip with a norm missing half its partials (the workspace holds the
    previous step's).  Parameters, clipped gradients and norms must be BIT-identical to the
    unskewed launch and to the two-launch form (same partials, same summation), and the error
    word must stay 0.  Shapes: the detector's parameter set (60 slices, one launch)."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    shapes = [tuple(p.shape) for p in LeakDetector(LTA_INP, sensors, pipes).parameters()]
    runs = {name: _adam_trajectory(shapes, env=env, monkeypatch=monkeypatch) for name, env in (
        ("plain", {}), ("skew", {"LEAKGNN_LAB_ADAM_SKEW": "24"}), ("two_launch", {"LEAKGNN_LAB_ADAM_TWO_LAUNCH": "1"}))}
    base = runs["plain"]
    for name, (ps, gs, norms, st) in runs.items():
        assert st[1:3].view(torch.int32).tolist() == [0, 0], f"{name}: counter / error word {st.tolist()}"
        assert st[0].item() == 3
        assert torch.equal(norms, base[2]), f"{name}: norms {norms.tolist()} vs {base[2].tolist()}"
        for k, (p, g) in enumerate(zip(ps, gs)):
            assert torch.equal(p, base[0][k]), f"{name}: param {k} differs"
            assert torch.equal(g, base[1][k]), f"{name}: clipped grad {k} differs"


def test_clip_adamw_two_million_parameters_matches_torch():
    """~2.1M parameters (2,050 slices, more than the CU count: the two-launch form)
    with the clip active, against torch's clip_grad_norm_ + fused AdamW at fp32 rounding."""
    from models.optim import ClipAdamW
    torch.manual_seed(7)
    shapes = [(1024, 1024), (1000,), (1024, 1000), (37, 3), (5,)]
    pa = [torch.randn(s, device=DEV).requires_grad_(True) for s in shapes]
    pb = [p.detach().clone().requires_grad_(True) for p in pa]
    oa = torch.optim.AdamW(pa, lr=1e-2, weight_decay=1e-2, fused=True)
    ob = ClipAdamW(pb, lr=1e-2, weight_decay=1e-2, max_norm=1.0)
    for it in range(3):
        for a, b in zip(pa, pb):
            g = torch.randn_like(a) * (1e-5 if it == 1 else 1.0)
            a.grad, b.grad = g.clone(), g.clone()
        na = torch.nn.utils.clip_grad_norm_(pa, 1.0)
        oa.step()
        ob.step()
        assert_close(ob.last_grad_norm[0], na, rtol=1e-6, what=f"total norm, step {it}")
        for k, (a, b) in enumerate(zip(pa, pb)):
            assert_close(b.grad, a.grad, rtol=1e-6, what=f"clipped grad {k}, step {it}")
            assert_close(b, a, rtol=1e-6, what=f"param {k} after step {it}")
    st = ob.param_groups[0]["step_t"]
    assert st[0].item() == 3 and st[1:3].view(torch.int32).tolist() == [0, 0]


def test_cross_entropy_matches_torch():
    """models/loss.py CrossEntropyLoss (one HIP launch each way) == torch's nn.CrossEntropyLoss:
    loss and dlogits at the detector's shape, with ignored rows, and the all-ignored NaN;
    a non-default configuration falls through to torch.  B = 65,536: 64x
    more rows than the capped grid's waves, so every workgroup loops over many rows before the
    fence-free last-workgroup hand-off (loss.hip header)."""
    from models.loss import CrossEntropyLoss
    torch.manual_seed(3)
    for B, C, n_ign in ((256, 765, 0), (37, 100, 5), (4, 3, 4), (65536, 765, 100)):
        x = torch.randn(B, C, device=DEV) * 3
        t = torch.randint(0, C, (B,), device=DEV)
        t[:n_ign] = -100
        xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
        la = torch.nn.CrossEntropyLoss()(xa, t)
        lb = CrossEntropyLoss()(xb, t)
        if n_ign == B:
            assert torch.isnan(la) and torch.isnan(lb)
            continue
        la.backward()
        lb.backward()
        assert_close(lb, la, rtol=1e-6, what=f"loss B={B}")
        assert_close(xb.grad, xa.grad, rtol=1e-5, what=f"dlogits B={B}")
    x = torch.randn(8, 5, device=DEV)
    t = torch.randint(0, 5, (8,), device=DEV)
    assert_close(CrossEntropyLoss(label_smoothing=0.1)(x, t), torch.nn.CrossEntropyLoss(label_smoothing=0.1)(x, t),
                 rtol=1e-6, what="fallback")


def test_cross_entropy_counter_per_stream():
    """the fused loss forward's completion counter is per (device, stream), so loss
    launches running concurrently on two streams never share tickets: every mean is right and
    both counters are back at 0."""
    from models.loss import CrossEntropyLoss, _counter
    torch.manual_seed(4)
    x = torch.randn(256, 765, device=DEV) * 3
    t = torch.randint(0, 765, (256,), device=DEV)
    ref = torch.nn.functional.cross_entropy(x, t)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream())
    outs = []
    with torch.no_grad():
        for _ in range(25):
            for s in (s1, s2):
                with torch.cuda.stream(s):
                    outs.append(CrossEntropyLoss()(x, t))
    torch.cuda.synchronize()
    for o in outs:
        assert_close(o, ref, rtol=1e-6, what="loss on a concurrent stream")
    c1, c2 = _counter(DEV, s1.cuda_stream), _counter(DEV, s2.cuda_stream)
    assert c1.data_ptr() != c2.data_ptr()
    assert int(c1.item()) == 0 and int(c2.item()) == 0


def test_reduce_batch_matches_per_op_reductions():
    """The backward ops' slab reductions merged into one launch per op group
    (lg_reduce_batch_begin / _flush; the trunk's layer-0 node-bias partials folded into the
    sensor projection's bias reduction) give the same gradients as one reduction launch per
    op: bitwise, except sensor_to_node.bias, whose two partial sets are now summed in one
    fp64 column instead of through a float intermediate."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(3)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train()
    r = torch.randn(64, 36, 29, device=DEV)
    tf = torch.randn(64, 36, 9, device=DEV)
    grads = []
    for batched in (True, False):
        library.REDUCE_BATCH = batched
        try:
            m.zero_grad(set_to_none=True)
            torch.manual_seed(11)
            m(r, tf).square().mean().backward()
            torch.cuda.synchronize()
        finally:
            library.REDUCE_BATCH = True
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for n, g in grads[0].items():
        ref = grads[1][n]
        if n == "sensor_to_node.bias":
            assert_close(g, ref, rtol=1e-6, atol=1e-6 * ref.abs().max().item(), what=n)
        else:
            assert torch.equal(g, ref), f"{n}: batched reduction differs"


@pytest.mark.parametrize("B,npipes", [(3, None), (64, None), (256, None), (300, None), (37, 6), (256, 6)])
def test_fused_pipe_scatter_matches_two_launches(B, npipes):
    """lg_edge_head_bwd_scatter (the incidence scatter fused into the EdgeHead backward, one
    workgroup per window) against lg_edge_head_bwd + lg_pipe_scatter_bwd: the node gradient
    is the same sums in the same order, so every gradient upstream of it (trunk, GRU, sensor
    projection) is bitwise equal; the EdgeHead's weight gradients change only by the slab
    grouping of the fixed-order reduction (window-owned tiles), and so do the NoLeakHead's when
    its backward runs in the streamed launch's prologue (lg_heads_bwd_scatter: windows grouped
    by the edge grid, one per CU, instead of lg_pool_head_bwd's two per CU).  The fused forms run
    a workgroup per window, so only from B = CUs (256 on MI355X) on; below it the call is the
    two launches itself (B = 3: window-major trunk; 64: node-major).  256: the streamed scatter
    (pipe schedule); 300: more windows than CUs (several windows per workgroup); 6 pipes (the
    synthetic training sets): fewer pipe rows than a tile, so the per-window grid is larger
    than the tile grid the workspace used to be sized for."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    if npipes is not None:
        pipes = pipes[:npipes]
    torch.manual_seed(5)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train()
    r = torch.randn(B, 36, 29, device=DEV)
    tf = torch.randn(B, 36, 9, device=DEV)
    grads = []
    saved = library._FUSED_SCATTER
    for fused in (True, False):
        library._FUSED_SCATTER = fused
        try:
            m.zero_grad(set_to_none=True)
            torch.manual_seed(17)
            m(r, tf).square().mean().backward()
            torch.cuda.synchronize()
        finally:
            library._FUSED_SCATTER = saved
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for n, g in grads[0].items():
        ref = grads[1][n]
        if n.startswith("edge_head.") or n.startswith("noleak_head."):
            assert_close(g, ref, rtol=1e-5, atol=1e-6 * ref.abs().max().item(), what=n)
        else:
            assert torch.equal(g, ref), f"{n}: fused scatter differs"


@pytest.mark.parametrize("B", [256, 300])
def test_fused_heads_backward_matches_separate(B):
    """lg_heads_bwd_scatter (the NoLeakHead backward in the streamed EdgeHead backward's
    prologue) against lg_pool_head_bwd + lg_edge_head_bwd_scatter: dpool per window is the same
    sum in the same order, so every gradient but the NoLeakHead's weights is bitwise equal; those
    are bitwise equal at B = 256 (a window per workgroup in both grids) and within rounding at
    B = 300 (windows grouped differently into slab rows)."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    torch.manual_seed(6)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train()
    r = torch.randn(B, 36, 29, device=DEV)
    tf = torch.randn(B, 36, 9, device=DEV)
    grads = []
    saved = library._FUSED_HEADS
    for fused in (True, False):
        library._FUSED_HEADS = fused
        try:
            m.zero_grad(set_to_none=True)
            torch.manual_seed(18)
            m(r, tf).square().mean().backward()
            torch.cuda.synchronize()
        finally:
            library._FUSED_HEADS = saved
        grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    for n, g in grads[0].items():
        ref = grads[1][n]
        if n.startswith("noleak_head.") and B != 256:
            assert_close(g, ref, rtol=1e-5, atol=1e-6 * ref.abs().max().item(), what=n)
        else:
            assert torch.equal(g, ref), f"{n}: fused heads backward differs"


@pytest.mark.parametrize("D", [64, 32])
@pytest.mark.parametrize("B", [256, 300])  # the fused forms need a window per CU (B >= CUs)
def test_streamed_scatter_odd_graph(D, B):
    """The streamed node scatter (ABI 22) on a graph built to hit its corner cases: a hub of
    degree 40 (more incidences than a tile has rows, events with many incidences), a self-loop
    pipe (both roles of one row on one node), nodes without pipes (dh = dpool / N only), windows
    whose last tile is short.  dh must equal lg_edge_head_bwd + lg_pipe_scatter_bwd over the
    schedule's incidence CSR bit for bit; the EdgeHead weight gradients within 1e-5."""
    import ctypes
    from models import _native as nat
    from models import ops
    lib = nat.load_library()
    rng = np.random.default_rng(D + B)
    N = 60
    ring = [(i, i + 1) for i in range(1, 44)]
    hub = [(0, int(j)) for j in rng.permutation(np.arange(1, 45))[:40]]
    ends_np = np.array(ring + hub + [(7, 7)], np.int64)  # nodes 45..59: no pipes
    P = ends_np.shape[0]
    inc = ops.Incidence.build(torch.from_numpy(ends_np), N, DEV)
    sched, hdr = inc.schedule(D)
    assert sched is not None and hdr[9] == N - 45  # the nodes without pipes
    gen = torch.Generator().manual_seed(D * 100 + B)
    h = torch.randn(N, B, D, generator=gen).to(DEV)  # node-major
    W1 = (torch.randn(128, 3 * D, generator=gen) / 8).to(DEV)
    b1 = (torch.randn(128, generator=gen) / 4).to(DEV)
    W2 = (torch.randn(1, 128, generator=gen) / 8).to(DEV)
    b2 = torch.randn(1, generator=gen).to(DEV)
    st = ops.stream_of(h)
    logits = torch.empty(B, P + 1, device=DEV)
    hid = torch.empty(B * P, 128, device=DEV)
    fl = nat.LG_F_NODE_MAJOR | nat.LG_F_DROPOUT
    ops.check(lib.lg_edge_head_fwd(ops.ptr(inc.ends), ops.ptr(h), ops.ptr(W1), ops.ptr(b1), ops.ptr(W2), ops.ptr(b2),
                                   ops.ptr(logits), P + 1, ops.ptr(hid), B, N, P, D, 128, fl, 0.1, 77, 5, st), "fwd")
    dl = torch.randn(B, P + 1, generator=gen).to(DEV)
    dpool = torch.randn(B, D, generator=gen).to(DEV)
    ws = torch.empty(int(lib.lg_edge_head_bwd_workspace_bytes(B, P, D, 128)), device=DEV, dtype=torch.uint8)
    hdr_c = (ctypes.c_int32 * 16)(*hdr)
    outs = []
    for streamed in (True, False):
        dh = torch.full((N, B, D), float("nan"), device=DEV)
        dpipe = torch.empty(B, P, 2, D, device=DEV)
        g = [torch.empty_like(W1), torch.empty_like(b1), torch.empty_like(W2), torch.empty(1, device=DEV)]
        if streamed:
            ops.check(lib.lg_edge_head_bwd_scatter(
                ops.ptr(inc.ends), ops.ptr(h), ops.ptr(W1), ops.ptr(W2), ops.ptr(hid), ops.ptr(dl), P + 1, ops.ptr(dpipe),
                *(ops.ptr(t) for t in g), ops.ptr(inc.rowptr), ops.ptr(inc.item), ops.ptr(sched), hdr_c, ops.ptr(dpool),
                ops.ptr(dh), B, N, P, D, 128, fl, 0.1, ops.ptr(ws), ws.numel(), st), "streamed")
        else:
            ops.check(lib.lg_edge_head_bwd(ops.ptr(inc.ends), ops.ptr(h), ops.ptr(W1), ops.ptr(W2), ops.ptr(hid),
                                           ops.ptr(dl), P + 1, ops.ptr(dpipe), *(ops.ptr(t) for t in g), B, N, P, D,
                                           128, fl, 0.1, ops.ptr(ws), ws.numel(), st), "bwd")
            ops.check(lib.lg_pipe_scatter_bwd(ops.ptr(inc.rowptr), ops.ptr(inc.item), ops.ptr(dpipe), ops.ptr(dpool),
                                              ops.ptr(dh), B, N, P, D, nat.LG_F_NODE_MAJOR, st), "scatter")
        torch.cuda.synchronize()
        outs.append((dh, g))
    assert not torch.isnan(outs[0][0]).any(), "a node row the streamed scatter never wrote"
    assert torch.equal(outs[0][0], outs[1][0]), "streamed dh differs from the two launches"
    for a, c, name in zip(outs[0][1], outs[1][1], ("dW1", "db1", "dW2", "db2")):
        assert_close(a, c, rtol=1e-5, atol=1e-6 * c.abs().max().item(), what=name)
