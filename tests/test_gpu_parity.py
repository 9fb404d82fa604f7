"""HIP path vs the CPU oracle (MI355X).  Every call goes through libleakgnn's C ABI.

Bars: bit-exact for integer / index outputs (CSR, incidence, batchified edge
index); fp32 outputs within RTOL=1e-5 of the oracle's scale (helpers.assert_close).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import (LTA_INP, RTOL, assert_close, assert_grads_close, assert_grads_match_truth, check_relu_ties,
                     hip_relu_masks, load, lta_ids, oracle_grads, oracle_run)
from oracle import gcn_ref, graph_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _native_loaded():
    from models import _native
    return _native.load_library()


def _rand_graph(N, E, seed, loops=True, dups=True):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(0, N, (E,), generator=g)
    dst = torch.randint(0, N, (E,), generator=g)
    if loops:
        src[: max(1, E // 50)] = dst[: max(1, E // 50)]
    if dups and E > 4:
        src[-2:], dst[-2:] = src[:2].clone(), dst[:2].clone()
    return torch.stack([src, dst])


def _check_csr(ei, N, add_loops=True, normalize=True, improved=False):
    from models.ops import GCNGraph
    g = GCNGraph.build(ei, N, DEV, add_self_loops=add_loops, normalize=normalize, improved=improved)
    torch.cuda.synchronize()
    fill = 2.0 if improved else 1.0
    for transpose, (rp, c, w) in ((False, (g.rowptr, g.col, g.w)), (True, (g.rowptr_t, g.col_t, g.w_t))):
        rp_o, c_o, w_o = graph_ref.gcn_csr(ei.numpy(), N, add_loops, normalize, fill, transpose=transpose)
        rp = rp.cpu().numpy()
        nnz = int(rp[-1])
        np.testing.assert_array_equal(rp, rp_o)
        np.testing.assert_array_equal(c.cpu().numpy()[:nnz], c_o)
        np.testing.assert_array_equal(w.cpu().numpy()[:nnz].view(np.uint32), w_o.view(np.uint32))  # bit-exact
    return g


def test_graph_build_bit_exact_ltown_a():
    _native_loaded()
    g = load("graph_ltown_a.npz")
    _check_csr(torch.from_numpy(g["edge_index"]), 661)


def test_graph_build_bit_exact_ltown_full():
    g = load("graph_ltown.npz")
    _check_csr(torch.from_numpy(g["edge_index"]), len(g["node_names"]))


@pytest.mark.parametrize("N,E,add_loops,normalize,improved",
                         [(50, 300, True, True, False), (1000, 7000, True, True, True), (300, 900, False, True, False),
                          (300, 900, True, False, False), (7, 0, True, True, False), (20000, 90000, True, True, False)])
def test_graph_build_bit_exact_random(N, E, add_loops, normalize, improved):
    _check_csr(_rand_graph(N, E, seed=N + E), N, add_loops, normalize, improved)


def test_incidence_and_batchify_bit_exact():
    from models.ops import Incidence, batchify_edge_index
    g = load("graph_ltown_a.npz")
    inc = Incidence.build(torch.from_numpy(g["pipe_ends"]), 661, DEV, schedule=False)
    rp, it = graph_ref.incidence_csr(g["pipe_ends"], 661)
    np.testing.assert_array_equal(inc.rowptr.cpu().numpy(), rp)
    np.testing.assert_array_equal(inc.item.cpu().numpy(), it)
    # the schedule-ordered CSR (ABI 22): the same rows, each node's items reordered
    sinc = Incidence.build(torch.from_numpy(g["pipe_ends"]), 661, DEV)
    np.testing.assert_array_equal(sinc.rowptr.cpu().numpy(), rp)
    sit = sinc.item.cpu().numpy()
    for n in range(661):
        assert sorted(sit[rp[n]:rp[n + 1]]) == list(it[rp[n]:rp[n + 1]])
    out = batchify_edge_index(torch.from_numpy(g["edge_index"]).to(DEV), 661, 3)
    np.testing.assert_array_equal(out.cpu().numpy(), g["batchified_b3"])
    from models.detector import _batchify_edge_index
    big = _batchify_edge_index(torch.from_numpy(g["edge_index"]).to(DEV), 661, 256)
    np.testing.assert_array_equal(big.cpu().numpy(), graph_ref.batchify(g["edge_index"], 661, 256))


@pytest.mark.parametrize("D", [64, 32])
@pytest.mark.parametrize("graph", ["ltown_a_b4", "random"])
def test_gcnconv_fwd_bwd_vs_oracle(D, graph):
    from models.gcn import GCNConv
    if graph == "random":
        N = 3001
        ei = _rand_graph(N, 12000, seed=5)
    else:
        g = load("graph_ltown_a.npz")
        ei = torch.from_numpy(graph_ref.batchify(g["edge_index"], 661, 4))
        N = 4 * 661
    torch.manual_seed(0)
    conv = GCNConv(D, D).to(DEV)
    with torch.no_grad():
        conv.bias.normal_()
    x = torch.randn(N, D)
    xg = x.to(DEV).requires_grad_(True)
    y = conv(xg, ei.to(DEV))
    gy = torch.randn(N, D)
    y.backward(gy.to(DEV))
    xc = x.clone().requires_grad_(True)
    Wc = conv.lin.weight.detach().cpu().clone().requires_grad_(True)
    bc = conv.bias.detach().cpu().clone().requires_grad_(True)
    yc = gcn_ref.gcn_conv(xc, ei, Wc, bc)
    yc.backward(gy)
    assert_close(y, yc, what="GCNConv fwd")
    assert_close(xg.grad, xc.grad, what="GCNConv dx")
    assert_close(conv.lin.weight.grad, Wc.grad, what="GCNConv dW")
    assert_close(conv.bias.grad, bc.grad, what="GCNConv db")


@pytest.mark.parametrize("din,dout", [(48, 80), (64, 16), (32, 64), (96, 96), (7, 5), (64, 128)])
@pytest.mark.parametrize("graph", ["ltown_a_b4", "random"])
def test_gcnconv_general_widths_vs_oracle(din, dout, graph):
    """GCNConv(in, out) at widths the fused kernels do not take (in != out, or not 32 / 64):
    lg_spmm_cols for the propagate (any column count; the bias fused; scalar columns at odd
    widths) and a library GEMM for the transform, against the PyG-semantics oracle, forward and
    all three gradients (1e-5 of each tensor's scale)."""
    from models.gcn import GCNConv
    if graph == "random":
        N = 3001
        ei = _rand_graph(N, 12000, seed=7)
    else:
        g = load("graph_ltown_a.npz")
        ei = torch.from_numpy(graph_ref.batchify(g["edge_index"], 661, 4))
        N = 4 * 661
    torch.manual_seed(din * 1000 + dout)
    conv = GCNConv(din, dout).to(DEV)
    with torch.no_grad():
        conv.bias.normal_()
    x = torch.randn(N, din)
    xg = x.to(DEV).requires_grad_(True)
    y = conv(xg, ei.to(DEV))
    assert y.shape == (N, dout)
    gy = torch.randn(N, dout)
    y.backward(gy.to(DEV))
    xc = x.clone().requires_grad_(True)
    Wc = conv.lin.weight.detach().cpu().clone().requires_grad_(True)
    bc = conv.bias.detach().cpu().clone().requires_grad_(True)
    yc = gcn_ref.gcn_conv(xc, ei, Wc, bc)
    yc.backward(gy)
    assert_close(y, yc, what=f"GCNConv({din},{dout}) fwd")
    assert_close(xg.grad, xc.grad, what=f"GCNConv({din},{dout}) dx")
    assert_close(conv.lin.weight.grad, Wc.grad, what=f"GCNConv({din},{dout}) dW")
    assert_close(conv.bias.grad, bc.grad, what=f"GCNConv({din},{dout}) db")


def test_spmm_cols_strided_and_empty_rows():
    """lg_spmm_cols through the C ABI: row strides wider than C, no bias, a graph whose last rows
    have only their self loop, and C = 0 / N = 0 (no launch); against the oracle's propagate."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    N = 500
    ei = _rand_graph(N - 50, 2000, seed=3)  # nodes 450..499: self loops only
    graph = GCNGraph.build(ei, N, DEV)
    for C, ld in ((40, 44), (13, 13), (64, 72)):
        x = torch.randn(N, ld)
        xd = x.to(DEV)
        y = torch.full((N, ld + 4), 7.0, device=DEV)
        ops.check(lib.lg_spmm_cols(ops.ptr(graph.rowptr), ops.ptr(graph.col), ops.ptr(graph.w), ops.ptr(xd), ld, None,
                                   ops.ptr(y), ld + 4, N, C, ops.stream_of(xd)), "spmm_cols")
        torch.cuda.synchronize()
        yc = gcn_ref.gcn_conv(x[:, :C].contiguous(), ei, torch.eye(C), None)
        assert_close(y[:, :C], yc, what=f"spmm_cols C={C} ld={ld}")
        assert torch.all(y[:, C:] == 7.0), "columns past C untouched"
    for n_, c_ in ((0, 8), (N, 0)):
        assert lib.lg_spmm_cols(ops.ptr(graph.rowptr), ops.ptr(graph.col), ops.ptr(graph.w), ops.ptr(xd), 64, None,
                                ops.ptr(y), 64, n_, c_, ops.stream_of(xd)) == 0


def test_spmm_vs_oracle_and_linearity():
    from models.ops import GCNGraph, spmm
    g = load("graph_ltown_a.npz")
    ei = torch.from_numpy(g["edge_index"])
    graph = GCNGraph.build(ei, 661, DEV)
    B = 16
    x = torch.randn(B, 661, 64)
    y = spmm(graph, x.to(DEV), B=B)
    eib = torch.from_numpy(graph_ref.batchify(g["edge_index"], 661, B))
    yc = gcn_ref.gcn_conv(x.reshape(-1, 64), eib, torch.eye(64), None).reshape(B, 661, 64)
    assert_close(y, yc, what="spmm")
    x2 = torch.randn(B, 661, 64, device=DEV)
    assert_close(spmm(graph, x.to(DEV) + 2 * x2, B), y + 2 * spmm(graph, x2, B), rtol=1e-5, what="linearity")


def _product_model(state: dict, B_dropout=0.1):
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=B_dropout)
    m.load_state_dict({k[len("param."):]: torch.from_numpy(v) for k, v in state.items() if k.startswith("param.")})
    return m.to(DEV)


@pytest.mark.parametrize("fixture", ["detector_b2.npz", "detector_b8.npz"])
def test_detector_vs_reference_fixture(fixture):
    """Eval-mode forward within 1e-5 of the reference fixture; grads vs fp64 truth (helpers)."""
    state = load("detector_b2.npz")
    fx = load(fixture)
    m = _product_model(state).eval()
    residual = torch.from_numpy(fx["residual"]).to(DEV).requires_grad_(True)
    logits = m(residual, torch.from_numpy(fx["tfeat"]).to(DEV))
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["label"]).to(DEV))
    loss.backward()
    assert_close(logits, fx["logits"], what="logits")
    assert abs(loss.item() - float(fx["loss"])) <= RTOL * abs(float(fx["loss"]))
    assert_close(residual.grad, fx["grad_residual"], what="grad residual")
    sd = {k[len("param."):]: torch.from_numpy(v) for k, v in state.items() if k.startswith("param.")}
    args = (fx["residual"], fx["tfeat"], fx["label"])
    _, g32 = oracle_grads(sd, *(torch.from_numpy(a) for a in args), torch.float32)
    _, g64 = oracle_grads(sd, *(torch.from_numpy(a) for a in args), torch.float64)
    for n in g32:  # the fixture (reference code, fp32) and the oracle fp32 agree
        assert_close(g32[n], fx["grad." + n], what="oracle vs fixture grad " + n)
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64)


@pytest.mark.parametrize("schedule", [True, False])
def test_detector_vs_oracle_b64_random_weights(schedule):
    """B=64, random weights (schedule: the pipe-schedule order of the EdgeHead backward's node
    sums, the default; False: the reference's ascending incidence order, per-window scatter)."""
    _b64_vs_oracle(schedule)


def _b64_vs_oracle(schedule: bool):
    """B=64, random weights.  Forward within 1e-5 of the oracle; backward driven by ONE
    fixed upstream gradient dL/dlogits (the fp64 cross-entropy gradient of the oracle's
    logits) fed to both paths, so the comparison covers the detector and not torch's
    GPU-vs-CPU cross-entropy (whose softmax normalisation error lands in the
    cancellation-heavy EdgeHead output-bias gradient).  Gradients against the fp64 truth on
    the HIP path's side of every ReLU / |h_u - h_v| kink (see test_gpu_configs.py's B = 256
    tests: a pre-activation within rounding of 0 falls either way in any fp32 evaluation)."""
    sensors, pipes = lta_ids()
    from oracle.detector_ref import LeakDetectorRef
    torch.manual_seed(11)
    ref = LeakDetectorRef(LTA_INP, sensors, pipes).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    from models.detector import LeakDetector
    m = LeakDetector(LTA_INP, sensors, pipes)
    m.incidence_schedule = schedule
    m = m.to(DEV).eval()
    m.load_state_dict(sd)
    B = 64
    gen = torch.Generator().manual_seed(12)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, 765, (B,), generator=gen)
    _, _, pre64, upstream = oracle_run(sd, r, tf, torch.float64, "cpu", lab=lab)
    m.capture = {}
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(upstream.float().to(DEV))
    masks = hip_relu_masks(m.capture, B, len(m.node_names), len(pipes), m.pipe_ends)
    check_relu_ties(pre64, masks)
    _, g64, _, _ = oracle_run(sd, r, tf, torch.float64, "cpu", up=upstream, masks=masks)
    o32, g32, _, _ = oracle_run(sd, r, tf, torch.float32, "cpu", up=upstream, masks=masks)
    assert_close(lg, o32, what="logits B=64")
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64)


def test_detector_c4_graph_vs_oracle(tmp_path):
    """C4 topology (synthetic 10k-node / 15k-pipe .inp, node_hidden = sensor_hidden = 32).
    Its CSR (≈0.3 MB) is too big for LDS, so this covers the global-CSR variants of the
    masked trunk kernels (ReLU / dropout backward flags) and the D = 32 heads.  B = 3,
    random weights, eval mode; same bars as the B = 64 test."""
    from models.synth import pick_sensors, write_synthetic_inp
    from oracle.detector_ref import LeakDetectorRef
    from models.detector import LeakDetector
    inp = tmp_path / "c4.inp"
    node_ids, pipe_ids = write_synthetic_inp(inp, 10_000, 15_000, seed=0)
    sensors = pick_sensors(node_ids, 29, seed=0)
    kw = dict(sensor_hidden=32, node_hidden=32)
    torch.manual_seed(21)
    ref = LeakDetectorRef(inp, sensors, pipe_ids, **kw).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    m = LeakDetector(inp, sensors, pipe_ids, **kw).to(DEV).eval()
    m.load_state_dict(sd)
    B = 3
    gen = torch.Generator().manual_seed(22)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipe_ids) + 1, (B,), generator=gen)
    grads, logits = {}, {}
    for dt in (torch.float64, torch.float32):
        mr = LeakDetectorRef(inp, sensors, pipe_ids, **kw).eval()
        mr.load_state_dict(sd)
        mr = mr.to(dt)
        logits[dt] = mr(r.to(dt), tf.to(dt))
        if dt == torch.float64:
            lg64 = logits[dt].detach().requires_grad_(True)
            torch.nn.functional.cross_entropy(lg64, lab).backward()
            upstream = lg64.grad.clone()
        logits[dt].backward(upstream.to(dt))
        grads[dt] = {n: p.grad.detach() for n, p in mr.named_parameters()}
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(upstream.float().to(DEV))
    assert_close(lg, logits[torch.float32], what="logits C4")
    # slack 8: the conv-bias grads are 30k-row sums with heavy cancellation, and ReLU masks
    # of pre-activations within fp32 roundoff of 0 differ between any two fp32 orderings
    # (CPU vs GPU), so the per-tensor fp32 error varies more than at L-TOWN-A size.
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, grads[torch.float32],
                             grads[torch.float64], slack=8.0)


def test_detector_c4_graph_b64_vs_oracle(tmp_path):
    """C4 at the bench's per-rank batch (BASELINE configs[3]: B = 64 windows per rank, D = 32,
    10k nodes / 15k pipes), eval mode: B >= 16 runs the NODE-MAJOR trunk kernels at D = 32
    (the B = 3 test above covers the window-major ones).  Logits within 1e-5 of the fp32
    oracle; gradients vs the fp64 oracle evaluated on the HIP run's own ReLU decisions
    (hip_relu_masks, as the L-TOWN-A B = 64 test), bounded by 4x the fp32 oracle's error
    (CPU or GPU torch) or 5e-5 of the tensor's scale."""
    from models.synth import pick_sensors, write_synthetic_inp
    from oracle.detector_ref import LeakDetectorRef
    from models.detector import LeakDetector
    from models import ops
    inp = tmp_path / "c4.inp"
    node_ids, pipe_ids = write_synthetic_inp(inp, 10_000, 15_000, seed=0)
    sensors = pick_sensors(node_ids, 29, seed=0)
    kw = dict(sensor_hidden=32, node_hidden=32)
    net = (inp, sensors, pipe_ids, kw)
    torch.manual_seed(23)
    ref = LeakDetectorRef(inp, sensors, pipe_ids, **kw).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    m = LeakDetector(inp, sensors, pipe_ids, **kw).to(DEV).eval()
    m.load_state_dict(sd)
    B = 64
    assert ops.use_node_major(B, len(m.node_names), 32)
    gen = torch.Generator().manual_seed(24)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipe_ids) + 1, (B,), generator=gen)
    _, _, pre64, upstream = oracle_run(sd, r, tf, torch.float64, "cpu", lab=lab, net=net)
    m.capture = {}
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(upstream.float().to(DEV))
    masks = hip_relu_masks(m.capture, B, len(m.node_names), len(pipe_ids), m.pipe_ends)
    check_relu_ties(pre64, masks)
    _, g64, _, _ = oracle_run(sd, r, tf, torch.float64, "cpu", up=upstream, masks=masks, net=net)
    o32, g32, _, _ = oracle_run(sd, r, tf, torch.float32, "cpu", up=upstream, masks=masks, net=net)
    assert_close(lg, o32, what="logits C4 B=64")
    # EdgeHead dW sums B * P = 960k rows: yardstick also torch fp32 on the GPU, tensor bar 5e-5
    # (as the B = 256 train-mode test, test_gpu_configs.py)
    _, g32d, _, _ = oracle_run(sd, r, tf, torch.float32, DEV, up=upstream, masks=masks, net=net)
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64, ref32=g32d, rtol_tensor=5e-5)


def test_detector_train_mode_dropout():
    state = load("detector_b2.npz")
    m = _product_model(state).train()
    B = 32
    r = torch.randn(B, 36, 29, device=DEV)
    tf = torch.randn(B, 36, 9, device=DEV)
    torch.manual_seed(5)
    a = m(r, tf)
    torch.manual_seed(5)
    b = m(r, tf)
    assert torch.equal(a, b), "dropout must be a pure function of torch's seed"
    c = m(r, tf)
    assert not torch.equal(a, c)
    # dropout p=0 in train mode == eval mode (up to the eval-mode parity bar)
    m0 = _product_model(state, B_dropout=0.0).train()
    me = _product_model(state).eval()
    assert_close(m0(r, tf), me(r, tf), what="p=0 train vs eval")
    # kept fraction of the node-init activations ~ 1 - p
    from models import ops
    x0 = torch.ones(4, 661, 64, device=DEV)
    slot = torch.full((661,), -1, dtype=torch.int32, device=DEV)
    lib = ops.load_library()
    ops.check(lib.lg_node_init_fwd(ops.ptr(slot), None, ops.ptr(torch.ones(64, device=DEV)), ops.ptr(x0), 4, 661, 0,
                                   64, ops.nat.LG_F_DROPOUT, 0.1, 1234, 0, ops.stream_of(x0)), "node_init")
    kept = (x0 > 0).float().mean().item()
    assert abs(kept - 0.9) < 0.01
    assert_close(x0[x0 > 0], torch.full_like(x0[x0 > 0], 1 / 0.9), what="dropout scale")


def _masks(seed: int, salt: int, shape, p: float, dev=DEV) -> torch.Tensor:
    from oracle.dropout_ref import keep_mask
    idx = np.arange(int(np.prod(shape)), dtype=np.uint64).reshape(shape)
    return torch.from_numpy(keep_mask(seed, salt, idx, p).astype(np.float32)).to(dev)


def test_detector_train_mode_replay_with_oracle_masks():
    """Train mode end to end: every dropout mask of the HIP path (node init, both GCN
    layers, EdgeHead hidden) is regenerated on the host by oracle/dropout_ref.py and the
    whole detector is replayed with explicit torch ops; forward and all grads must agree."""
    from models import ops
    state = load("detector_b2.npz")
    m = _product_model(state).train()
    B, N, D, P = 6, 661, 64, 764
    r = torch.randn(B, 36, 29, device=DEV)
    tf = torch.randn(B, 36, 9, device=DEV)
    torch.manual_seed(9)
    out = m(r, tf)
    out.square().sum().backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    torch.manual_seed(9)
    seed_t = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item())   # gnn_trunk draw
    seed_h = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item())   # detector_heads draw
    sc = 1.0 / 0.9
    R = B * N
    from oracle.dropout_ref import row_stream_mask
    mk = [   # node init (salt 0) and the GCN layers (salts 1, 2): row streams
        torch.from_numpy(row_stream_mask(seed_t, l, np.arange(R), D, 0.1).astype(np.float32)).to(DEV)
        for l in (0, 1, 2)]
    from oracle.dropout_ref import edge_stream_mask
    me = torch.from_numpy(edge_stream_mask(seed_h, ops.EDGE_HEAD_SALT, np.arange(B * P), 0.1)
                          .astype(np.float32)).to(DEV)   # EdgeHead: row streams
    ei = torch.from_numpy(graph_ref.batchify(m.edge_index_single.numpy(), N, B))
    row, col, w = (t.to(DEV) for t in gcn_ref.gcn_norm(ei, R))
    h_s = m.sensor_encoder(r, tf)
    Wn, bn = m.sensor_to_node.weight, m.sensor_to_node.bias
    h0 = torch.zeros(B, N, 64, device=DEV)
    h0[:, m.sensor_node_idx.to(DEV)] = h_s
    mask = torch.zeros(N, 1, device=DEV)
    mask[m.sensor_node_idx.to(DEV)] = 1
    x = (torch.relu(torch.cat([h0, mask.expand(B, -1, -1)], -1) @ Wn.t() + bn).reshape(R, D)) * mk[0] * sc
    for l, conv in enumerate(m.convs):
        hh = x @ conv.lin.weight.t()
        agg = torch.zeros_like(hh).index_add_(0, col, w.view(-1, 1) * hh[row])
        x = torch.relu(agg + conv.bias) * mk[l + 1] * sc
    hn = x.view(B, N, D)
    u, v = m.pipe_ends[:, 0].to(DEV), m.pipe_ends[:, 1].to(DEV)
    feat = torch.cat([hn[:, u], hn[:, v], (hn[:, u] - hn[:, v]).abs()], -1).reshape(B * P, 3 * D)
    mlp = m.edge_head.mlp
    hid = torch.relu(feat @ mlp[0].weight.t() + mlp[0].bias) * me * sc
    pl = (hid @ mlp[3].weight.t() + mlp[3].bias).view(B, P)
    mn = _masks(seed_h, ops.NOLEAK_HEAD_SALT, (B, 128), 0.1)
    nm = m.noleak_head.mlp
    nl = (torch.relu(hn.mean(1) @ nm[0].weight.t() + nm[0].bias) * mn * sc) @ nm[3].weight.t() + nm[3].bias
    out2 = torch.cat([pl, nl], -1)
    assert_close(out, out2, what="train-mode forward replay")
    out2.square().sum().backward()
    # both sides are fp32 GPU with different summation orders; a mask/structure bug is O(1)
    assert_grads_close(list(grads.items()), {n: p.grad for n, p in m.named_parameters()}, rtol=1e-4,
                       prefix="train grad ")


@pytest.mark.parametrize("B", [1, 37, 256])
@pytest.mark.parametrize("D", [64, 32])
@pytest.mark.parametrize("drop", [False, True])
def test_gcn_node_major_matches_window_major(B, D, drop):
    """lg_gcn_fwd_nm / lg_gcn_bwd_nm on [N][B][D] vs lg_gcn_fwd / lg_gcn_bwd on [B][N][D]
    (themselves oracle-checked above).  Forward with LG_F_F32_MFMA bit-exact (same entry
    order, same MFMA order, same row-stream dropout masks), with the default split-bf16
    transform within 1e-6 of the output scale; backward dx bit-exact-or-1e-5, dW / db / node
    bias (different reduction trees) within 1e-5.  B = 37 leaves a ragged window group."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    g = load("graph_ltown_a.npz")
    N = 661
    graph = GCNGraph.build(torch.from_numpy(g["edge_index"]), N, DEV)
    gen = torch.Generator().manual_seed(B * 7 + D + drop)
    x = torch.randn(B, N, D, generator=gen).relu().to(DEV)  # trunk inputs are post-ReLU
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    flags = ops.nat.LG_F_BIAS | ops.nat.LG_F_RELU | (ops.nat.LG_F_DROPOUT if drop else 0)
    p, seed, salt = (0.1 if drop else 0.0), 987654321, 2
    st = ops.stream_of(x)
    y = torch.empty_like(x)
    ops.check(lib.lg_gcn_fwd(ops.ptr(graph.rowptr), ops.ptr(graph.col), ops.ptr(graph.w), ops.ptr(x), ops.ptr(W),
                             ops.ptr(b), ops.ptr(y), B, N, D, graph.nnz_cap, flags, p, seed, salt, st), "fwd")
    xn = x.transpose(0, 1).contiguous()
    yn = torch.empty_like(xn)
    F32 = ops.nat.LG_F_F32_MFMA
    ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                ops.ptr(yn), B, N, D, graph.nnz_cap, flags | F32, p, seed, salt, st), "fwd_nm")
    assert torch.equal(yn.transpose(0, 1), y), "node-major forward (f32 MFMA) must match the window-major kernel bit for bit"
    scale = yn.abs().amax().item()

    def run(fl):
        out = torch.empty_like(xn)
        ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                    ops.ptr(out), B, N, D, graph.nnz_cap, flags | fl, p, seed, salt, st), "fwd_nm")
        return out
    # default transform (pc, 2-way fp16 split): fp32-level accuracy, bar 1e-6 of the output scale
    ys = run(0)
    err = (ys.double() - yn.double()).abs().max().item()
    assert err <= 1e-6 * scale, f"default transform off by {err:.3e} (scale {scale:.3e})"
    # the 3-way bf16 split: the same bits in both pipelines, fp32-level accuracy (1e-6 of the scale:
    # the MFMA's K order differs from the exact-fp32 reference's)
    y3 = run(ops.nat.LG_F_BF16X3)
    assert torch.equal(run(ops.nat.LG_F_NM3), y3), "pc and nm3 3-way split transforms must agree bit for bit"
    err3 = (y3.double() - yn.double()).abs().max().item()
    assert err3 <= 1e-6 * scale, f"3-way split off by {err3:.3e} (scale {scale:.3e})"
    # backward with both masks and the node-bias sum
    slot = torch.full((N,), -1, dtype=torch.int32)
    slot[torch.randperm(N, generator=gen)[:29]] = torch.arange(29, dtype=torch.int32)
    slot = slot.to(DEV)
    dy = torch.randn(B, N, D, generator=gen).to(DEV)
    sc = 1.0 / 0.9 if drop else 1.0
    bflags = ops.nat.LG_F_MASK_IN | ops.nat.LG_F_MASK_OUT
    outs = []
    for nm in (False, True):
        xx, yy, dd = (xn, yn, dy.transpose(0, 1).contiguous()) if nm else (x, y, dy)
        dx = torch.empty_like(xx)
        dW, db, dnb = (torch.empty(D, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV))
        if nm:
            ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            ops.check(lib.lg_gcn_bwd_nm(ops.ptr(graph.nodetab_t), ops.ptr(graph.pairs_t), ops.ptr(dd), ops.ptr(yy),
                                        ops.ptr(xx), ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db),
                                        ops.ptr(slot), ops.ptr(dnb), B, N, D, bflags, sc, sc, ops.ptr(ws), ws.numel(), st),
                      "bwd_nm")
            dx = dx.transpose(0, 1)
        else:
            ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            ops.check(lib.lg_gcn_bwd(ops.ptr(graph.rowptr_t), ops.ptr(graph.col_t), ops.ptr(graph.w_t), ops.ptr(dd),
                                     ops.ptr(yy), ops.ptr(xx), ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db),
                                     ops.ptr(slot), ops.ptr(dnb), B, N, D, graph.nnz_cap, bflags, sc, sc,
                                     ops.ptr(ws), ws.numel(), st), "bwd")
        outs.append((dx, dW, db, dnb))
    for a, r, n in zip(outs[1], outs[0], ("dx", "dW", "db", "dnode_bias")):
        assert_close(a, r, what=f"node-major {n}")


@pytest.mark.parametrize("train", [False, True])
def test_detector_node_major_matches_window_major(train, monkeypatch):
    """The whole detector (train mode: same dropout masks) in both trunk layouts."""
    from models import ops
    state = load("detector_b2.npz")
    m = _product_model(state).train(train)
    B = 40
    r = torch.randn(B, 36, 29, device=DEV)
    tf = torch.randn(B, 36, 9, device=DEV)
    res = []
    for nm in (False, True):
        monkeypatch.setattr(ops, "TRUNK_NODE_MAJOR", nm)
        m.zero_grad()
        torch.manual_seed(3)
        out = m(r, tf)
        out.square().sum().backward()
        res.append((out.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    assert_close(res[1][0], res[0][0], what="logits node-major vs window-major")
    assert_grads_close(list(res[1][1].items()), res[0][1], prefix="layout grad ")


@pytest.mark.parametrize("nm", [False, True])
@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("D", [64, 32])
def test_fused_heads_vs_torch(train, D, nm):
    """leakgnn::detector_heads (fused EdgeHead, mean pool + NoLeakHead, one (B, P+1) output,
    incidence-reduced backward) vs float64 torch with the same dropout masks
    (oracle/dropout_ref.py)."""
    _heads_case(train, D, nm, 5)


@pytest.mark.parametrize("D", [64, 32])
def test_fused_heads_multi_tile(D):
    """B = 70 (53,480 pipe rows): every workgroup of both EdgeHead kernels runs several tiles
    (prefetch pipeline, LDS buffer parity) and the last tile is ragged."""
    _heads_case(True, D, True, 70)


def _heads(inc, p, nm, params, keep=True):
    """leakgnn::detector_heads on (h, W1, b1, W2, b2, V1, c1, V2, c2); the seed drawn as the
    detector draws it (torch's CPU generator), logits only."""
    from models import library
    seed = library.seed_tensor(DEV) if p > 0 else torch.zeros(1, dtype=torch.long)
    return torch.ops.leakgnn.detector_heads(*params, inc.ends, inc.rowptr, inc.item, p, p, nm, keep, seed)[0]


def test_edge_head_eval_without_hidden():
    """No-grad forward passes hid = NULL (nothing kept for a backward); logits unchanged."""
    from models.ops import Incidence
    g = load("graph_ltown_a.npz")
    inc = Incidence.build(torch.from_numpy(g["pipe_ends"]), 661, DEV)
    gen = torch.Generator().manual_seed(3)
    ps = [torch.randn(*s, generator=gen).to(DEV) / 8 for s in
          ((4, 661, 64), (128, 192), (128,), (1, 128), (1,), (128, 64), (128,), (1, 128), (1,))]
    a = _heads(inc, 0.0, False, ps, keep=False)
    ps[1].requires_grad_(True)
    b = _heads(inc, 0.0, False, ps, keep=True)
    assert torch.equal(a, b.detach())


@pytest.mark.parametrize("wide", [False, True])
def test_edge_fwd_f16x2_transform_accuracy(wide):
    """The EdgeHead forward's default fp32-tier transform at D = 64 (2-way f16 split, W1 scaled
    per wave, features per pipe row) and the 3-way bf16 split (LG_F_BF16X3) both within 1e-6
    of each row's hidden-layer scale of the float64 product; `wide` spreads the node rows
    over 2^-12 .. 2^12 so a per-row scale that failed to follow its row would show."""
    from models import ops
    nat = ops.nat
    lib = ops.load_library()
    g = load("graph_ltown_a.npz")
    ends = torch.from_numpy(g["pipe_ends"]).long()
    B, N, P, D = 37, 661, 764, 64
    gen = torch.Generator().manual_seed(13 + wide)
    h = torch.randn(B, N, D, generator=gen)
    if wide:
        h = h * torch.exp2(torch.randint(-12, 13, (B, N, 1), generator=gen).float())
    W1 = torch.randn(128, 3 * D, generator=gen) / 8
    b1 = torch.randn(128, generator=gen) / 4
    W2 = torch.randn(128, generator=gen) / 8
    b2 = torch.randn(1, generator=gen)
    u, v = ends[:, 0], ends[:, 1]
    hd = h.double()
    feat = torch.cat([hd[:, u], hd[:, v], (hd[:, u] - hd[:, v]).abs()], -1).reshape(B * P, 3 * D)
    pre = feat @ W1.double().t()
    ref = torch.relu(pre + b1.double())
    # per-row bound: the products' magnitude |feat| |W1| (the f16 split drops <= 2^-22 of it)
    scale = (feat.abs() @ W1.double().abs().t()).amax(1, keepdim=True) + b1.double().abs().max()
    hs, e, w1d, b1d, w2d, b2d = (t.to(DEV) for t in (h, ends, W1, b1, W2, b2))  # alive across the launch
    for fl in (0, nat.LG_F_BF16X3):
        logits = torch.empty(B, P, device=DEV)
        hid = torch.full((B * P, 128), float("nan"), device=DEV)
        ops.check(lib.lg_edge_head_fwd(ops.ptr(e), ops.ptr(hs), ops.ptr(w1d), ops.ptr(b1d), ops.ptr(w2d), ops.ptr(b2d),
                                       ops.ptr(logits), P, ops.ptr(hid), B, N, P, D, 128, fl, 0.0, 0, 0,
                                       ops.stream_of(hs)), "edge fwd")
        torch.cuda.synchronize()
        err = ((hid.cpu().double() - ref).abs() / scale).max().item()
        assert err <= 1e-6, f"flags {fl:#x}: hidden layer err {err:.3e} of the row scale"
        lr = (ref @ W2.double() + b2.double()).view(B, P)
        assert_close(logits, lr, rtol=1e-5, what=f"logits flags {fl:#x}")


def _heads_case(train, D, nm, B):
    from models import ops
    from models.ops import Incidence
    g = load("graph_ltown_a.npz")
    ends = torch.from_numpy(g["pipe_ends"])
    inc = Incidence.build(ends, 661, DEV)
    N, P = 661, 764
    gen = torch.Generator().manual_seed(D + train)
    h = torch.randn(B, N, D, generator=gen)
    h[0, :40] = 0.25  # ties -> |h_u - h_v| = 0, sign 0
    W1 = torch.randn(128, 3 * D, generator=gen) / 8
    b1 = torch.randn(128, generator=gen) / 4
    W2 = torch.randn(1, 128, generator=gen) / 8
    b2 = torch.randn(1, generator=gen)
    V1 = torch.randn(128, D, generator=gen) / 8
    c1 = torch.randn(128, generator=gen) / 4
    V2 = torch.randn(1, 128, generator=gen) / 8
    c2 = torch.randn(1, generator=gen)
    dl = torch.randn(B, P + 1, generator=gen)
    params = [t.to(DEV).requires_grad_(True) for t in (h, W1, b1, W2, b2, V1, c1, V2, c2)]
    if nm:  # node-major input (N, B, D): the grad is compared in the same layout below
        params[0] = h.transpose(0, 1).contiguous().to(DEV).requires_grad_(True)
    torch.manual_seed(77)
    logits = _heads(inc, 0.1 if train else 0.0, nm, params)
    (logits * dl.to(DEV)).sum().backward()
    # float64 reference with the same dropout masks
    ref = [t.double().requires_grad_(True) for t in (h, W1, b1, W2, b2, V1, c1, V2, c2)]
    hr, W1r, b1r, W2r, b2r, V1r, c1r, V2r, c2r = ref
    u, v = ends[:, 0], ends[:, 1]
    feat = torch.cat([hr[:, u], hr[:, v], (hr[:, u] - hr[:, v]).abs()], -1)
    hid = torch.relu(feat @ W1r.t() + b1r)
    pooled = hr.mean(1)
    nhid = torch.relu(pooled @ V1r.t() + c1r)
    if train:
        torch.manual_seed(77)
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item())
        from oracle.dropout_ref import edge_stream_mask
        me = torch.from_numpy(edge_stream_mask(seed, ops.EDGE_HEAD_SALT, np.arange(B * P), 0.1))
        hid = hid * me.double().view(B, P, 128) / 0.9
        nhid = nhid * _masks(seed, ops.NOLEAK_HEAD_SALT, (B, 128), 0.1, dev="cpu").double() / 0.9
    lr = torch.cat([(hid @ W2r.t()).squeeze(-1) + b2r, nhid @ V2r.t() + c2r], -1)
    (lr * dl.double()).sum().backward()
    assert_close(logits, lr, what="head logits")
    for a, b, n in zip(params, ref, ("dh", "dW1", "db1", "dW2", "db2", "dV1", "dc1", "dV2", "dc2")):
        ga = a.grad.transpose(0, 1) if (nm and n == "dh") else a.grad
        assert_close(ga, b.grad, rtol=2e-5, what=n)


def test_pipe_features_kernel():
    from models.ops import Incidence, pipe_features
    g = load("graph_ltown_a.npz")
    inc = Incidence.build(torch.from_numpy(g["pipe_ends"]), 661, DEV)
    h = torch.randn(3, 661, 64, device=DEV)
    e = torch.from_numpy(g["pipe_ends"]).to(DEV)
    hu, hv = h[:, e[:, 0]], h[:, e[:, 1]]
    assert torch.equal(pipe_features(h, inc), torch.cat([hu, hv, (hu - hv).abs()], -1))


def test_full_size_properties_c5():
    """C5-size graph (100k nodes / 300k edge columns): size-independent checks.
    Ahat is symmetric for an undirected graph, so <Ahat x, z> == <x, Ahat z>;
    CSR == transposed CSR for a symmetric edge set."""
    from models.ops import GCNGraph, spmm
    from models.synth import synthetic_pipe_graph
    ei, _ = synthetic_pipe_graph(100_000, 150_000, seed=0)
    graph = GCNGraph.build(ei, 100_000, DEV)
    x = torch.randn(1, 100_000, 64, device=DEV, dtype=torch.float32)
    z = torch.randn(1, 100_000, 64, device=DEV, dtype=torch.float32)
    a = (spmm(graph, x) * z).double().sum()
    b = (x * spmm(graph, z)).double().sum()
    assert abs(a.item() - b.item()) <= 1e-5 * abs(a.item()) + 1e-2
    nnz = int(graph.rowptr[-1].item())
    assert nnz == 300_000 + 100_000
    # Ahat = D^-1/2 (A+I) D^-1/2 has sqrt(deg) as an eigenvector with eigenvalue 1
    # (deg counts the self loop): a size-independent check of every row sum.
    deg = graph.rowptr.diff().double()
    v = deg.sqrt().float().reshape(1, -1, 1).expand(1, 100_000, 64).contiguous()
    assert_close(spmm(graph, v), v, rtol=1e-5, what="Ahat sqrt(deg) = sqrt(deg)")
    # linearity on the full size
    assert_close(spmm(graph, x + 2 * z), spmm(graph, x) + 2 * spmm(graph, z), rtol=1e-5, what="C5 linearity")
    assert torch.equal(graph.rowptr, graph.rowptr_t)
    # per-row multiset equality of neighbours (orders differ: in-edge vs out-edge order)
    c, ct = graph.col[:nnz].long(), graph.col_t[:nnz].long()
    rows = torch.repeat_interleave(torch.arange(100_000, device=DEV), graph.rowptr.diff().long())
    k1 = torch.sort(rows * 100_000 + c).values
    k2 = torch.sort(rows * 100_000 + ct).values
    assert torch.equal(k1, k2)


@pytest.mark.parametrize("use_time,dx,H", [(True, True, 64), (False, True, 64), (True, False, 64),
                                             (False, False, 64), (True, False, 32)])
@pytest.mark.parametrize("B", [5, 64])
def test_gru_encoder_vs_torch_cpu(use_time, dx, H, B):
    """Fused HIP GRU vs nn.GRU on the CPU (the reference's own op), fwd h_L and all grads.
    dx=False is the detector's training case (the residual is data): the split-bf16
    backward k_gru_bwd2 (32 sequences per workgroup; B = 5 leaves a ragged last one);
    dx=True runs the fp32 kernel that also writes d residual / d tfeat."""
    from models.detector import SharedSensorGRUEncoder
    from oracle.detector_ref import _GRUEncoder
    torch.manual_seed(B)
    ref = _GRUEncoder(H, use_time=use_time)
    with torch.no_grad():
        for p in ref.parameters():
            p.uniform_(-0.3, 0.3)
    enc = SharedSensorGRUEncoder(hidden_size=H, use_time=use_time)
    enc.gru.load_state_dict(ref.gru.state_dict())
    enc = enc.to(DEV)
    gen = torch.Generator().manual_seed(3)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    gy = torch.randn(B, 29, H, generator=gen)
    rc, tc = r.clone().requires_grad_(dx), tf.clone().requires_grad_(use_time and dx)
    yc = ref(rc, tc if use_time else None)
    (yc * gy).sum().backward()
    rg, tg = r.to(DEV).requires_grad_(dx), tf.to(DEV).requires_grad_(use_time and dx)
    yg = enc(rg, tg if use_time else None)
    (yg * gy.to(DEV)).sum().backward()
    assert_close(yg, yc, what="GRU h_L")
    if dx:
        assert_close(rg.grad, rc.grad, what="GRU d residual")
    if use_time and dx:
        assert_close(tg.grad, tc.grad, what="GRU d tfeat")
    assert_grads_close([(n, p.grad) for n, p in enc.gru.named_parameters()],
                       {n: p.grad for n, p in ref.gru.named_parameters()}, prefix="GRU grad ")


@pytest.mark.parametrize("gscale,wmax,H", [(1e-9, 0.3, 64), (1e6, 0.3, 64), (1.0, 0.5, 64), (1.0, 1.0, 64),
                                            (3e-5, 1.0, 32)])
def test_gru_bwd_f16x2_scales(gscale, wmax, H):
    """The training backward (k_gru_bwd2 on the f16x2 split) keeps fp32-level accuracy when the
    incoming gradient is tiny or huge (the per-step dG scale follows it: bound from the previous
    step's maxima) and with larger weights, whose dh grows or shrinks fast over the 36 steps.
    Judged against the fp64 truth (nn.GRU in float64 on the CPU): every gradient within 4x the
    fp32 CPU reference's own error or 1e-5 of its scale.  At +-1 and H = 64 the recurrence
    amplifies rounding (any fp32 evaluation is ~1e-3 of the gradient off fp64, r04n2), so a
    direct GPU-vs-fp32-CPU comparison measures the CPU's error as much as the kernel's."""
    from models.detector import SharedSensorGRUEncoder
    from oracle.detector_ref import _GRUEncoder
    from helpers import assert_grads_match_truth
    torch.manual_seed(7)
    ref = _GRUEncoder(H, use_time=True)
    with torch.no_grad():
        for p in ref.parameters():
            p.uniform_(-wmax, wmax)
    enc = SharedSensorGRUEncoder(hidden_size=H, use_time=True)
    enc.gru.load_state_dict(ref.gru.state_dict())
    enc = enc.to(DEV)
    gen = torch.Generator().manual_seed(11)
    B = 40
    r = torch.randn(B, 36, 29, generator=gen) * 3.0
    tf = torch.randn(B, 36, 9, generator=gen)
    gy = torch.randn(B, 29, H, generator=gen) * gscale
    grads = {}
    for dt in (torch.float32, torch.float64):
        m = _GRUEncoder(H, use_time=True)
        m.load_state_dict(ref.state_dict())
        m = m.to(dt)
        (m(r.to(dt), tf.to(dt)) * gy.to(dt)).sum().backward()
        grads[dt] = {n: p.grad.detach() for n, p in m.gru.named_parameters()}
    (enc(r.to(DEV), tf.to(DEV)) * gy.to(DEV)).sum().backward()
    assert_grads_match_truth({n: p.grad for n, p in enc.gru.named_parameters()}, grads[torch.float32],
                             grads[torch.float64])


@pytest.mark.parametrize("K,M,N", [(7424, 64, 64), (1857, 32, 32), (3, 64, 32), (250, 32, 64)])
def test_linear_dw_vs_fp64(K, M, N):
    """lg_linear_dw (node-init Linear weight grad on [x, 1] rows) vs float64 torch, ragged K."""
    from models import ops
    lib = ops.load_library()
    gen = torch.Generator().manual_seed(K + M + N)
    dy = torch.randn(K, M, generator=gen)
    x = torch.randn(K, N, generator=gen)
    dw = torch.empty(M, N + 1, device=DEV)
    db = torch.empty(M, device=DEV)
    ws = torch.empty(int(lib.lg_linear_dw_workspace_bytes(K, M, N)), device=DEV, dtype=torch.uint8)
    dyg, xg = dy.to(DEV), x.to(DEV)
    ops.check(lib.lg_linear_dw(ops.ptr(dyg), ops.ptr(xg), K, M, N, ops.ptr(dw), ops.ptr(db), ops.ptr(ws), ws.numel(),
                               ops.stream_of(dyg)), "lg_linear_dw")
    ref = torch.cat([dy.double().t() @ x.double(), dy.double().sum(0, keepdim=True).t()], 1)
    assert_close(dw, ref, what="dW")
    assert_close(db, ref[:, N], what="db")


@pytest.mark.parametrize("D", [64, 32])
def test_gcn_node_major_high_degree_graph(D):
    """Node-major forward on a random graph with hubs (degree up to ~40, past the kernel's
    prefetched neighbours), isolated nodes and duplicate edges: bit-exact with the
    window-major kernel, which is oracle-checked on random graphs above."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    gen = torch.Generator().manual_seed(77 + D)
    N, E, B = 300, 2400, 40
    src = torch.randint(0, N - 20, (E,), generator=gen)
    dst = torch.where(torch.rand(E, generator=gen) < 0.3, torch.randint(0, 5, (E,), generator=gen),
                      torch.randint(0, N - 20, (E,), generator=gen))  # nodes 0..4 are hubs; N-20.. isolated
    graph = GCNGraph.build(torch.stack([src, dst]), N, DEV)
    x = torch.randn(B, N, D, generator=gen).to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    st = ops.stream_of(x)
    for flags in (ops.nat.LG_F_BIAS | ops.nat.LG_F_RELU | ops.nat.LG_F_DROPOUT, ops.nat.LG_F_BIAS):
        y = torch.empty_like(x)
        ops.check(lib.lg_gcn_fwd(ops.ptr(graph.rowptr), ops.ptr(graph.col), ops.ptr(graph.w), ops.ptr(x), ops.ptr(W),
                                 ops.ptr(b), ops.ptr(y), B, N, D, graph.nnz_cap, flags, 0.2, 5, 3, st), "fwd")
        xn = x.transpose(0, 1).contiguous()
        yn = torch.empty_like(xn)
        ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                    ops.ptr(yn), B, N, D, graph.nnz_cap, flags | ops.nat.LG_F_F32_MFMA, 0.2, 5, 3, st),
                  "fwd_nm")
        assert torch.equal(yn.transpose(0, 1), y)
        ys = torch.empty_like(xn)
        ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                    ops.ptr(ys), B, N, D, graph.nnz_cap, flags, 0.2, 5, 3, st), "fwd_nm split")
        assert (ys.double() - yn.double()).abs().max().item() <= 1e-6 * yn.abs().amax().item()


@pytest.mark.parametrize("drop", [False, True])
def test_gcn_node_major_schedule_order_changes_no_result(drop):
    """The node table's schedule section (reverse Cuthill-McKee order, lg_rcm_order) only
    reorders tiles: forward y and backward dx are bit-identical to the node-order schedule;
    dW / db / node bias (other slab groupings) within 1e-6 of scale."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    N, B, D = 661, 48, 64
    graph = GCNGraph.build(torch.from_numpy(load("graph_ltown_a.npz")["edge_index"]), N, DEV)
    assert not torch.equal(graph.order.cpu(), torch.arange(N, dtype=torch.int32))
    st = ops.stream_of(graph.w)
    tab_id, tab_id_t = torch.empty_like(graph.nodetab), torch.empty_like(graph.nodetab_t)
    ops.check(lib.lg_nm_table_build(ops.ptr(graph.rowptr), ops.ptr(graph.pairs), N, None, ops.ptr(tab_id), st), "t")
    ops.check(lib.lg_nm_table_build(ops.ptr(graph.rowptr_t), ops.ptr(graph.pairs_t), N, None, ops.ptr(tab_id_t), st),
              "t")
    gen = torch.Generator().manual_seed(5 + drop)
    x = torch.randn(N, B, D, generator=gen).relu().to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    dy = torch.randn(N, B, D, generator=gen).to(DEV)
    slot = torch.full((N,), -1, dtype=torch.int32)
    slot[:29] = torch.arange(29, dtype=torch.int32)
    slot = slot.to(DEV)
    flags = ops.nat.LG_F_BIAS | ops.nat.LG_F_RELU | (ops.nat.LG_F_DROPOUT if drop else 0)
    p = 0.1 if drop else 0.0
    res = []
    for tab, tab_t in ((graph.nodetab, graph.nodetab_t), (tab_id, tab_id_t)):
        y = torch.empty_like(x)
        ops.check(lib.lg_gcn_fwd_nm(ops.ptr(tab), ops.ptr(graph.pairs), ops.ptr(x), ops.ptr(W), ops.ptr(b), ops.ptr(y),
                                    B, N, D, graph.nnz_cap, flags, p, 77, 1, st), "fwd")
        dx = torch.empty_like(x)
        dW, db, dnb = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
        sc = 1.0 / 0.9 if drop else 1.0
        ops.check(lib.lg_gcn_bwd_nm(ops.ptr(tab_t), ops.ptr(graph.pairs_t), ops.ptr(dy), ops.ptr(y), ops.ptr(x),
                                    ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db), ops.ptr(slot), ops.ptr(dnb), B, N,
                                    D, ops.nat.LG_F_MASK_IN | ops.nat.LG_F_MASK_OUT, sc, sc, ops.ptr(ws), ws.numel(), st), "bwd")
        torch.cuda.synchronize()
        res.append((y, dx, dW, db, dnb))
    assert torch.equal(res[0][0], res[1][0]), "schedule order changed the forward"
    assert torch.equal(res[0][1], res[1][1]), "schedule order changed dx"
    for k, name in ((2, "dW"), (3, "db"), (4, "node bias")):
        assert_close(res[0][k], res[1][k], rtol=1e-6, atol=1e-7, what=name)


@pytest.mark.parametrize("D,B", [(64, 48), (32, 37)])
def test_gcn_node_major_mask_bits_equal_y_gather(D, B):
    """lg_gcn_fwd_nm_bits writes [y > 0] as bits beside the same y; lg_gcn_bwd_nm_bits with
    those bits (y passed as NULL) gives dx bit for bit equal to the y-gather backward (dW, db
    and the node bias within 1e-6).  B = 37 leaves a ragged window group."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    N = 661
    graph = GCNGraph.build(torch.from_numpy(load("graph_ltown_a.npz")["edge_index"]), N, DEV)
    st = ops.stream_of(graph.w)
    gen = torch.Generator().manual_seed(D + B)
    x = torch.randn(N, B, D, generator=gen).relu().to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    dy = torch.randn(N, B, D, generator=gen).to(DEV)
    slot = torch.full((N,), -1, dtype=torch.int32)
    slot[:29] = torch.arange(29, dtype=torch.int32)
    slot = slot.to(DEV)
    flags = ops.nat.LG_F_BIAS | ops.nat.LG_F_RELU | ops.nat.LG_F_DROPOUT
    y, y2 = torch.empty_like(x), torch.empty_like(x)
    bits = torch.zeros(N * ((B + 15) // 16) * 64, dtype=torch.int16, device=DEV)
    ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(x), ops.ptr(W), ops.ptr(b),
                                ops.ptr(y), B, N, D, graph.nnz_cap, flags, 0.1, 99, 2, st), "fwd")
    ops.check(lib.lg_gcn_fwd_nm_bits(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(x), ops.ptr(W), ops.ptr(b),
                                     ops.ptr(y2), B, N, D, graph.nnz_cap, flags, 0.1, 99, 2, st, ops.ptr(bits)), "fwd bits")
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    # the bits restate [y > 0] in the gather layout (lane l: row (64/(D/4)) k + l/(D/4), cols 4 (l % (D/4)) + i)
    lpr = D // 4
    rpi = 64 // lpr
    bb = bits.view(N, (B + 15) // 16, 64).to(torch.int32).cpu() & 0xFFFF
    yc = (y.cpu() > 0)
    for g in range((B + 15) // 16):
        for lane in (0, 5, lpr - 1, 63):
            for k in range(16 // rpi):
                row = g * 16 + rpi * k + lane // lpr
                if row >= B:
                    continue
                for i in range(4):
                    want = yc[:, row, 4 * (lane % lpr) + i]
                    got = ((bb[:, g, lane] >> (4 * k + i)) & 1).bool()
                    assert torch.equal(got, want), (g, lane, k, i)
    sc = 1.0 / 0.9
    outs = []
    for use_bits in (False, True):
        dx = torch.empty_like(x)
        dW, db, dnb = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
        ops.check(lib.lg_gcn_bwd_nm_bits(ops.ptr(graph.nodetab_t), ops.ptr(graph.pairs_t), ops.ptr(dy),
                                         None if use_bits else ops.ptr(y), ops.ptr(x), ops.ptr(W), ops.ptr(dx),
                                         ops.ptr(dW), ops.ptr(db), ops.ptr(slot), ops.ptr(dnb), B, N, D,
                                         ops.nat.LG_F_MASK_IN | ops.nat.LG_F_MASK_OUT, sc, sc, ops.ptr(ws), ws.numel(), st,
                                         ops.ptr(bits) if use_bits else None), "bwd")
        torch.cuda.synchronize()
        outs.append((dx, dW, db, dnb))
    assert torch.equal(outs[0][0], outs[1][0]), "dx: mask bits differ from the y gather"
    for a, c, name in zip(outs[0][1:], outs[1][1:], ("dW", "db", "node bias")):  # slab grouping may differ
        assert_close(c, a, rtol=1e-6, atol=1e-7, what=name)


@pytest.mark.parametrize("D,B", [(64, 256), (64, 37), (32, 40)])
def test_gcn_bwd_dx_sensor_rows_only(D, B):
    """LG_F_DX_SENSOR_ROWS (ABI 20, layer 0's backward in the detector): the sensor rows of dx
    are bit for bit those of the full backward, the non-sensor rows are left as they were
    (sentinel), and dW / db / node-bias sums are bitwise unchanged (same tiles, same order)."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    N = 661
    graph = GCNGraph.build(torch.from_numpy(load("graph_ltown_a.npz")["edge_index"]), N, DEV)
    st = ops.stream_of(graph.w)
    gen = torch.Generator().manual_seed(7 * D + B)
    x = torch.randn(N, B, D, generator=gen).relu().to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    dy = torch.randn(N, B, D, generator=gen).to(DEV)
    slot = torch.full((N,), -1, dtype=torch.int32)
    sens = torch.randperm(N, generator=gen)[:29]
    slot[sens] = torch.arange(29, dtype=torch.int32)
    slot = slot.to(DEV)
    sc = 1.0 / 0.9
    outs = []
    for only in (False, True):
        dx = torch.full_like(x, 12345.0)
        dW, db, dnb = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
        flags = ops.nat.LG_F_MASK_OUT | (ops.nat.LG_F_DX_SENSOR_ROWS if only else 0)
        ops.check(lib.lg_gcn_bwd_nm_bits(ops.ptr(graph.nodetab_t), ops.ptr(graph.pairs_t), ops.ptr(dy), None,
                                         ops.ptr(x), ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db), ops.ptr(slot),
                                         ops.ptr(dnb), B, N, D, flags, sc, sc, ops.ptr(ws), ws.numel(), st, None), "bwd")
        torch.cuda.synchronize()
        outs.append((dx, dW, db, dnb))
    full, part = outs
    sens_d = sens.to(DEV)
    assert torch.equal(part[0][sens_d], full[0][sens_d]), "sensor rows of dx changed"
    keep = torch.ones(N, dtype=torch.bool, device=DEV)
    keep[sens_d] = False
    assert bool((part[0][keep] == 12345.0).all()), "non-sensor rows of dx were written"
    for a, c, name in zip(full[1:], part[1:], ("dW", "db", "node bias")):
        assert torch.equal(a, c), name
