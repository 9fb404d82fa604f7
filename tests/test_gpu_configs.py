"""GPU parity at the BASELINE.json configs the round-1 suite did not cover (SURVEY §8 d):

  configs[4] / C5  synthetic 100k nodes / 300k edge columns, D = 64, one graph, fwd + bwd:
                   GCNConv (the single-graph row-tile kernels lg_gcn_{fwd,bwd}_rows, and the
                   window-major ones at D = 32) vs the fp64 oracle, the node-major trunk
                   kernels vs the oracle directly, and one full LeakDetector (S = 29,
                   P = 150,000) forward + backward vs the oracle;
  configs[2]       L-TOWN-A detector at its own batch, B = 256, vs the CPU oracle in eval
                   mode, and in train mode with every dropout mask regenerated on the host
                   by oracle/dropout_ref.py and fed to a CPU replay of the oracle;
  configs[1]       the predictor at B = 64 on the GPU (stock torch modules).

Plus the drop-in robustness checks of this round: autocast / half inputs, dropout under a
plain torch.cuda.graph capture, the GCNConv CSR cache on a recycled edge_index address.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import (LTA_INP, RTOL, assert_close, assert_grads_match_truth, check_relu_ties, hip_relu_masks, load,
                     lta_ids, oracle_run)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


# ----------------------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5_graph():
    from models.synth import synthetic_pipe_graph
    ei, _ = synthetic_pipe_graph(100_000, 150_000, seed=0)
    return ei


def test_c5_gcnconv_fwd_bwd_vs_oracle(c5_graph):
    """GCNConv(64, 64) on the C5 graph (N = 100,000, 300,000 edge columns + self loops):
    output within 1e-5 of the CPU oracle; dx, dW, db vs an fp64 oracle run, bounded by
    4x the fp32 CPU oracle's own error or 1e-5 of scale (helpers.assert_grads_match_truth)."""
    from models.gcn import GCNConv
    from oracle.gcn_ref import GCNConvRef
    N, D = 100_000, 64
    torch.manual_seed(5)
    ref = GCNConvRef(D, D)
    with torch.no_grad():
        ref.bias.normal_(0, 0.1)
    conv = GCNConv(D, D).to(DEV)
    conv.load_state_dict(ref.state_dict())
    gen = torch.Generator().manual_seed(6)
    x = torch.randn(N, D, generator=gen)
    dy = torch.randn(N, D, generator=gen)
    xg = x.to(DEV).requires_grad_(True)
    y = conv(xg, c5_graph.to(DEV))
    y.backward(dy.to(DEV))
    outs, grads = {}, {}
    for dt in (torch.float32, torch.float64):
        r = GCNConvRef(D, D)
        r.load_state_dict(ref.state_dict())
        r = r.to(dt)
        xr = x.detach().to(dt).clone().requires_grad_(True)
        o = r(xr, c5_graph)
        o.backward(dy.to(dt))
        outs[dt] = o.detach()
        grads[dt] = {"x": xr.grad, "lin.weight": r.lin.weight.grad, "bias": r.bias.grad}
    assert_close(y, outs[torch.float64], what="C5 GCNConv forward")
    gpu = {"x": xg.grad, "lin.weight": conv.lin.weight.grad, "bias": conv.bias.grad}
    assert_grads_match_truth(gpu, grads[torch.float32], grads[torch.float64])


@pytest.mark.parametrize("drop", [False, True])
def test_c5_node_major_trunk_kernels(c5_graph, drop):
    """lg_gcn_fwd_nm / lg_gcn_bwd_nm at C5 size (N = 100,000, B = 16 windows: 1.6M rows)
    against the window-major kernels that the previous test pins to the oracle: forward
    bit-exact on the exact-fp32 transform and within 1e-6 on the split-bf16 one; backward
    (masked, both flags) within 1e-5 of scale."""
    from models import ops
    from models.ops import GCNGraph
    lib = ops.load_library()
    nat = ops.nat
    N, D, B = 100_000, 64, 16
    graph = GCNGraph.build(c5_graph, N, DEV)
    gen = torch.Generator().manual_seed(7)
    x = torch.relu(torch.randn(B, N, D, generator=gen)).to(DEV)
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    st = ops.stream_of(x)
    flags = nat.LG_F_BIAS | nat.LG_F_RELU | (nat.LG_F_DROPOUT if drop else 0)
    y = torch.empty_like(x)
    ops.check(lib.lg_gcn_fwd(ops.ptr(graph.rowptr), ops.ptr(graph.col), ops.ptr(graph.w), ops.ptr(x), ops.ptr(W),
                             ops.ptr(b), ops.ptr(y), B, N, D, graph.nnz_cap, flags, 0.1, 77, 2, st), "fwd")
    xn = x.transpose(0, 1).contiguous()
    yn = torch.empty_like(xn)
    ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                ops.ptr(yn), B, N, D, graph.nnz_cap, flags | nat.LG_F_F32_MFMA, 0.1, 77, 2, st),
              "fwd_nm f32")
    assert torch.equal(yn.transpose(0, 1), y)
    ys = torch.empty_like(xn)
    ops.check(lib.lg_gcn_fwd_nm(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(W), ops.ptr(b),
                                ops.ptr(ys), B, N, D, graph.nnz_cap, flags, 0.1, 77, 2, st), "fwd_nm split")
    assert (ys.double() - yn.double()).abs().max().item() <= 1e-6 * yn.abs().amax().item()
    # backward: dy random, masks from y (this layer) and x (the previous op)
    dy = torch.randn(B, N, D, generator=gen).to(DEV)
    bflags = nat.LG_F_MASK_IN | nat.LG_F_MASK_OUT
    sc = 1.0 / 0.9 if drop else 1.0
    outs = {}
    for nm in (False, True):
        dx = torch.empty(N, B, D, device=DEV) if nm else torch.empty_like(x)
        dW, db = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV)
        if nm:
            ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            ops.check(lib.lg_gcn_bwd_nm(ops.ptr(graph.nodetab_t), ops.ptr(graph.pairs_t),
                                        ops.ptr(dy.transpose(0, 1).contiguous()), ops.ptr(yn), ops.ptr(xn), ops.ptr(W),
                                        ops.ptr(dx), ops.ptr(dW), ops.ptr(db), None, None, B, N, D, bflags, sc, sc,
                                        ops.ptr(ws), ws.numel(), st), "bwd_nm")
            dx = dx.transpose(0, 1)
        else:
            ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
            ops.check(lib.lg_gcn_bwd(ops.ptr(graph.rowptr_t), ops.ptr(graph.col_t), ops.ptr(graph.w_t), ops.ptr(dy),
                                     ops.ptr(y), ops.ptr(x), ops.ptr(W), ops.ptr(dx), ops.ptr(dW), ops.ptr(db), None,
                                     None, B, N, D, graph.nnz_cap, bflags, sc, sc, ops.ptr(ws), ws.numel(), st), "bwd")
        outs[nm] = (dx, dW, db)
    for i, what in enumerate(("dx", "dW", "db")):
        assert_close(outs[True][i], outs[False][i], what=f"C5 node-major bwd {what}")


@pytest.mark.parametrize("drop", [False, True])
def test_c5_node_major_trunk_vs_fp64_oracle(c5_graph, drop):
    """The node-major trunk kernels the product runs at B >= 16 (lg_gcn_fwd_nm_bits default:
    producer / consumer waves, 2-way fp16 split transform; lg_gcn_bwd_nm_bits) at C5 size
    (N = 100,000, 300,000 edge columns + self loops, B = 16, D = 64) against the oracle's
    GCNConv arithmetic (oracle/gcn_ref.py gcn_norm / gcn_conv) in fp64 DIRECTLY, with the
    dropout keep mask regenerated by oracle/dropout_ref.py.  Forward within 1e-5 of scale,
    mask bits == [y64 > 0] away from ties; backward (ReLU/dropout of this layer and of the
    previous op, from the forward's mask bits) dx, dW, db within 1e-5 of scale."""
    from models import ops
    from models.ops import GCNGraph
    from oracle.dropout_ref import row_stream_mask
    from oracle.gcn_ref import gcn_norm
    lib = ops.load_library()
    nat = ops.nat
    N, D, B, p, seed, salt = 100_000, 64, 16, 0.1, 91, 2
    graph = GCNGraph.build(c5_graph, N, DEV)
    gen = torch.Generator().manual_seed(17)
    xw = torch.relu(torch.randn(B, N, D, generator=gen))               # window-major truth layout
    W = torch.randn(D, D, generator=gen) / 8
    b = torch.randn(D, generator=gen) / 4
    dy = torch.randn(B, N, D, generator=gen)
    sc = 1.0 / (1.0 - p) if drop else 1.0
    # fp64 truth (gcn_conv: h = x W^T; out[col] += w h[row]; + b), batched over windows
    row, col, w = gcn_norm(c5_graph, N, dtype=torch.float64)
    h = (xw.double() @ W.double().t()).transpose(0, 1).reshape(N, B * D)
    z64 = torch.zeros(N, B * D, dtype=torch.float64).index_add_(0, col, w.view(-1, 1) * h.index_select(0, row))
    z64 = z64.view(N, B, D) + b.double()
    keep = torch.ones(N, B, D, dtype=torch.float64)
    if drop:  # row b * N + n of the disjoint union (the kernels' dropout row index)
        rows = (np.arange(B)[None, :] * N + np.arange(N)[:, None]).reshape(-1)
        keep = torch.from_numpy(row_stream_mask(seed, salt, rows, D, p).reshape(N, B, D)).double()
    y64 = torch.relu(z64) * keep * sc
    del h
    # the product kernels, node-major [N][B][D]
    xn = xw.transpose(0, 1).contiguous().to(DEV)
    Wd, bd = W.to(DEV), b.to(DEV)
    st = ops.stream_of(xn)
    flags = nat.LG_F_BIAS | nat.LG_F_RELU | (nat.LG_F_DROPOUT if drop else 0)
    ng = (B + 15) // 16
    yn = torch.empty_like(xn)
    ybits = torch.zeros(N * ng * 64, dtype=torch.int16, device=DEV)
    ops.check(lib.lg_gcn_fwd_nm_bits(ops.ptr(graph.nodetab), ops.ptr(graph.pairs), ops.ptr(xn), ops.ptr(Wd),
                                     ops.ptr(bd), ops.ptr(yn), B, N, D, graph.nnz_cap, flags, p, seed, salt, st,
                                     ops.ptr(ybits)), "fwd_nm_bits")
    y = yn.cpu()
    assert_close(y, y64, what="C5 node-major forward vs fp64 oracle")
    pos = y > 0
    tie = (z64.abs() <= 1e-5 * z64.abs().max()).logical_and(keep > 0)
    assert torch.equal(pos[~tie], (y64 > 0)[~tie]), "ReLU/dropout decisions differ away from ties"
    # backward, masks on the HIP run's side of every kink
    dz64 = dy.double().transpose(0, 1) * pos.double() * sc                                   # [N, B, D]
    t64 = torch.zeros(N, B * D, dtype=torch.float64).index_add_(
        0, row, w.view(-1, 1) * dz64.reshape(N, B * D).index_select(0, col)).view(N, B, D)   # Ahat^T dz
    xin = xw.double().transpose(0, 1)
    dx64 = (t64 @ W.double()) * (xin > 0).double() * sc
    dW64 = t64.reshape(-1, D).t() @ xin.reshape(-1, D)
    db64 = dz64.reshape(-1, D).sum(0)
    dyn = dy.transpose(0, 1).contiguous().to(DEV)
    dx = torch.empty_like(xn)
    dW, db = torch.empty(D, D, device=DEV), torch.empty(D, device=DEV)
    ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=DEV, dtype=torch.uint8)
    ops.check(lib.lg_gcn_bwd_nm_bits(ops.ptr(graph.nodetab_t), ops.ptr(graph.pairs_t), ops.ptr(dyn), None,
                                     ops.ptr(xn), ops.ptr(Wd), ops.ptr(dx), ops.ptr(dW), ops.ptr(db), None, None, B,
                                     N, D, nat.LG_F_MASK_IN | nat.LG_F_MASK_OUT, sc, sc, ops.ptr(ws), ws.numel(), st,
                                     ops.ptr(ybits)), "bwd_nm_bits")
    assert_close(dx, dx64, what="C5 node-major dx vs fp64 oracle")
    assert_close(dW, dW64, what="C5 node-major dW vs fp64 oracle")
    assert_close(db, db64, what="C5 node-major db vs fp64 oracle")


def test_c5_detector_vs_oracle(tmp_path):
    """One full LeakDetector on the C5 network written as an EPANET .inp (100,000 nodes,
    150,000 pipes, S = 29 sensors, P = 150,000 pipe classes), B = 1, eval mode, random
    weights: logits within 1e-5 of the CPU oracle; parameter gradients for one fixed
    upstream gradient vs the fp64 oracle (same bars as the L-TOWN-A tests)."""
    from models.detector import LeakDetector
    from models.synth import pick_sensors, write_synthetic_inp
    from oracle.detector_ref import LeakDetectorRef
    inp = tmp_path / "c5.inp"
    node_ids, pipe_ids = write_synthetic_inp(inp, 100_000, 150_000, seed=0)
    sensors = pick_sensors(node_ids, 29, seed=0)
    torch.manual_seed(31)
    ref = LeakDetectorRef(inp, sensors, pipe_ids).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    m = LeakDetector(inp, sensors, pipe_ids).to(DEV).eval()
    m.load_state_dict(sd)
    gen = torch.Generator().manual_seed(32)
    r = torch.randn(1, 36, 29, generator=gen)
    tf = torch.randn(1, 36, 9, generator=gen)
    up = torch.randn(1, len(pipe_ids) + 1, generator=gen) / 100
    logits, grads = {}, {}
    for dt in (torch.float32, torch.float64):
        mr = LeakDetectorRef(inp, sensors, pipe_ids).eval()
        mr.load_state_dict(sd)
        mr = mr.to(dt)
        lg = mr(r.to(dt), tf.to(dt))
        lg.backward(up.to(dt))
        logits[dt] = lg.detach()
        grads[dt] = {n: p.grad.detach() for n, p in mr.named_parameters()}
    lg = m(r.to(DEV), tf.to(DEV))
    assert lg.shape == (1, 150_001)
    lg.backward(up.to(DEV))
    # the no-leak logit pools a mean over 100,000 nodes: the fp32 reference itself is off
    # from the fp64 truth by more than 1e-5 of scale there, so the bar is against the fp64
    # run: within 1e-5 of scale, or within 2x the fp32 reference's own error
    t64 = logits[torch.float64]
    e_ref = (logits[torch.float32].double() - t64).abs().max().item()
    e_gpu = (lg.detach().double().cpu() - t64).abs().max().item()
    assert e_gpu <= max(RTOL * t64.abs().max().item() + 1e-7, 2 * e_ref), (e_gpu, e_ref)
    assert_close(lg[:, :-1], t64[:, :-1], what="C5 pipe logits")
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, grads[torch.float32],
                             grads[torch.float64])


# ----------------------------------------------------------------------------- configs[2] at B = 256
def lta_pipes_p382(pipes):
    """configs[2] with the reference example's `--pipe_sample_ratio 0.5` (cmd.sh:10): 382 of the
    764 pipes, picked as leak_generation.py:90-99 does (models/synth.pick_pipes)."""
    from models.synth import pick_pipes
    from models.utils import parse_epanet_inp
    inp_order = [ln.split()[0] for ln in parse_epanet_inp(LTA_INP)["PIPES"]]
    sub = pick_pipes(inp_order, 0.5, seed=198)
    assert len(sub) == 382 and set(sub) <= set(pipes)
    return sub


def _random_ref(seed: int, pipes=None):
    from oracle.detector_ref import LeakDetectorRef
    sensors, all_pipes = lta_ids()
    pipes = all_pipes if pipes is None else pipes
    torch.manual_seed(seed)
    ref = LeakDetectorRef(LTA_INP, sensors, pipes).eval()
    with torch.no_grad():
        for c in ref.convs:
            c.bias.normal_(0, 0.1)
    return {k: v.clone() for k, v in ref.state_dict().items()}


@pytest.mark.parametrize("P", [764, 382])
def test_detector_b256_eval_vs_oracle(P):
    """P = 764 (every pipe) and P = 382 (cmd.sh:10's --pipe_sample_ratio 0.5: a different pipe
    schedule, 12 pipe tiles per window instead of 24).  L-TOWN-A at the bench batch (B = 256, node-major trunk), eval mode, random weights:
    logits within 1e-5 of the oracle; grads for the oracle's fp64 CE gradient vs fp64 truth
    on the same side of every kink.  A ReLU pre-activation within fp32 rounding of 0, or an
    h_u - h_v of two nodes with (near-)identical features behind |h_u - h_v|, may fall
    either way in ANY fp32 evaluation; one such unit moves a gradient by a whole term
    (measured: 8 sign ties of h_u - h_v put torch fp32 2e-2 off fp64 in the GRU input
    gradient).  check_relu_ties proves every differing decision is such a tie, then the
    fp64 truth and the fp32 yardsticks are all evaluated on the HIP path's side."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    if P == 382:
        pipes = lta_pipes_p382(pipes)
    net = (LTA_INP, sensors, pipes, {})
    sd = _random_ref(41, pipes)
    B = 256
    gen = torch.Generator().manual_seed(42)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen)
    _, _, pre64, up = oracle_run(sd, r, tf, torch.float64, "cpu", lab=lab, net=net)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    m.load_state_dict(sd)
    m.capture = {}
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(up.float().to(DEV))
    masks = hip_relu_masks(m.capture, B, len(m.node_names), len(pipes), m.pipe_ends)
    check_relu_ties(pre64, masks)
    # truth and fp32 yardsticks all on the HIP path's side of every kink
    _, g64, _, _ = oracle_run(sd, r, tf, torch.float64, "cpu", up=up, masks=masks, net=net)
    o32, g32, _, _ = oracle_run(sd, r, tf, torch.float32, "cpu", up=up, masks=masks, net=net)
    _, g32d, _, _ = oracle_run(sd, r, tf, torch.float32, DEV, up=up, masks=masks, net=net)
    assert_close(lg, o32, what="B=256 logits")
    # The CE gradient makes dW1 of the EdgeHead and the conv bias grads the difference of two
    # sums over ~2e5 rows that nearly cancel (the label rows against all the others): per
    # tensor 5e-5 of scale, or 4x the error of the reference arithmetic in fp32 (torch on the
    # CPU or on this GPU); the whole-vector 2-norm bar stays at 1e-5
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64, ref32=g32d, rtol_tensor=5e-5)


def test_bf16_tier_b256():
    """BASELINE configs[2] as written ("bf16 node-MLP on MFMA"): LeakDetector(mlp_dtype="bf16")
    at B = 256 against the fp64 oracle.  Its bar is SURVEY §7's: logits within 2e-2 of their
    scale.  Gradients for a dense random upstream gradient, against the fp64 truth, are held
    to the reference model's own bf16 arithmetic: torch.autocast(bfloat16) of the oracle on
    this GPU sets the yardstick (per tensor and whole vector: at most 3x its error, or 1e-2;
    measured: whole vector 6.8e-2 against autocast's 4.4e-2, conv grads ~1.7e-1 against
    ~8.8e-2 — the tier rounds the aggregated features where autocast rounds x).
    bf16 rounding of the pre-activations moves ReLU decisions, so ~1e-1 gradient errors are
    the nature of the tier, not a kernel defect.  (Not the CE gradient of a random-init
    model: its parameter gradients are differences of sums that cancel to ~1e-3 of their
    terms, and bf16 rounding moves thousands of ReLU decisions, so no bf16 evaluation is
    within 1e-1 of them — measured: EdgeHead db1 99 % off while the kernels agree with the
    fp32 ones to 0.25 % on the same hidden layer, tools/diag_bf16.py.)  A train-mode step
    with dropout is finite."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    sd = _random_ref(41)
    B = 256
    gen = torch.Generator().manual_seed(42)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen)
    up = torch.randn(B, len(pipes) + 1, generator=gen, dtype=torch.float64) / B
    o64, g64, _, _ = oracle_run(sd, r, tf, torch.float64, "cpu", up=up)
    m = LeakDetector(LTA_INP, sensors, pipes, mlp_dtype="bf16").to(DEV).eval()
    m.load_state_dict(sd)
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(up.float().to(DEV))
    err = (lg.detach().double().cpu() - o64.double()).abs().max().item()
    scale = o64.abs().max().item()
    print(f"bf16 tier: logits max err {err:.3e} of scale {scale:.3e} ({err / scale:.2e})")
    assert err <= 2e-2 * scale
    _, gac, _, _ = oracle_run(sd, r, tf, torch.float32, DEV, up=up, autocast=True)
    num = den = nac = 0.0
    bad = []
    for n, p in m.named_parameters():
        t = g64[n].double()
        t2 = (t ** 2).sum().item()
        d = ((p.grad.double().cpu() - t) ** 2).sum().item()
        da = ((gac[n].double() - t) ** 2).sum().item()
        rel, rel_ac = (d / max(t2, 1e-300)) ** 0.5, (da / max(t2, 1e-300)) ** 0.5
        print(f"  {n:40s} rel 2-norm err {rel:.2e}   torch autocast-bf16 {rel_ac:.2e}")
        if rel > max(3 * rel_ac, 1e-2):
            bad.append(n)
        num, den, nac = num + d, den + t2, nac + da
    print(f"  whole vector rel 2-norm err {(num / den) ** 0.5:.2e}   torch autocast-bf16 {(nac / den) ** 0.5:.2e}")
    assert num <= max(9 * nac, 1e-4 * den)
    assert not bad, bad
    # train mode (dropout) step
    m.train()
    m.zero_grad(set_to_none=True)
    loss = torch.nn.functional.cross_entropy(m(r.to(DEV), tf.to(DEV)), lab.to(DEV))
    loss.backward()
    assert np.isfinite(loss.item()) and all(torch.isfinite(p.grad).all() for p in m.parameters())


def _replay_train_cpu(sd: dict, r, tf, seeds: tuple, dt, up, dev="cpu", masks=None, aux=None):
    """The oracle detector (reference detector.py:170-218 op for op) in train mode on the
    CPU, with every dropout mask the HIP path draws regenerated by oracle/dropout_ref.py
    from the same seeds: node init (per-element hash), GCN layers (row streams), EdgeHead
    hidden (row streams), NoLeakHead hidden (per-element hash).  Returns logits, grads for
    the upstream gradient `up`, the ReLU pre-activations and the dropout keep masks per
    site; masks: ReLU decisions to use instead of the pre-activations' signs; aux: a dict
    that receives h_s and the node-init pre-activation z0 (their .grad kept)."""
    from models import ops
    from oracle import gcn_ref, graph_ref
    from oracle.detector_ref import LeakDetectorRef
    from oracle.dropout_ref import edge_stream_mask, keep_mask, row_stream_mask
    sensors, pipes = lta_ids()
    m = LeakDetectorRef(LTA_INP, sensors, pipes).train()
    m.load_state_dict(sd)
    m = m.to(dt).to(dev)
    seed_t, seed_h = seeds
    B = r.shape[0]
    N, D, P = len(m.node_names), 64, len(pipes)
    R = B * N
    sc = 1.0 / 0.9
    pre = {}

    def relu(site, z):
        pre[site] = z.detach()
        if masks is None or site not in masks:
            return torch.relu(z)
        return z * masks[site].to(dt).to(dev).reshape(z.shape)

    def t(a):
        return torch.from_numpy(a.astype(np.float64)).to(dt).to(dev)
    mk0 = t(row_stream_mask(seed_t, 0, np.arange(R), D, 0.1))
    mkl = [t(row_stream_mask(seed_t, l, np.arange(R), D, 0.1)) for l in (1, 2)]
    me = t(edge_stream_mask(seed_h, ops.EDGE_HEAD_SALT, np.arange(B * P), 0.1))
    mn = t(keep_mask(seed_h, ops.NOLEAK_HEAD_SALT, np.arange(B * 128, dtype=np.uint64).reshape(B, 128), 0.1))
    h_s = m.sensor_encoder(r.to(dt).to(dev), tf.to(dt).to(dev))
    h0 = torch.zeros(B, N, 64, dtype=dt, device=dev)
    si = m.sensor_node_idx.to(dev)
    h0[:, si] = h_s
    mask = torch.zeros(N, 1, dtype=dt, device=dev)
    mask[si] = 1
    z0 = m.sensor_to_node(torch.cat([h0, mask.expand(B, -1, -1)], -1))
    if aux is not None:
        h_s.retain_grad()
        z0.retain_grad()
        aux.update(h_s=h_s, z0=z0)
    x = relu("init", z0).reshape(R, D) * mk0 * sc
    ei = torch.from_numpy(graph_ref.batchify(m.edge_index_single.numpy(), N, B))
    for l, conv in enumerate(m.convs):
        x = relu(f"conv{l}", conv(x, ei)) * mkl[l] * sc
    hn = x.view(B, N, D)
    u, v = m.pipe_ends[:, 0].to(dev), m.pipe_ends[:, 1].to(dev)
    d = hn[:, u] - hn[:, v]
    pre["absdiff"] = d.detach()
    ad = d.abs() if masks is None or "absdiff" not in masks else d * masks["absdiff"].to(dt).to(dev)
    feat = torch.cat([hn[:, u], hn[:, v], ad], -1).reshape(B * P, 3 * D)
    mlp = m.edge_head.mlp
    hid = relu("edge", mlp[0](feat).view(B, P, -1)).reshape(B * P, -1) * me * sc
    pl = mlp[3](hid).view(B, P)
    pooled = gcn_ref.global_mean_pool(x, torch.arange(B).repeat_interleave(N), size=B)  # follows x's device
    nmlp = m.noleak_head.mlp
    nl = nmlp[3](relu("noleak", nmlp[0](pooled)) * mn * sc)
    out = torch.cat([pl, nl], -1)
    out.backward(up.to(dt).to(dev))
    keep = {"init": mk0, "conv0": mkl[0], "conv1": mkl[1], "edge": me, "noleak": mn}
    return out.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()}, pre, keep


def test_detector_b256_train_vs_oracle_masks():
    """Train mode at B = 256: the HIP path's dropout masks (drawn on the device from two
    seeds off torch's CPU generator) regenerated on the host and fed to a CPU replay of the
    oracle; logits within 1e-5, grads vs the fp64 replay (same bars)."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    sd = _random_ref(51)
    B = 256
    gen = torch.Generator().manual_seed(52)
    r = torch.randn(B, 36, 29, generator=gen)
    tf = torch.randn(B, 36, 9, generator=gen)
    up = torch.randn(B, len(pipes) + 1, generator=gen) / B
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train()
    m.load_state_dict(sd)
    torch.manual_seed(53)
    m.capture = {}
    lg = m(r.to(DEV), tf.to(DEV))
    lg.backward(up.to(DEV))
    masks = hip_relu_masks(m.capture, B, len(m.node_names), len(pipes), m.pipe_ends)
    torch.manual_seed(53)
    seeds = tuple(int(torch.randint(0, 2 ** 62, (1,), dtype=torch.long).item()) for _ in range(2))
    m.capture = None
    o64, _, pre64, keep = _replay_train_cpu(sd, r, tf, seeds, torch.float64, up)
    assert_close(lg, o64, what="B=256 train-mode logits")
    check_relu_ties(pre64, masks, keep)
    # truth and fp32 yardsticks on the HIP path's side of every kink (see the eval test)
    _, g64, _, _ = _replay_train_cpu(sd, r, tf, seeds, torch.float64, up, masks=masks)
    o32, g32, _, _ = _replay_train_cpu(sd, r, tf, seeds, torch.float32, up, masks=masks)
    assert_close(o32, o64, rtol=1e-5, what="replay fp32 vs fp64 (self-check)")
    _, g32d, _, _ = _replay_train_cpu(sd, r, tf, seeds, torch.float32, up, dev=DEV, masks=masks)
    assert_grads_match_truth({n: p.grad for n, p in m.named_parameters()}, g32, g64, ref32=g32d, rtol_tensor=5e-5)


# ----------------------------------------------------------------------------- configs[1]
def test_predictor_b64_gpu_vs_cpu():
    """configs[1]: NormalPredictorTCN (stock torch on the GPU) forward + MSE
    backward at B = 64 against the same module on the CPU in fp64."""
    from models.predictor import NormalPredictorTCN
    torch.manual_seed(61)
    m = NormalPredictorTCN(29, 9)
    gen = torch.Generator().manual_seed(62)
    x = torch.randn(64, 36, 29, generator=gen)
    xt = torch.randn(64, 36, 9, generator=gen)
    y = torch.randn(64, 29, generator=gen)
    m64 = NormalPredictorTCN(29, 9).double()
    m64.load_state_dict(m.state_dict())
    m64.train()
    mg = m.to(DEV).train()
    for mod in (m64, mg):
        for d in [x for x in mod.modules() if isinstance(x, torch.nn.Dropout)]:
            d.p = 0.0
    l64 = torch.nn.functional.mse_loss(m64(x.double(), xt.double()), y.double())
    l64.backward()
    lg = torch.nn.functional.mse_loss(mg(x.to(DEV), xt.to(DEV)), y.to(DEV))
    lg.backward()
    assert abs(lg.item() - l64.item()) <= 1e-5 * abs(l64.item())
    num = sum(((a.grad.double().cpu() - b.grad) ** 2).sum().item() for a, b in zip(mg.parameters(), m64.parameters()))
    den = sum((b.grad ** 2).sum().item() for b in m64.parameters())
    assert num ** 0.5 <= 1e-4 * den ** 0.5


# ----------------------------------------------------------------------------- drop-in robustness
def test_autocast_and_half_inputs():
    """Under torch.autocast(bfloat16) the ops run their fp32 kernels on fp32-cast inputs:
    logits equal the fp32 run.  A model converted with .half() runs (weights cast to fp32
    on entry) and matches an fp32 model holding the same fp16-rounded weights."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    sd = _random_ref(71)
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    m.load_state_dict(sd)
    gen = torch.Generator().manual_seed(72)
    r = torch.randn(8, 36, 29, generator=gen).to(DEV)
    tf = torch.randn(8, 36, 9, generator=gen).to(DEV)
    ref = m(r, tf)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg = m(r, tf)
    assert lg.dtype == torch.float32
    assert_close(lg, ref, what="autocast logits")
    mh = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    mh.load_state_dict(sd)
    mh = mh.half()
    m32 = LeakDetector(LTA_INP, sensors, pipes).to(DEV).eval()
    m32.load_state_dict({k: v.half().float() for k, v in sd.items()})
    lh = mh(r.half(), tf.half())
    l32 = m32(r.half().float(), tf.half().float())
    assert_close(lh.float(), l32, what="half-model logits")
    lh.float().sum().backward()
    assert all(p.grad is not None and p.grad.dtype == torch.float16 for p in mh.parameters())


def test_dropout_under_plain_cuda_graph_capture():
    """A train-mode forward captured with torch.cuda.graph (no SeedSlots installed) must
    not freeze its dropout seeds: two replays draw different masks."""
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(DEV).train()
    r = torch.randn(4, 36, 29, device=DEV)
    tf = torch.randn(4, 36, 9, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            m(r, tf)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        out = m(r, tf)
    g.replay()
    a = out.clone()
    g.replay()
    b = out.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(a).all() and not torch.equal(a, b)


def test_gcnconv_cache_on_recycled_edge_index():
    """GCNConv caches the CSR of the last edge_index it saw.  A different graph of the same
    shape handed over at a recycled address (the caching allocator's common case) must be
    rebuilt, not served from the stale CSR."""
    from models.gcn import GCNConv
    from oracle.gcn_ref import GCNConvRef
    N, D = 500, 64
    torch.manual_seed(81)
    ref = GCNConvRef(D, D)
    conv = GCNConv(D, D).to(DEV)
    conv.load_state_dict(ref.state_dict())
    x = torch.randn(N, D)
    gen = torch.Generator().manual_seed(82)
    e1 = torch.randint(0, N, (2, 3000), generator=gen)
    e2 = torch.randint(0, N, (2, 3000), generator=gen)
    a = e1.to(DEV)
    conv(x.to(DEV), a)
    addr = a.data_ptr()
    del a
    b = e2.to(DEV)
    same_addr = b.data_ptr() == addr
    y = conv(x.to(DEV), b)
    assert_close(y, ref(x, e2).detach(), what="second graph")
    b[0, :10] = (b[0, :10] + 1) % N  # in-place edit of the same tensor
    assert_close(conv(x.to(DEV), b), ref(x, b.cpu()).detach(), what="edited graph")
    assert same_addr or True  # address reuse is likely, not guaranteed; the check above holds either way
