"""Host side of the product (CPU): graph builder parity with the reference,
module / state-dict boundary, residual builder and predictors, and the C ABI
(library loads and exports every symbol include/leakgnn.h declares)."""
from __future__ import annotations

import ctypes
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import PKG, REPO
from helpers import LTA_INP, assert_close, load, lta_ids


def test_product_graph_builder_bit_exact():
    from models.utils import build_wdn_graph_from_inp
    g = load("graph_ltown_a.npz")
    sensors, pipes = lta_ids()
    wg = build_wdn_graph_from_inp(LTA_INP, sensors, pipes, add_self_loops=False, make_undirected=True)
    assert wg.node_names == [str(n) for n in g["node_names"]]
    assert wg.edge_index.dtype == torch.long
    np.testing.assert_array_equal(wg.edge_index.numpy(), g["edge_index"])
    np.testing.assert_array_equal(wg.pipe_ends, g["pipe_ends"])
    wg2 = build_wdn_graph_from_inp(LTA_INP, sensors, pipes, add_self_loops=True, make_undirected=False)
    np.testing.assert_array_equal(wg2.edge_index.numpy(), g["edge_index_loops_directed"])
    with pytest.raises(ValueError):
        build_wdn_graph_from_inp(LTA_INP, sensors, ["no_such_pipe"])


def test_parse_epanet_edge_cases(tmp_path):
    from models.utils import parse_epanet_inp
    from oracle.graph_ref import parse_inp
    p = tmp_path / "t.inp"
    p.write_text("junk before\n[junctions]\n a 1 ; c\n;only comment\n\n [PIPES] \np1 a b 3\n[PIPES] ;x\n[]\n")
    assert parse_epanet_inp(p) == parse_inp(p)
    assert parse_epanet_inp(p)["JUNCTIONS"] == ["a 1"]


def test_detector_boundary_state_dict():
    from models.detector import LeakDetector
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1)
    fx = load("detector_b2.npz")
    ref = {k[len("param."):]: v for k, v in fx.items() if k.startswith("param.")}
    sd = m.state_dict()
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        assert tuple(sd[k].shape) == v.shape, k
    m.load_state_dict({k: torch.from_numpy(v) for k, v in ref.items()}, strict=True)
    # public attributes used by the callers
    g = load("graph_ltown_a.npz")
    assert m.sensor_node_ids == sensors
    np.testing.assert_array_equal(m.sensor_node_idx.numpy(), g["sensor_node_idx"])
    np.testing.assert_array_equal(m.pipe_ends.numpy(), g["pipe_ends"])
    np.testing.assert_array_equal(m.edge_index_single.numpy(), g["edge_index"])
    assert m.pipe_ids == pipes and m.pipe_to_idx[pipes[5]] == 5
    assert len(m.node_names) == 661 and m.node_to_idx[m.node_names[7]] == 7
    with pytest.raises(RuntimeError):  # no CPU path
        m(torch.zeros(1, 36, 29), torch.zeros(1, 36, 9))


def test_predictors_and_residual_builder_match_reference():
    from models.predictor import NormalPredictorGRU, NormalPredictorTCN
    from models.utils import build_residual_sequence_from_segment
    fx = load("predictor.npz")
    tcn = NormalPredictorTCN(29, 9).eval()
    tcn.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("tcn.")}, strict=True)
    gru = NormalPredictorGRU(29, 9).eval()
    gru.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("gru.")}, strict=True)
    x, xt = torch.from_numpy(fx["x"]), torch.from_numpy(fx["x_time"])
    with torch.no_grad():
        assert_close(tcn(x, xt), fx["y_tcn"], what="tcn")
        assert_close(gru(x, xt), fx["y_gru"], what="gru")
        res = build_residual_sequence_from_segment(tcn, torch.from_numpy(fx["seg"]), torch.from_numpy(fx["tseg"]),
                                                   36, 36)
        assert_close(res, fx["residual"], what="residual")
        one = build_residual_sequence_from_segment(tcn, torch.from_numpy(fx["seg"][0]),
                                                   torch.from_numpy(fx["tseg"][0]), 36, 36)
        assert_close(one, fx["residual"][0], what="residual 2-D input")


def _header_symbols():
    text = (REPO / "include" / "leakgnn.h").read_text()
    return sorted(set(re.findall(r"\b(lg_[a-z0-9_]+)\s*\(", text)))


def test_c_abi_exports_every_declared_symbol():
    from models import _native
    lib = _native.load_library()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in leakgnn.h but not exported"
        assert s in _native.SIGNATURES, f"{s} has no ctypes signature"
    assert set(_native.SIGNATURES) == set(syms)
    raw = ctypes.CDLL(str(_native.LIB_PATH))
    for s in syms:
        getattr(raw, s)


def test_c_abi_host_only_calls():
    """Entry points that do not touch the GPU: version, error strings, workspace
    sizes and argument validation (returns LG_EINVAL before any HIP call)."""
    from models import _native
    lib = _native.load_library()
    assert lib.lg_abi_version() == _native.ABI_VERSION == 26
    assert lib.lg_timing_arm(-1) == -1 and lib.lg_timing_disarm() == 0 and lib.lg_timing_elapsed(0, None) == -1
    assert lib.lg_nm_table_build(None, None, 661, None, None, None) == -1
    assert lib.lg_strerror(0) == b"ok" and lib.lg_strerror(-1) == b"invalid argument"
    assert lib.lg_graph_workspace_bytes(1532, 661) >= 4 * (5 * 661 + 2 * (1532 + 661))
    assert lib.lg_graph_workspace_bytes(-1, 5) == -1
    assert lib.lg_incidence_workspace_bytes(764, 661) >= 8 * 661
    assert lib.lg_gcn_bwd_workspace_bytes(48) == -2
    assert lib.lg_gcn_fwd(None, None, None, None, None, None, None, 1, 661, 64, 2193, 0, 0.0, 0, 0, None) == -1
    assert lib.lg_gcn_bwd(None, None, None, None, None, None, None, None, None, None, None, None, 1, 661, 64, 2193, 0,
                          1.0, 1.0,
                          None, 0, None) == -1
    assert lib.lg_gcn_bwd_nm_workspace_bytes(48) == -2
    assert lib.lg_gcn_fwd_nm(None, None, None, None, None, None, 16, 661, 64, 2193, 0, 0.0, 0, 0, None) == -1
    assert lib.lg_gcn_bwd_nm(None, None, None, None, None, None, None, None, None, None, None, 16, 661, 64, 0, 1.0,
                             1.0, None, 0, None) == -1
    assert lib.lg_graph_build(None, 5, 0, 1, 1, 1.0, None, None, None, None, None, None, None, 0, None) == -1
    assert lib.lg_pipe_gather_fwd(None, None, None, 1, 10, 5, 64, None) == -1
    assert lib.lg_mean_pool_fwd(None, None, 2, 10, 64, None) == -1
    assert lib.lg_pool_head_bwd_workspace_bytes(256, 64, 64) == -2   # hidden must be 128
    assert lib.lg_linear_dw_workspace_bytes(7424, 64, 48) == -2
    assert lib.lg_linear_dw(None, None, 7424, 64, 64, None, None, None, 0, None) == -1
    assert lib.lg_pool_head_fwd(None, None, None, None, None, None, None, None, 765, 764, 2, 661, 64, 128, 0, 0.0, 0,
                                102, None) == -1
    assert lib.lg_edge_head_fwd(None, None, None, None, None, None, None, 764, None, 2, 661, 764, 64, 128, 0, 0.0, 0,
                                101, None) == -1
    assert lib.lg_edge_head_bwd(None, None, None, None, None, None, 764, None, None, None, None, None, 2, 661, 764, 64,
                                128, 0, 0.0, None, 0, None) == -1
    # GRU: H in {32, 64} tiled, other H in 1..1024 generic (ABI 26: 512 slab rows at most);
    # the backward needs the saved gates; gates need h_seq
    assert lib.lg_gru_bwd_workspace_bytes(256, 29, 10, 48) == 512 * (3 * 48 * (48 + 10) + 6 * 48) * 4
    assert lib.lg_gru_bwd_workspace_bytes(256, 29, 10, 1025) == -1
    assert lib.lg_gru_bwd_workspace_bytes(256, 29, 10, 32) > 0
    assert lib.lg_gru_fwd(None, None, None, None, None, None, None, None, None, 2, 36, 29, 10, 48, None) == -1
    assert lib.lg_gru_fwd(None, None, None, None, None, None, None, None, None, 2, 36, 29, 10, 1025, None) == -2
    assert lib.lg_gru_bwd(None, None, None, None, None, None, None, None, None, None, None, None, 2, 36, 29, 10, 64,
                          None, 0, None) == -1


def test_undersized_workspace_returns_einval():
    """Every workspace-taking entry point checks the caller's ws_bytes against the slab its own
    launch grid writes and returns LG_EINVAL (-1) before launching anything when it is short
    (ABI 21; round 3's trainer hang was a silent overrun of a grid-sized slab).  No GPU is
    needed: the checks run on the host before any HIP call, with stand-in device pointers."""
    from models import _native
    lib = _native.load_library()
    F = 16  # a non-NULL stand-in device pointer (never dereferenced on these paths)
    B, N, D, P, S = 256, 661, 64, 764, 29
    need = lib.lg_gcn_bwd_nm_workspace_bytes(D)
    assert need > 0
    args = (F, F, F, F, F, F, F, F, F, None, None, B, N, D, 0x10, 1.0, 1.0, F)
    assert lib.lg_gcn_bwd_nm_bits(*args, need - 1, None, None) == -1
    assert lib.lg_gcn_bwd_nm(*args, 0, None) == -1
    assert lib.lg_gcn_bwd_rows(F, F, F, F, F, F, F, F, 100_000, 64, F, need - 1, None) == -1
    assert lib.lg_gcn_bwd(F, F, F, F, None, F, F, F, F, F, None, None, B, N, D, 2193, 0, 1.0, 1.0, F,
                          lib.lg_gcn_bwd_workspace_bytes(D) - 1, None) == -1
    wse = lib.lg_edge_head_bwd_workspace_bytes(B, P, D, 128)
    assert wse > 0
    eargs = (F, F, F, F, F, F, P, F, F, F, F, F)
    assert lib.lg_edge_head_bwd(*eargs, B, N, P, D, 128, 0, 0.0, F, wse - 1, None) == -1
    assert lib.lg_edge_head_bwd_scatter(*eargs, F, F, None, None, None, F, B, N, P, D, 128, 0x20, 0.0, F, wse - 1,
                                        None) == -1
    hdr = (ctypes.c_int32 * 16)(1, P, N, D)  # a schedule header (the streamed path checks the workspace too)
    for D2 in (64, 32):
        hdr[3] = D2
        assert lib.lg_edge_head_bwd_scatter(*eargs, F, F, F, hdr, None, F, B, N, P, D2, 128, 0x20, 0.0, F,
                                            lib.lg_edge_head_bwd_workspace_bytes(B, P, D2, 128) - 1, None) == -1
    wsp = lib.lg_pool_head_bwd_workspace_bytes(B, D, 128)
    assert lib.lg_pool_head_bwd(F, F, F, F, F, P + 1, P, F, F, F, F, F, B, D, 128, 0, 0.0, F, wsp - 1, None) == -1
    hargs = (F, F, F, F, F, F, P + 1, F, F, F, F, F, F, F, None, None, F, F, B, N, P, D, 128, 0x20, 0.0, F, wse, None)
    assert lib.lg_heads_bwd_scatter(F, F, F, F, F, F, F, F, 0, 0.0, F, wsp - 1, *hargs) == -1
    wsg = lib.lg_gru_bwd_workspace_bytes(B, S, 10, 64)
    assert lib.lg_gru_bwd(F, F, F, F, F, F, F, None, F, F, F, F, B, 36, S, 10, 64, F, wsg // 2 - 1, None) == -1
    wss = lib.lg_sensor_proj_bwd_workspace_bytes(B, S, D, D)
    assert lib.lg_sensor_proj_bwd(F, F, F, F, F, None, F, F, F, B, N, S, D, D, 0x20, F, wss - 1, None) == -1
    wsl = lib.lg_linear_dw_workspace_bytes(B * S, D, D)
    assert lib.lg_linear_dw(F, F, B * S, D, D, F, F, F, wsl - 1, None) == -1
    assert lib.lg_graph_build(F, 1532, N, 1, 1, 1.0, F, F, F, F, F, F, F,
                              lib.lg_graph_workspace_bytes(1532, N) - 1, None) == -1
    assert lib.lg_incidence_build(F, P, N, F, F, F, lib.lg_incidence_workspace_bytes(P, N) - 1, None) == -1
    sizes = (ctypes.c_int64 * 1)(1000)
    table = (ctypes.c_int64 * 4)(F, F, F, F)
    wsa = lib.lg_clip_adamw_workspace_bytes(ctypes.addressof(sizes), 1)
    assert wsa == 8  # one launch since ABI 23: no partials (the workspace stays a sized argument)
    assert lib.lg_clip_adamw(ctypes.addressof(table), ctypes.addressof(sizes), 1, F, 1e-3, 0.9, 0.999, 1e-8, 0.0,
                             1.0, None, F, wsa - 1, None) == -1
    wsn = lib.lg_gru_node_init_bwd_workspace_bytes(B, S, 10, 64)
    assert wsn > 0
    assert lib.lg_gru_node_init_bwd(F, F, F, F, F, F, F, F, None, F, None, F, F, F, F, F, F, B, 36, S, 10, 64, N, F,
                                    wsn - 1, None) == -1


def test_library_built_for_gfx950_only():
    """The offload bundle inside libleakgnn.so carries gfx950 code objects and nothing else."""
    blob = (PKG / "lib" / "libleakgnn.so").read_bytes()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_graft_entry_build():
    """The driver's build check: make (no-op when up to date) + import + ABI match."""
    import __graft_entry__ as ge
    ge.build()


def test_seed_pointer_salt_bit_matches_header():
    """The device-seed salt bit of the Python side is the header's LG_SALT_SEED_PTR."""
    import re
    from models import _native
    from pathlib import Path
    hdr = (Path(__file__).resolve().parents[1] / "include" / "leakgnn.h").read_text()
    m = re.search(r"#define LG_SALT_SEED_PTR (0x[0-9a-fA-F]+)u", hdr)
    assert m and int(m.group(1), 16) == _native.LG_SALT_SEED_PTR == 1 << 31


def test_rcm_schedule_order():
    """lg_rcm_order (host): a permutation, deterministic, bandwidth-reducing on L-TOWN-A
    (largest |u - v| over the pipes 656 -> <= 32), self loops / duplicates / isolated nodes
    and a second component handled, out-of-range ids refused."""
    from models import _native, ops
    with np.load(REPO / "tests" / "golden" / "graph_ltown_a.npz") as g:
        ei = g["edge_index"]
    o = ops.schedule_order(torch.from_numpy(ei), 661).numpy()
    assert sorted(o.tolist()) == list(range(661))
    assert np.array_equal(o, ops.schedule_order(torch.from_numpy(ei), 661).numpy())
    inv = np.empty(661, np.int64)
    inv[o] = np.arange(661)
    assert np.abs(ei[0] - ei[1]).max() > 600
    assert np.abs(inv[ei[0]] - inv[ei[1]]).max() <= 32
    # path 0-2-4 plus self loop and duplicate, a separate edge 1-3, isolated node 5
    small = torch.tensor([[0, 2, 2, 4, 1, 0], [2, 4, 0, 4, 3, 2]])
    o = ops.schedule_order(small, 6).numpy()
    assert sorted(o.tolist()) == list(range(6))
    pos = {int(n): i for i, n in enumerate(o)}
    assert abs(pos[0] - pos[2]) == 1 and abs(pos[2] - pos[4]) == 1 and abs(pos[1] - pos[3]) == 1
    lib = _native.load_library()
    bad = torch.tensor([[0], [7]], dtype=torch.long)
    out = torch.empty(6, dtype=torch.int32)
    assert lib.lg_rcm_order(bad.data_ptr(), 1, 6, out.data_ptr()) == -1


def test_gcn_conv_row_tiles_only_within_one_launch():
    """GCNConv at D = 64 takes the row-tile kernels only while N * D * 4 fits one launch's 32-bit
    buffer offsets; past it (and at D = 32) it falls back to lg_gcn_fwd / lg_gcn_bwd."""
    from models import library, ops
    limit = ops.NM_MAX_BYTES // (64 * 4)
    assert library._use_rows(100_000, 64)
    assert library._use_rows(limit, 64)
    assert not library._use_rows(limit + 1, 64)
    assert not library._use_rows(100_000, 32)


def _schedule(lib, ends, N, D):
    P = ends.shape[0]
    words = int(lib.lg_pipe_schedule_words(P, N, D))
    sc = np.zeros(words, np.int32)
    rp = np.zeros(N + 1, np.int32)
    it = np.zeros(max(2 * P, 1), np.int32)
    e = np.ascontiguousarray(ends, dtype=np.int64)
    rc = lib.lg_pipe_schedule_build(e.ctypes.data, P, N, D, sc.ctypes.data, words, rp.ctypes.data, it.ctypes.data)
    return rc, sc, rp, it


def _stream_sums(sc, ends, g0, dp):
    """The streamed EdgeHead scatter (edge.hip edge_stream_scatter) replayed on the host in
    float32: events of a tile run in parallel, so they must touch distinct nodes and slots."""
    ver, P, N, D, TR, tpw, nslots, maxev, bw, nzero, offp, offb, offz, total = (int(v) for v in sc[:14])
    perm = sc[offp:offp + 4 * P].reshape(P, 4)[:, 2]
    lacc = np.full((max(nslots, 1), dp.shape[-1]), np.nan, np.float32)
    out = np.full((N, dp.shape[-1]), np.nan, np.float32)
    seen = np.zeros(N, np.int64)
    for t in range(tpw):
        blk = sc[offb + t * bw: offb + (t + 1) * bw]
        ne = int(blk[0])
        ev = blk[2:2 + 2 * ne].reshape(ne, 2).view(np.uint32)
        incl = blk[2 + 2 * maxev:].view(np.uint8)
        nodes, slots = [], []
        for w0, w1 in ev:
            node, first, last = int(w0 & 0xFFFFFF), bool((w0 >> 24) & 1), bool((w0 >> 25) & 1)
            slot, st, cnt = int(w1 & 0xFFFF), int((w1 >> 16) & 0xFF), int(w1 >> 24)
            nodes.append(node)
            if not (first and last):  # reads and/or writes its slot
                slots.append(slot)
            acc = g0.copy() if first else lacc[slot].copy()
            assert not np.isnan(acc).any(), "an open node's running sum was read before it was written"
            for i in range(cnt):
                b = int(incl[st + i])
                row = t * TR + (b >> 1)
                assert row < P
                acc = acc + dp[perm[row], b & 1]
                seen[node] += 1
            if last:
                out[node] = acc
            else:
                lacc[slot] = acc
        assert len(set(nodes)) == len(nodes), "a node with two events in one tile"
        assert len(set(slots)) == len(slots), f"tile {t}: two events share an open-node slot"
    for n in sc[offz:offz + nzero]:
        out[n] = g0
    return out, seen, perm


@pytest.mark.parametrize("D", [64, 32])
@pytest.mark.parametrize("graph", ["ltown", "odd"])
def test_pipe_schedule_streams_the_csr_order_sums(D, graph):
    """lg_pipe_schedule_build (ABI 22, host): the pipe order is a permutation, every incidence
    is in exactly one event, the open-node slots never collide, and the streamed sums equal the
    sums over its schedule-ordered incidence CSR (lg_pipe_scatter_bwd's order) bit for bit.
    'odd': a hub of degree 40 (more incidences than a tile has rows), a self-loop pipe, nodes
    without pipes."""
    from models import _native
    lib = _native.load_library()
    if graph == "ltown":
        ends, N = load("graph_ltown_a.npz")["pipe_ends"].astype(np.int64), 661
    else:
        rng = np.random.default_rng(3)
        N = 60
        ring = [(i, i + 1) for i in range(1, 44)]
        hub = [(0, int(j)) for j in rng.permutation(np.arange(1, 45))[:40]]
        ends = np.array(ring + hub + [(7, 7)], np.int64)
    P = ends.shape[0]
    rc, sc, rp, it = _schedule(lib, ends, N, D)
    assert rc == 0
    assert int(sc[0]) == 1 and tuple(int(v) for v in sc[1:4]) == (P, N, D) and int(sc[4]) == 2048 // D
    rng = np.random.default_rng(D)
    dp = (rng.standard_normal((P, 2, 4)) * np.exp2(rng.integers(-20, 20, (P, 2, 1)))).astype(np.float32)
    g0 = rng.standard_normal(4).astype(np.float32)
    out, seen, perm = _stream_sums(sc, ends, g0, dp)
    assert sorted(perm.tolist()) == list(range(P))
    np.testing.assert_array_equal(sc[16:16 + 4 * P].reshape(P, 4)[:, :2], ends[perm])
    deg = np.bincount(ends.ravel(), minlength=N)
    np.testing.assert_array_equal(seen, deg)
    np.testing.assert_array_equal(rp, np.concatenate([[0], np.cumsum(deg)]))
    spos = np.empty(P, np.int64)
    spos[perm] = np.arange(P)
    ref = np.empty((N, 4), np.float32)
    for n in range(N):
        items = it[rp[n]:rp[n + 1]]
        keys = [(spos[i >> 1], i & 1) for i in items]
        assert keys == sorted(keys), f"node {n}: CSR items not in schedule order"
        acc = g0.copy()
        for i in items:
            acc = acc + dp[i >> 1, i & 1]
        ref[n] = acc
    assert out.tobytes() == ref.tobytes(), "streamed sums differ from the CSR-order sums"
    if graph == "ltown":
        assert int(sc[6]) <= 48, f"{int(sc[6])} open slots"  # RCM keeps L-TOWN-A's frontier small


def test_pipe_schedule_rejects_bad_input():
    from models import _native
    lib = _native.load_library()
    ends = np.array([[0, 1], [1, 5]], np.int64)
    rc, *_ = _schedule(lib, ends, 3, 64)
    assert rc == -1  # an endpoint id out of range
    assert lib.lg_pipe_schedule_words(2, 3, 48) == -2
    rc, sc, rp, it = _schedule(lib, np.zeros((0, 2), np.int64), 3, 64)
    assert rc == 0 and int(sc[5]) == 0 and int(sc[9]) == 3  # no tiles; every node without pipes


def _vm_ins(lines):
    """(addr, mnemonic, operands, target) tuples for tools/check_vmcnt.check_kernel."""
    out = []
    for i, ln in enumerate(lines):
        mn, _, ops = ln.partition(" ")
        out.append((4 * i, mn, ops, None))
    return out


def test_vmcnt_checker_catches_an_early_copy():
    """tools/check_vmcnt.py: a copy of a register whose load is in flight is
    reported, in both modes; after the covering s_waitcnt it is not; vmcnt counts stores too."""
    sys.path.insert(0, str(REPO / "tools"))
    import check_vmcnt as cv
    early = _vm_ins(["buffer_load_dwordx4 v[0:3], v8, s[0:3], 0 offen", "v_mov_b32_e32 v5, v1",
                     "s_waitcnt vmcnt(0)", "v_add_f32_e32 v6, v0, v1", "s_endpgm"])
    for copies_only in (False, True):
        v = cv.check_kernel(early, copies_only=copies_only)
        assert [a for a, _, _ in v] == [4], v
    late = _vm_ins(["buffer_load_dwordx4 v[0:3], v8, s[0:3], 0 offen", "buffer_store_dword v9, v8, s[0:3], 0 offen",
                    "s_waitcnt vmcnt(1)", "v_mov_b32_e32 v5, v1", "s_endpgm"])
    assert cv.check_kernel(late) == []
    short = _vm_ins(["buffer_load_dwordx4 v[0:3], v8, s[0:3], 0 offen", "buffer_store_dword v9, v8, s[0:3], 0 offen",
                     "s_waitcnt vmcnt(2)", "v_mov_b32_e32 v5, v1", "s_endpgm"])
    assert [a for a, _, _ in cv.check_kernel(short)] == [12]


def test_every_kernel_waits_for_its_loads():
    """Every gfx950 kernel of the library passes tools/check_vmcnt.py: no instruction touches a
    VGPR whose vector-memory load is still in flight (k_gcn_fwd_pc, whose producers issue their
    prefetch through inline asm with hand-written vmcnt waits: no copy, select or spill of such
    a register before its wait)."""
    objs = sorted((PKG / "build").glob("*.o"))
    if not objs:
        pytest.skip("no build/*.o (run make)")
    r = subprocess.run([sys.executable, str(REPO / "tools" / "check_vmcnt.py")] + [str(o) for o in objs],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "k_gcn_fwd_pc" in (REPO / "tools" / "check_vmcnt.py").read_text()
