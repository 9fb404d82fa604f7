"""Pin the CPU oracle against the reference's own outputs (tests/golden) and
against an independent formulation.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import LTA_INP, assert_close, load, lta_ids
from oracle import dense_ref, detector_ref, gcn_ref, graph_ref


@pytest.mark.parametrize("fixture", ["graph_ltown_a.npz"])
def test_graph_ref_matches_reference_builder(fixture):
    g = load(fixture)
    sensors, pipes = [str(s) for s in g["sensor_ids"]], [str(p) for p in g["pipe_ids"]]
    names, ei, ends = graph_ref.build_graph(LTA_INP, sensors, pipes)
    assert names == [str(n) for n in g["node_names"]]
    np.testing.assert_array_equal(ei, g["edge_index"])
    np.testing.assert_array_equal(ends, g["pipe_ends"])
    names2, ei2, _ = graph_ref.build_graph(LTA_INP, sensors, pipes, add_self_loops=True, make_undirected=False)
    np.testing.assert_array_equal(ei2, g["edge_index_loops_directed"])


def test_graph_ref_shape_facts():
    """N=661, E=1532, no duplicates, no self loops, symmetric."""
    g = load("graph_ltown_a.npz")
    ei = g["edge_index"]
    assert len(g["node_names"]) == 661 and ei.shape == (2, 1532) and g["pipe_ends"].shape == (764, 2)
    assert not np.any(ei[0] == ei[1])
    pairs = set(map(tuple, ei.T.tolist()))
    assert len(pairs) == ei.shape[1]
    assert all((d, s) in pairs for s, d in pairs)
    indeg = np.bincount(ei[1], minlength=661)
    assert dict(zip(*np.unique(indeg, return_counts=True))) == {1: 24, 2: 427, 3: 187, 4: 22, 5: 1}


def test_batchify_ref_matches_reference():
    g = load("graph_ltown_a.npz")
    np.testing.assert_array_equal(graph_ref.batchify(g["edge_index"], 661, 3), g["batchified_b3"])


def test_gcn_csr_matches_scatter_norm():
    g = load("graph_ltown_a.npz")
    ei = torch.from_numpy(g["edge_index"])
    row, col, w = gcn_ref.gcn_norm(ei, 661)
    rowptr, c, wc = graph_ref.gcn_csr(g["edge_index"], 661)
    # rebuild the (dst, src) -> w map from the CSR and compare bit-exactly
    m = {}
    for d in range(661):
        for k in range(rowptr[d], rowptr[d + 1]):
            m[(d, int(c[k]))] = wc[k]
    assert len(m) == row.numel()
    for s, d, x in zip(row.tolist(), col.tolist(), w.numpy()):
        assert m[(d, s)] == x
    # self loop is the last entry of every row
    assert all(c[rowptr[d + 1] - 1] == d for d in range(661))


def test_gcn_scatter_vs_dense_and_hand_computed():
    # 4-node path 0-1-2-3 (both directions): deg with loop = [2, 3, 3, 2]
    ei = torch.tensor([[0, 1, 1, 2, 2, 3], [1, 0, 2, 1, 3, 2]])
    x = torch.tensor([[1.0], [2.0], [3.0], [4.0]])
    W = torch.ones(1, 1)
    out = gcn_ref.gcn_conv(x, ei, W, None)
    d = np.array([2.0, 3.0, 3.0, 2.0])
    A = np.array([[1, 1, 0, 0], [1, 1, 1, 0], [0, 1, 1, 1], [0, 0, 1, 1]], dtype=np.float64)
    expect = (A / np.sqrt(np.outer(d, d))) @ np.array([1.0, 2.0, 3.0, 4.0])
    np.testing.assert_allclose(out[:, 0].numpy(), expect, rtol=1e-6)
    # hand values: row 0 = 1/2 + 2/sqrt(6)
    assert abs(out[0, 0].item() - (0.5 + 2 / np.sqrt(6))) < 1e-6
    # scatter vs dense on L-TOWN-A with random features
    g = load("graph_ltown_a.npz")
    eil = torch.from_numpy(g["edge_index"])
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(661, 64, generator=gen)
    W = torch.randn(64, 64, generator=gen) / 8
    b = torch.randn(64, generator=gen)
    s = gcn_ref.gcn_conv(x, eil, W, b)
    dense = (dense_ref.dense_ahat(eil, 661) @ (x @ W.t()).double()).float() + b
    assert_close(s, dense, what="scatter vs dense GCNConv")


def _ref_model(B_fixture: dict | None = None):
    sensors, pipes = lta_ids()
    m = detector_ref.LeakDetectorRef(LTA_INP, sensors, pipes)
    st = load("detector_b2.npz")
    sd = {k[len("param."):]: torch.from_numpy(v) for k, v in st.items() if k.startswith("param.")}
    m.load_state_dict(sd, strict=True)
    return m.eval()


@pytest.mark.parametrize("fixture", ["detector_b2.npz", "detector_b8.npz"])
def test_detector_ref_matches_reference_fixture(fixture):
    fx = load(fixture)
    m = _ref_model()
    residual = torch.from_numpy(fx["residual"]).requires_grad_(True)
    logits = m(residual, torch.from_numpy(fx["tfeat"]))
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(fx["label"]))
    loss.backward()
    assert_close(logits, fx["logits"], what="logits")
    assert abs(loss.item() - float(fx["loss"])) <= 1e-5 * abs(float(fx["loss"]))
    assert_close(residual.grad, fx["grad_residual"], what="grad residual")
    for name, p in m.named_parameters():
        assert_close(p.grad, fx["grad." + name], what="grad " + name)
    if "trace.conv1" in fx:
        for k in ("node_init", "conv0", "conv1"):
            assert_close(m.trace[k].reshape(fx["trace." + k].shape), fx["trace." + k], what=k)


def test_state_dict_keys_match_reference():
    fx = load("detector_b2.npz")
    ref_keys = sorted(k[len("param."):] for k in fx if k.startswith("param."))
    assert ref_keys == sorted(n for n, _ in _ref_model().named_parameters())
    assert sum(fx["param." + k].size for k in ref_keys) == 60418


def test_row_stream_dropout_oracle_matches_scalar_restatement():
    """oracle/dropout_ref.row_stream_mask (vectorised) vs a scalar transcription of
    common.h lg_row_stream_seed / lg_xorshift32 / lg_keep_threshold16; and the keep rate."""
    from oracle.dropout_ref import dropout_key, row_stream_mask

    def mix32(x):
        x &= 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        return x ^ (x >> 16)

    seed, salt, p, D = 0x1234_5678_9ABC_DEF0, 2, 0.1, 64
    key = dropout_key(seed, salt)
    rows = [0, 1, 17, 660, 169215, (1 << 33) + 5]
    got = row_stream_mask(seed, salt, np.array(rows), D, p)
    for ri, row in enumerate(rows):
        for q in range(4):
            a = mix32(((row & 0xFFFFFFFF) * 0x9E3779B9) ^ key)
            s = mix32(a ^ (((row >> 32) * 0x85EBCA6B) & 0xFFFFFFFF) ^ ((q * 0x632BE5AB) & 0xFFFFFFFF)) or 0x6D2B79F5
            thr = int(round(p * 65536))  # 6554 for p = 0.1 (no tie)
            for t in range(D // 16 * 4):
                if t % 2 == 0:
                    s ^= (s << 13) & 0xFFFFFFFF
                    s ^= s >> 17
                    s ^= (s << 5) & 0xFFFFFFFF
                u16 = s & 0xFFFF if t % 2 == 0 else s >> 16
                assert got[ri, 16 * (t // 4) + 4 * q + t % 4] == (u16 >= thr)
    big = row_stream_mask(7, 1, np.arange(20000), D, p)
    assert abs(big.mean() - 0.9) < 0.003
    # neighbouring channels / rows are not trivially correlated
    assert abs(np.corrcoef(big[:, 0], big[:, 1])[0, 1]) < 0.03
    assert abs(np.corrcoef(big[:-1, 5], big[1:, 5])[0, 1]) < 0.03


def test_edge_stream_dropout_oracle_matches_scalar_restatement():
    """oracle/dropout_ref.edge_stream_mask vs a scalar transcription of the EdgeHead
    forward's stream (edge.hip: lg_row_stream_seed(key, row, 4 nh + q), units
    32 nh + 16 i + 4 q + reg); and the keep rate."""
    from oracle.dropout_ref import dropout_key, edge_stream_mask

    def mix32(x):
        x &= 0xFFFFFFFF
        x ^= x >> 16
        x = (x * 0x7FEB352D) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x846CA68B) & 0xFFFFFFFF
        return x ^ (x >> 16)

    seed, salt, p = 0x0F0E_0D0C_0B0A_0908, 101, 0.1
    key = dropout_key(seed, salt)
    rows = [0, 3, 764, 195583, (1 << 32) + 9]
    got = edge_stream_mask(seed, salt, np.array(rows), p)
    thr = int(round(p * 65536))
    for ri, row in enumerate(rows):
        for g in range(16):
            nh, q = g // 4, g % 4
            a = mix32(((row & 0xFFFFFFFF) * 0x9E3779B9) ^ key)
            s = mix32(a ^ (((row >> 32) * 0x85EBCA6B) & 0xFFFFFFFF) ^ ((g * 0x632BE5AB) & 0xFFFFFFFF)) or 0x6D2B79F5
            for t in range(8):
                if t % 2 == 0:
                    s ^= (s << 13) & 0xFFFFFFFF
                    s ^= s >> 17
                    s ^= (s << 5) & 0xFFFFFFFF
                u16 = s & 0xFFFF if t % 2 == 0 else s >> 16
                assert got[ri, 32 * nh + 16 * (t // 4) + 4 * q + t % 4] == (u16 >= thr)
    big = edge_stream_mask(5, 101, np.arange(20000), p)
    assert abs(big.mean() - 0.9) < 0.003
    assert abs(np.corrcoef(big[:, 0], big[:, 1])[0, 1]) < 0.03
    assert abs(np.corrcoef(big[:, 3], big[:, 35])[0, 1]) < 0.03
