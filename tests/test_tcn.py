"""Frozen-predictor residual builder (SURVEY §8 f rank 1): oracle, shared-window plan,
and the HIP path (lg_tcn_conv_fwd) against both.

Fixtures: tests/golden/predictor.npz (seeded TCN, l_pred = l_det = 36) and
tests/golden/residual.npz (TCN with non-trivial LayerNorm affine, four (l_pred, l_det)
cases), both the output of the reference's build_residual_sequence_from_segment
(oracle/make_golden.py).  Bar: fp32 within RTOL = 1e-5 of the fixture's scale.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from helpers import RTOL, assert_close, load
from oracle import tcn_ref


def _sd(fx):
    return {k[4:]: torch.from_numpy(v) for k, v in fx.items() if k.startswith("tcn.")}


def _module(fx, device="cpu"):
    from models.predictor import NormalPredictorTCN
    m = NormalPredictorTCN(29, 9).eval()
    m.load_state_dict(_sd(fx), strict=True)
    return m.to(device)


def _cases():
    fx = load("residual.npz")
    return fx, [(int(lp), int(ld), i) for i, (lp, ld, _) in enumerate(fx["cases"])]


# ---------------------------------------------------------------- CPU: oracle + plan
def test_oracle_matches_reference_residual_fixtures():
    fx = load("predictor.npz")
    res = tcn_ref.residual_ref(_sd(fx), torch.from_numpy(fx["seg"]), torch.from_numpy(fx["tseg"]), 36, 36)
    assert_close(res, fx["residual"], what="oracle residual (predictor.npz)")
    fx, cases = _cases()
    for lp, ld, i in cases:
        res = tcn_ref.residual_ref(_sd(fx), torch.from_numpy(fx[f"seg{i}"]), torch.from_numpy(fx[f"tseg{i}"]), lp, ld)
        assert_close(res, fx[f"res{i}"], what=f"oracle residual l_pred={lp} l_det={ld}")


def test_shared_window_plan_matches_reference():
    from models.tcn_plan import emulate, make_plan
    fx, cases = _cases()
    m = _module(fx)
    with torch.no_grad():
        for lp, ld, i in cases:
            res = emulate(make_plan(lp, ld), m, torch.from_numpy(fx[f"seg{i}"]), torch.from_numpy(fx[f"tseg{i}"]))
            assert_close(res, fx[f"res{i}"], what=f"plan emulation l_pred={lp} l_det={ld}")


def test_plan_shape_default_config():
    from models.tcn_plan import make_plan
    p = make_plan(36, 36)
    assert p.seg_len == 72 and p.n_win == 36 and len(p.convs) == 8
    assert [c.dilation for c in p.convs] == [1, 1, 2, 2, 4, 4, 8, 8]
    # 72 shared rows per layer + 24 special positions per window over the 8 layers
    assert sum(len(c.special_t) for c in p.convs) == 24
    assert sum(c.rows for c in p.convs) == 8 * 72 + 36 * 24
    for li, c in enumerate(p.convs):
        prev_rows = 72 if li == 0 else p.convs[li - 1].rows
        assert c.taps.shape == (c.rows, 3) and c.taps.dtype == np.int32
        assert c.taps.min() >= -1 and c.taps.max() < prev_rows
        assert (c.taps[:, 0] >= 0).all()  # tap t always exists
        if li % 2 == 1:
            blk_rows = 72 if li == 1 else p.convs[li - 2].rows
            assert (c.res >= 0).all() and c.res.max() < blk_rows
        else:
            assert (c.res == -1).all()
    assert p.out_rows.min() >= 0 and p.out_rows.max() < p.convs[-1].rows


def test_fast_path_eligibility():
    from models.predictor import NormalPredictorGRU, NormalPredictorTCN
    from models.tcn_plan import fast_path_eligible
    assert fast_path_eligible(NormalPredictorTCN(29, 9).eval())
    assert not fast_path_eligible(NormalPredictorTCN(29, 9).train())
    assert not fast_path_eligible(NormalPredictorTCN(29, 9, hidden_channels=64).eval())
    assert not fast_path_eligible(NormalPredictorTCN(29, 9, num_blocks=3).eval())
    assert not fast_path_eligible(NormalPredictorGRU(29, 9).eval())


# ---------------------------------------------------------------- GPU: HIP path
DEV = torch.device("cuda:0")


def _residual_gpu(m, seg, tseg, lp, ld):
    from models import tcn_plan
    from models.utils import build_residual_sequence_from_segment
    calls = []
    orig = tcn_plan.tcn_residual

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    tcn_plan.tcn_residual = spy
    try:
        with torch.no_grad():
            out = build_residual_sequence_from_segment(m, seg.to(DEV), tseg.to(DEV), l_pred=lp, l_det=ld)
        torch.cuda.synchronize()
    finally:
        tcn_plan.tcn_residual = orig
    assert calls, "the GPU residual builder did not take the HIP fast path"
    return out


@pytest.mark.gpu
def test_hip_residual_matches_reference_fixtures():
    fx = load("predictor.npz")
    m = _module(fx, DEV)
    res = _residual_gpu(m, torch.from_numpy(fx["seg"]), torch.from_numpy(fx["tseg"]), 36, 36)
    assert_close(res, fx["residual"], what="HIP residual (predictor.npz)")
    fx, cases = _cases()
    m = _module(fx, DEV)
    for lp, ld, i in cases:
        res = _residual_gpu(m, torch.from_numpy(fx[f"seg{i}"]), torch.from_numpy(fx[f"tseg{i}"]), lp, ld)
        assert_close(res, fx[f"res{i}"], what=f"HIP residual l_pred={lp} l_det={ld}")


@pytest.mark.gpu
def test_hip_residual_vs_oracle_random_predictor():
    """B = 64 (residual for C2's batch) with every parameter randomised, vs the per-window oracle."""
    from models.predictor import NormalPredictorTCN
    torch.manual_seed(21)
    m = NormalPredictorTCN(29, 9).eval()
    g = torch.Generator().manual_seed(22)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.2 * torch.randn(p.shape, generator=g))
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    seg, tseg = torch.randn(64, 72, 29, generator=g), torch.randn(64, 72, 9, generator=g)
    ref = tcn_ref.residual_ref(sd, seg, tseg, 36, 36)
    res = _residual_gpu(m.to(DEV), seg, tseg, 36, 36)
    assert_close(res, ref, what="HIP residual vs oracle (B=64)")


@pytest.mark.gpu
def test_hip_residual_large_batch_vs_plan_emulation():
    """B = 1000 segments (many tiles per persistent workgroup, all XCD groups busy):
    HIP vs the same plan executed by torch on the GPU, and vs the stock per-window
    module path on a slice."""
    from models import utils as mutils
    from models.predictor import NormalPredictorTCN
    from models.tcn_plan import emulate, make_plan
    torch.manual_seed(5)
    m = NormalPredictorTCN(29, 9).eval().to(DEV)
    g = torch.Generator().manual_seed(6)
    seg, tseg = torch.randn(1000, 72, 29, generator=g), torch.randn(1000, 72, 9, generator=g)
    res = _residual_gpu(m, seg, tseg, 36, 36)
    with torch.no_grad():
        emu = emulate(make_plan(36, 36), m, seg.to(DEV), tseg.to(DEV))
    assert_close(res, emu, what="HIP vs plan emulation (B=1000)")
    old = mutils.RESIDUAL_FAST_PATH
    mutils.RESIDUAL_FAST_PATH = False
    try:
        with torch.no_grad():
            stock = mutils.build_residual_sequence_from_segment(m, seg[:50].to(DEV), tseg[:50].to(DEV), 36, 36)
    finally:
        mutils.RESIDUAL_FAST_PATH = old
    assert_close(res[:50], stock, what="HIP vs stock per-window module (B=50)")


def _conv_ref(x, blk, table, weight, bias, lw, lb, eps, nseg, rows_in, rows_blk):
    """torch restatement of one lg_tcn_conv_fwd call (fp64)."""
    C = 128
    x = x.double().view(nseg, rows_in, C)
    xz = torch.cat([x, torch.zeros(nseg, 1, C, dtype=x.dtype, device=x.device)], 1)
    t = table.long()
    taps = torch.where(t[:, :3] < 0, torch.full_like(t[:, :3], rows_in), t[:, :3])
    gath = xz[:, taps]                                                  # (nseg, rows, 3, C)
    Wt = weight.double().flip(-1).permute(0, 2, 1).reshape(C, 3 * C)
    y = gath.reshape(nseg, -1, 3 * C) @ Wt.t() + bias.double()
    y = torch.relu(torch.nn.functional.layer_norm(y, (C,), lw.double(), lb.double(), eps))
    if blk is not None:
        bz = torch.cat([blk.double().view(nseg, rows_blk, C), torch.zeros(nseg, 1, C, dtype=y.dtype, device=y.device)], 1)
        r = torch.where(t[:, 3] < 0, torch.full_like(t[:, 3], rows_blk), t[:, 3])
        y = y + bz[:, r]
    return y.reshape(-1, C)


@pytest.mark.gpu
def test_tcn_conv_abi_random_tables():
    """lg_tcn_conv_fwd on arbitrary plan tables (zero taps, missing residuals, row counts
    that are not multiples of the 16-row tile, odd segment counts) vs fp64 torch."""
    from models import _native as nat
    lib = nat.load_library()
    C = 128
    g = torch.Generator().manual_seed(9)
    n_packed = lib.lg_tcn_packed_weight_floats(C)
    assert n_packed == C * 3 * C and lib.lg_tcn_packed_weight_floats(64) == 0
    for nseg, rows_in, rows_out, with_blk in ((5, 40, 37, True), (1, 3, 1, False), (33, 72, 144, True),
                                              (7, 200, 250, False)):
        rows_blk = 29 if with_blk else 0
        x = torch.randn(nseg * rows_in, C, generator=g).to(DEV)
        blk = torch.randn(nseg * rows_blk, C, generator=g).to(DEV) if with_blk else None
        table = torch.randint(-1, rows_in, (rows_out, 4), generator=g, dtype=torch.int32)
        table[:, 3] = torch.randint(-1, max(rows_blk, 1), (rows_out,), generator=g, dtype=torch.int32)
        if not with_blk:
            table[:, 3] = -1
        table = table.to(DEV)
        weight = (torch.randn(C, C, 3, generator=g) * 0.05).to(DEV)
        bias, lw, lb = (torch.randn(C, generator=g).to(DEV) for _ in range(3))
        packed = torch.empty(n_packed, device=DEV)
        s = nat.stream_of(x)
        nat.check(lib.lg_tcn_pack_weight(nat.ptr(weight), nat.ptr(packed), C, s), "pack")
        out = torch.full((nseg * rows_out, C), float("nan"), device=DEV)
        nat.check(lib.lg_tcn_conv_fwd(nat.ptr(x), nat.ptr(blk), nat.ptr(table), nat.ptr(packed), nat.ptr(bias),
                                      nat.ptr(lw), nat.ptr(lb), 1e-5, nat.ptr(out), nseg, rows_in, rows_blk,
                                      rows_out, C, s), "lg_tcn_conv_fwd")
        torch.cuda.synchronize()
        ref = _conv_ref(x, blk, table, weight, bias, lw, lb, 1e-5, nseg, rows_in, rows_blk)
        assert_close(out, ref, what=f"tcn conv nseg={nseg} rows_in={rows_in} rows_out={rows_out} blk={with_blk}")
    # argument errors come back as codes, nothing is launched
    assert lib.lg_tcn_conv_fwd(nat.ptr(x), None, nat.ptr(table), nat.ptr(packed), nat.ptr(bias), nat.ptr(lw),
                               nat.ptr(lb), 1e-5, nat.ptr(out), 1, 8, 0, 4, 64, s) == -2
    assert lib.lg_tcn_conv_fwd(nat.ptr(x), None, nat.ptr(table), nat.ptr(packed), nat.ptr(bias), nat.ptr(lw),
                               nat.ptr(lb), 1e-5, nat.ptr(out), 1, 8, 0, 4096, C, s) == -1
    assert lib.lg_tcn_conv_fwd(nat.ptr(x), None, nat.ptr(table), nat.ptr(packed), nat.ptr(bias), nat.ptr(lw),
                               nat.ptr(lb), 1e-5, nat.ptr(out), 0, 8, 0, 4, C, s) == 0
