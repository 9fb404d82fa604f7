"""Diagnose lg_gcn_fwd_nm_x0 vs lg_gcn_fwd_nm_bits at B=256 (r04e failure): unwritten tiles
(NaN-filled outputs), run-to-run determinism, mismatch locations."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(REPO / "leak-det-gnn_amd"))
sys.path.insert(0, str(REPO / "tests"))
import torch
from helpers import LTA_INP, lta_ids
from models import _native as nat
from models import ops
from models.detector import LeakDetector

DEV = torch.device("cuda:0")
sensors, pipes = lta_ids()
m = LeakDetector(LTA_INP, sensors, pipes).to(DEV)
g, inc, slot, sidx, live, nons = m._device_state(DEV)
lib = nat.load_library()
N, S, D = 661, sidx.numel(), 64
for B in (256, 37):
    gen = torch.Generator().manual_seed(B + D)
    h_s = torch.randn(B, S, D, generator=gen).to(DEV)
    Wp = (torch.randn(D, D + 1, generator=gen) / 8).to(DEV)
    nbias = torch.randn(D, generator=gen).to(DEV)
    p = 0.1
    st = ops.stream_of(h_s)
    x0 = torch.full((N, B, D), float("nan"), device=DEV)
    ops.check(lib.lg_node_init_proj_fwd(ops.ptr(slot), ops.ptr(sidx), ops.ptr(h_s), ops.ptr(Wp), ops.ptr(nbias),
                                        ops.ptr(x0), B, N, S, D, D, nat.LG_F_DROPOUT | nat.LG_F_NODE_MAJOR, p, 99, 0, st), "ni")
    xs0 = torch.zeros(S, B, D, device=DEV)
    bits = torch.full((N * ((B + 15) // 16) * 64,), -1, device=DEV, dtype=torch.int16)
    ops.check(lib.lg_node_init_bits_fwd(ops.ptr(slot), ops.ptr(sidx), ops.ptr(h_s), ops.ptr(Wp), ops.ptr(nbias),
                                        ops.ptr(xs0), ops.ptr(bits), B, N, S, D, D, nat.LG_F_DROPOUT, p, 99, 0, st), "nib")
    W = (torch.randn(D, D, generator=gen) / 8).to(DEV)
    b = (torch.randn(D, generator=gen) / 4).to(DEV)
    base = nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT
    mk = m._x0marks(g, slot)
    outs = {}
    for name, xf in [("dflt", 0), ("x3", nat.LG_F_BF16X3), ("f32", nat.LG_F_F32_MFMA)]:
        for rep in range(2):
            y = torch.full((N, B, D), float("nan"), device=DEV)
            ops.check(lib.lg_gcn_fwd_nm_bits(ops.ptr(g.nodetab), ops.ptr(g.pairs), ops.ptr(x0), ops.ptr(W), ops.ptr(b),
                                             ops.ptr(y), B, N, D, g.nnz_cap, base | xf, p, 7, 1, st, None), "dense")
            outs[("dense", name, rep)] = y
            if name != "f32":
                y2 = torch.full((N, B, D), float("nan"), device=DEV)
                ops.check(lib.lg_gcn_fwd_nm_x0(ops.ptr(mk.nodetab_s), ops.ptr(mk.pairs_s), ops.ptr(xs0), ops.ptr(bits),
                                               ops.ptr(nbias), ops.ptr(W), ops.ptr(b), ops.ptr(y2), B, N, S, D, base | xf,
                                               p, 7, 1, st), "x0")
                outs[("x0", name, rep)] = y2
    torch.cuda.synchronize()
    ref = outs[("dense", "f32", 0)]
    sens = torch.zeros(N, dtype=torch.bool, device=DEV)
    sens[sidx] = True
    for k, y in outs.items():
        nan = torch.isnan(y)
        d = (y - ref).abs()
        d[nan] = 0
        bad_nodes = torch.nonzero(nan.any(2).any(1)).flatten()
        print(B, k, "nan", int(nan.sum()), "nodes with nan", bad_nodes[:10].tolist(), "max|y-f32|",
              float(d.max()), "scale", float(ref.abs().max()))
    for name in ("dflt", "x3"):
        a, c = outs[("x0", name, 0)], outs[("dense", name, 0)]
        ne = (a != c) & ~(torch.isnan(a) & torch.isnan(c))
        idx = torch.nonzero(ne)
        print(B, name, "x0 != dense:", int(ne.sum()), "first", idx[:8].tolist(),
              "sensor nodes among mismatches", int(sens[idx[:, 0]].sum()) if idx.numel() else 0,
              "max diff", float((a - c).abs().nan_to_num(0).max()))
        print(B, name, "x0 rep eq", torch.equal(outs[("x0", name, 0)].nan_to_num(7), outs[("x0", name, 1)].nan_to_num(7)),
              "dense rep eq", torch.equal(outs[("dense", name, 0)].nan_to_num(7), outs[("dense", name, 1)].nan_to_num(7)))
