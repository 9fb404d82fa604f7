"""x0 path with an identity transform: y = sum_j w_j x0[j] (no bias / relu / dropout), to see
which neighbour term of the compressed layer-0 gather is wrong."""
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
N, S, D, B = 661, sidx.numel(), 64, 256
gen = torch.Generator().manual_seed(5)
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
W = torch.eye(D, device=DEV)
b = torch.zeros(D, device=DEV)
fl = nat.LG_F_BF16X3 | nat.LG_F_DROPOUT  # layer-0 dropout: the same mask in both; x0's scale needs p
mk = m._x0marks(g, slot)
yd = torch.full((N, B, D), float("nan"), device=DEV)
yx = torch.full((N, B, D), float("nan"), device=DEV)
ops.check(lib.lg_gcn_fwd_nm_bits(ops.ptr(g.nodetab), ops.ptr(g.pairs), ops.ptr(x0), ops.ptr(W), ops.ptr(b),
                                 ops.ptr(yd), B, N, D, g.nnz_cap, fl, p, 7, 1, st, None), "dense")
ops.check(lib.lg_gcn_fwd_nm_x0(ops.ptr(mk.nodetab_s), ops.ptr(mk.pairs_s), ops.ptr(xs0), ops.ptr(bits),
                               ops.ptr(nbias), ops.ptr(W), ops.ptr(b), ops.ptr(yx), B, N, S, D, fl, p, 7, 1, st), "x0")
torch.cuda.synchronize()
rp, col, w = g.rowptr.cpu(), g.col.cpu(), g.w.cpu()
sens = set(sidx.tolist())
print("sensor nodes", sorted(sens)[:40])
ne = (yx - yd).abs() > 1e-5 * yd.abs().max()
print("mismatch elems", int(ne.sum()), "nodes", torch.nonzero(ne.any(2).any(1)).flatten().tolist()[:40])
byw = ne.any(2).sum(0)
print("mismatching (node) count per window (first 32):", byw[:32].tolist())
x0c, yxc, ydc = x0.cpu(), yx.cpu(), yd.cpu()
for n in torch.nonzero(ne.any(2).any(1)).flatten().tolist()[:6]:
    nb = [(int(col[e]), float(w[e])) for e in range(int(rp[n]), int(rp[n + 1]))]
    print("node", n, "nbrs", [(c, round(ww, 4), c in sens, int(slot[c])) for c, ww in nb])
    wins = torch.nonzero(ne[n].any(1)).flatten().tolist()
    print("  windows", wins[:20])
    bb = wins[0]
    diff = (yxc[n, bb] - ydc[n, bb]) * (1 - p)  # the layer's dropout scale undone (dropped: 0)
    for c, ww in nb:
        cand = x0c[c, bb] - diff / ww   # the value the kernel must have used for neighbour c
        print("   nbr", c, "implied value (first 8)", [round(v, 4) for v in cand[:8].tolist()],
              "x0 (first 8)", [round(v, 4) for v in x0c[c, bb, :8].tolist()])
    print("  diff (first 16)", [round(v, 4) for v in diff[:16].tolist()])
    v0 = torch.relu(nbias.cpu()) / (1 - p)
    print("  v0 (first 8)", [round(v, 4) for v in v0[:8].tolist()])
