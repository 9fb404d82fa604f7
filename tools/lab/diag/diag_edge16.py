"""EdgeHead forward f16x2 transform vs the 3-way split and a float64 reference (r04e failure)."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(REPO / "leak-det-gnn_amd"))
import numpy as np
import torch
from models import _native as nat
from models import ops

import ctypes
DEV = torch.device("cuda:0")
LIBS = {"new": REPO / "leak-det-gnn_amd/lib/libleakgnn.so", "old": REPO / "leak-det-gnn_amd/lib/old/libleakgnn.so"}
_p, _i64, _i32, _f32, _u64, _u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_uint32
def _load(path):
    l = ctypes.CDLL(str(path))
    l.lg_edge_head_fwd.restype = _i32
    l.lg_edge_head_fwd.argtypes = [_p] * 7 + [_i64, _p, _i64, _i64, _i64, _i64, _i64, _i32, _f32, _u64, _u32, _p]
    return l
g = np.load(REPO / "tests/golden/graph_ltown_a.npz")
ends = torch.from_numpy(g["pipe_ends"]).long()
B, N, P, D = 4, 661, 764, 64
gen = torch.Generator().manual_seed(13)
h = torch.randn(B, N, D, generator=gen)
W1 = torch.randn(128, 3 * D, generator=gen) / 8
b1 = torch.randn(128, generator=gen) / 4
W2 = torch.randn(128, generator=gen) / 8
b2 = torch.randn(1, generator=gen)
u, v = ends[:, 0], ends[:, 1]
hd = h.double()
feat = torch.cat([hd[:, u], hd[:, v], (hd[:, u] - hd[:, v]).abs()], -1).reshape(B * P, 3 * D)
ref = torch.relu(feat @ W1.double().t() + b1.double())
pre = feat @ W1.double().t() + b1.double()
e = ends.to(DEV)
res = {}
for name, fl, lp in [("f16", 0, "new"), ("x3", nat.LG_F_BF16X3, "new"), ("bf", nat.LG_F_BF16, "new"),
                     ("old_x3", 0, "old"), ("old_nm_x3", nat.LG_F_NODE_MAJOR, "old"), ("nm_f16", nat.LG_F_NODE_MAJOR, "new")]:
    lib = _load(LIBS[lp])
    hs = (h.transpose(0, 1).contiguous() if fl & nat.LG_F_NODE_MAJOR else h).to(DEV)
    logits = torch.empty(B, P, device=DEV)
    hid = torch.full((B * P, 128), float("nan"), device=DEV)
    w1d, b1d, w2d, b2d = W1.to(DEV), b1.to(DEV), W2.to(DEV), b2.to(DEV)
    rc = lib.lg_edge_head_fwd(e.data_ptr(), hs.data_ptr(), w1d.data_ptr(), b1d.data_ptr(), w2d.data_ptr(),
                              b2d.data_ptr(), logits.data_ptr(), P, hid.data_ptr(), B, N, P, D, 128, fl, 0.0, 0, 0,
                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0, (name, rc)
    torch.cuda.synchronize()
    res[name] = hid.cpu().double()
    err = (res[name] - ref).abs()
    print(name, "nan", int(torch.isnan(res[name]).sum()), "max err", float(err.max()), "scale", float(ref.abs().max()))
a = res["f16"]
m = (ref > 1e-3) & (a > 1e-3)
r = (a[m] / ref[m])
print("ratio f16/ref: min", float(r.min()), "max", float(r.max()), "median", float(r.median()))
bad = (a - ref).abs() > 1e-4
print("bad elems", int(bad.sum()), "of", bad.numel(), "bad rows", int(bad.any(1).sum()), "bad cols", int(bad.any(0).sum()))
print("bad per col (hidden unit) first 128:", bad.sum(0).tolist())
rows = torch.nonzero(bad.any(1)).flatten()[:10].tolist()
print("bad rows", rows, "rows mod 32", [x % 32 for x in rows])
r0 = rows[0] if rows else 0
cols = torch.nonzero(bad[r0]).flatten()[:10].tolist()
print("row", r0, "cols", cols, "f16", [round(float(a[r0, c]), 4) for c in cols], "ref", [round(float(ref[r0, c]), 4) for c in cols],
      "pre", [round(float(pre[r0, c]), 4) for c in cols])
