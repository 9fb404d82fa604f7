"""Kernel lab (GPU): the f16x2 backward variants of lg_gcn_bwd_nm_bits (k_gcn_bwd_pc:
LG_F_PC | LG_F_F16X2; k_gcn_bwd_nm3 F16: LG_F_F16X2) against the default 3-way bf16 nm3
kernel on the same inputs: dx, dW, db, node-bias errors relative to scale, and where dx
differs (rows / columns).

  python tools/bpc_check.py
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import numpy as np
import torch

from models import _native as nat
from models.ops import GCNGraph, check, ptr


def main():
    lib = nat.load_library()
    dev = torch.device("cuda:0")
    g = np.load(REPO / "tests/golden/graph_ltown_a.npz")
    N, D = 661, 64
    graph = GCNGraph.build(torch.from_numpy(g["edge_index"]), N, dev)
    cs = torch.cuda.current_stream().cuda_stream
    bad = 0
    for B, mi, mo, nb in ((256, True, True, False), (256, False, True, True), (200, True, False, False),
                          (7, True, True, True)):
        torch.manual_seed(B)
        x = torch.relu(torch.randn(N, B, D, device=dev))
        W = torch.randn(D, D, device=dev) / 8
        bias = torch.randn(D, device=dev)
        dy = torch.randn(N, B, D, device=dev)
        yy = torch.empty_like(x)
        ng = (B + 15) // 16
        bits = torch.zeros(N * ng * 64, device=dev, dtype=torch.int16)
        check(lib.lg_gcn_fwd_nm_bits(ptr(graph.nodetab), ptr(graph.pairs), ptr(x), ptr(W), ptr(bias), ptr(yy), B, N, D,
                                     graph.nnz_cap, nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT, 0.1, 123, 2, cs,
                                     ptr(bits)), "fwd bits")
        slot = torch.full((N,), -1, dtype=torch.int32, device=dev)
        slot[:29] = torch.arange(29, dtype=torch.int32, device=dev)
        fl = (nat.LG_F_MASK_IN if mi else 0) | (nat.LG_F_MASK_OUT if mo else 0)

        def run(extra):
            dx = torch.full_like(x, float("nan"))
            dW, db, dnb = torch.empty(D, D, device=dev), torch.empty(D, device=dev), torch.empty(D, device=dev)
            ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=dev, dtype=torch.uint8)
            check(lib.lg_gcn_bwd_nm_bits(ptr(graph.nodetab_t), ptr(graph.pairs_t), ptr(dy), ptr(yy), ptr(x), ptr(W),
                                         ptr(dx), ptr(dW), ptr(db), ptr(slot) if nb else None, ptr(dnb) if nb else None,
                                         B, N, D, fl | extra, 1.0 / 0.9, 1.0 / 0.9, ptr(ws), cs,
                                         ptr(bits) if mi else None), "bwd")
            torch.cuda.synchronize()
            return dx, dW, db, dnb
        ref = run(0)
        for name, extra in (("pc", nat.LG_F_PC | nat.LG_F_F16X2), ("nm3f16", nat.LG_F_F16X2)):
            got = run(extra)
            errs = []
            for what, a, b in zip(("dx", "dW", "db", "dnb"), got, ref):
                if what == "dnb" and not nb:
                    continue
                e = ((a.double() - b.double()).abs().max() / b.abs().max().clamp_min(1e-30)).item()
                errs.append(f"{what} {e:.2e}")
                bad += not (e <= 2e-6)
            print(f"B={B} mi={mi} mo={mo} nb={nb} {name}: " + ", ".join(errs))
            d = (got[0] - ref[0]).abs()
            if d.max().item() > 1e-3 * ref[0].abs().max().item() or not torch.isfinite(got[0]).all():
                rows = (d.amax(dim=2) > 1e-3).nonzero()
                cols = (d.amax(dim=(0, 1)) > 1e-3).nonzero().flatten().tolist()
                print(f"   dx wrong at {rows.shape[0]} (node, window) rows, e.g. {rows[:8].tolist()}; columns {cols[:64]}")
                print(f"   nan count {int((~torch.isfinite(got[0])).sum())}")
    print("OK" if bad == 0 else f"{bad} MISMATCHES")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
