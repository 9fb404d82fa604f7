"""Kernel lab (GPU): every OPT variant of the D = 64 node-major forward (LG_F_LAB_OPT) must
give y and the [y > 0] mask bits bit-identical to OPT 0, in eval and train mode, at the
bench batch and at a ragged one.  LEAKGNN_LIB=leak-det-gnn_amd/lib/lab/libleakgnn.so.

  python tools/nm3_opt_check.py [--opts 1,2,3,...]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import numpy as np
import torch

from models import _native as nat
from models.ops import GCNGraph, check, ptr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opts", default=",".join(str(i) for i in range(1, 16)))
    ap.add_argument("--nm5", action="store_true", help="also the W-in-registers pipeline (LG_F_NM5), bf16 tier too")
    args = ap.parse_args()
    lib = nat.load_library()
    dev = torch.device("cuda:0")
    g = np.load(REPO / "tests/golden/graph_ltown_a.npz")
    N, D = 661, 64
    graph = GCNGraph.build(torch.from_numpy(g["edge_index"]), N, dev)
    cs = torch.cuda.current_stream().cuda_stream
    bad = 0
    for B in (256, 200, 7):
        torch.manual_seed(B)
        x = torch.randn(N, B, D, device=dev)
        W = torch.randn(D, D, device=dev) / 8
        bias = torch.randn(D, device=dev)
        ng = (B + 15) // 16
        for fl in (0, nat.LG_F_DROPOUT):
            def run(opt, extra=0):
                y = torch.full((N, B, D), float("nan"), device=dev)
                m = torch.zeros(N * ng * 64, device=dev, dtype=torch.int16)
                bits = ((0x00001000 | (opt << 8)) if opt is not None else 0) | extra
                check(lib.lg_gcn_fwd_nm_bits(ptr(graph.nodetab), ptr(graph.pairs), ptr(x), ptr(W), ptr(bias), ptr(y),
                                             B, N, D, graph.nnz_cap, nat.LG_F_BIAS | nat.LG_F_RELU | fl | bits, 0.1,
                                             123, 1, cs, ptr(m)), "fwd")
                torch.cuda.synchronize()
                return y, m
            y0, m0 = run(0)
            if args.nm5:
                for name, ex in (("nm5", nat.LG_F_NM5), ("nm5-bf16", nat.LG_F_NM5 | nat.LG_F_BF16),
                                 ("pc", nat.LG_F_PC), ("pc-bf16", nat.LG_F_PC | nat.LG_F_BF16),
                                 ("pc1", nat.LG_F_PC | nat.LG_F_PC1)):
                    ya, ma = run(None, ex)
                    yb, mb = (y0, m0) if "bf16" not in name else run(None, nat.LG_F_BF16)
                    same_y = torch.equal(ya.view(torch.int32), yb.view(torch.int32))
                    same_m = torch.equal(ma, mb)
                    print(f"B={B} drop={bool(fl)} {name}: y {'==' if same_y else '!='} mask {'==' if same_m else '!='}")
                    bad += (not same_y) + (not same_m)
            if args.nm5:  # the fp16x2 transform: fp32-level accuracy, not bit-identical
                ya, ma = run(None, nat.LG_F_NM5 | nat.LG_F_F16X2)
                scale = y0.abs().max().item()
                err = (ya.double() - y0.double()).abs().max().item() / scale
                nbits = int((ma.view(torch.int16) ^ m0.view(torch.int16)).ne(0).sum().item())
                print(f"B={B} drop={bool(fl)} nm5-f16x2: max|dy|/scale = {err:.2e}, mask words differing {nbits}")
                bad += err > 1e-6
                yc, mc = run(None, nat.LG_F_PC | nat.LG_F_F16X2)
                same = torch.equal(ya.view(torch.int32), yc.view(torch.int32)) and torch.equal(ma, mc)
                print(f"B={B} drop={bool(fl)} pc-f16x2 {'==' if same else '!='} nm5-f16x2")
                bad += not same
            for opt in [int(v) for v in args.opts.split(",") if v]:
                y1, m1 = run(opt)
                same_y = torch.equal(y0.view(torch.int32), y1.view(torch.int32))
                same_m = torch.equal(m0, m1)
                print(f"B={B} drop={bool(fl)} opt={opt}: y {'==' if same_y else '!='} mask {'==' if same_m else '!='}")
                bad += (not same_y) + (not same_m)
    print("OK" if bad == 0 else f"{bad} MISMATCHES")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
