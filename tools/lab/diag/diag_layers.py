"""Diagnostic (GPU box): why the second GCN layer of the step is slower than the first.
Times lg_gcn_fwd_nm (train mode, B = 256, L-TOWN-A) with hipExt kernel events in
sequences: x0 -> x1 -> x2 (the step's order), x1 -> x2 alone, repeated layer-2 launches, and
with a 512 MB write in front (cache state like after the GRU forward's gate stores)."""
from __future__ import annotations

import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[3]
for p in (ROOT, ROOT / "leak-det-gnn_amd", ROOT / "tests"):
    sys.path.insert(0, str(p))
from helpers import LTA_INP, lta_ids  # noqa: E402


def main():
    from models import library  # noqa: F401
    from models import ops
    from models import _native as nat
    from models.detector import LeakDetector
    dev = torch.device("cuda:0")
    sensors, pipes = lta_ids()
    m = LeakDetector(LTA_INP, sensors, pipes).to(dev)
    g = m._device_state(dev)[0]
    lib = nat.load_library()
    N, B, D = 661, 256, 64
    x0 = torch.randn(N, B, D, device=dev).relu_()
    W = [torch.randn(D, D, device=dev) / 8 for _ in range(2)]
    b = [torch.randn(D, device=dev) / 10 for _ in range(2)]
    big = torch.empty(128 << 20, device=dev)
    st = nat.stream_of(x0)
    flags = nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT

    def layer(x, l, slot):
        y = torch.empty_like(x)
        nat.check(lib.lg_timing_arm(slot), "arm")
        nat.check(lib.lg_gcn_fwd_nm(nat.ptr(g.nodetab), nat.ptr(g.pairs), nat.ptr(x), nat.ptr(W[l]), nat.ptr(b[l]),
                                    nat.ptr(y), B, N, D, g.col.numel(), flags, 0.1, 1234, l + 1, st), "fwd")
        return y

    import ctypes
    ms = ctypes.c_float()

    def el(slot):
        torch.cuda.synchronize()
        nat.check(lib.lg_timing_elapsed(slot, ctypes.byref(ms)), "el")
        return ms.value * 1e3

    for trial in range(3):
        big.fill_(1.0)  # 512 MB of dirty lines, as after the GRU gate stores
        x1 = layer(x0, 0, 0)
        x2 = layer(x1, 1, 1)
        x2b = layer(x1, 1, 2)
        x3 = layer(x2, 1, 3)
        print(f"after 512MB fill: L1 {el(0):6.2f}  L2 {el(1):6.2f}  L2 again {el(2):6.2f}  L2 on x2 {el(3):6.2f} us")
        x1 = layer(x0, 0, 4)
        x2 = layer(x1, 1, 5)
        print(f"warm:             L1 {el(4):6.2f}  L2 {el(5):6.2f} us")
        del x1, x2, x2b, x3


if __name__ == "__main__":
    main()
