"""Time single TCN conv layers (lg_tcn_conv_fwd) across batch sizes: python tools/tcn_lab.py 256,1024 [0]."""
import os, sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import torch
from models import _native as nat, tcn_plan
from models.predictor import NormalPredictorTCN
from models.ops import check, ptr
lib = nat.load_library(); dev = torch.device("cuda:0")
BS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [256]
LABS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 4, 7, 8, 15]
m = NormalPredictorTCN(29, 9).eval().to(dev)
plan = tcn_plan.plan_for(36, 36); dp = tcn_plan._DevicePlan(plan, dev); packed = tcn_plan._packed_weights(m, dev)
st = torch.cuda.current_stream().cuda_stream
for B, li in [(B, li) for B in BS for li in (4, 7)]:
    cp = plan.convs[li]; rp = plan.convs[li - 1].rows; rb = plan.convs[li - 2].rows if li % 2 else 0
    xin = torch.randn(B * rp, 128, device=dev); bi = torch.randn(B * rb, 128, device=dev) if rb else None
    out = torch.empty(B * cp.rows, 128, device=dev)
    blk = m.tcn[li // 2]; conv, norm = (blk.conv1.conv, blk.norm1) if li % 2 == 0 else (blk.conv2.conv, blk.norm2)
    for lab in LABS:
        os.environ["LEAKGNN_TCN_LAB"] = str(lab)
        f = lambda: check(lib.lg_tcn_conv_fwd(ptr(xin), ptr(bi), ptr(dp.tables[li]), ptr(packed[li]), ptr(conv.bias),
                                              ptr(norm.weight), ptr(norm.bias), 1e-5, ptr(out), B, rp, rb, cp.rows, 128, st), "c")
        for _ in range(3): f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(30): f()
        b.record(); torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / 30
        print(f"B {B:5d} layer {li} rows {cp.rows} lab {lab:2d}: {us:8.1f} us  {B * cp.rows * 2 * 128 * 384 / us / 1e6:6.1f} TF", flush=True)
