"""Kernel micro-benchmark (GPU): times individual libleakgnn kernels in isolation with
HIP events on the launch stream.  Used for tuning and under rocprofv3 --pmc.

  python tools/kbench.py [--which gcn_fwd,gcn_bwd,spmm,edge_fwd,edge_bwd,gru_fwd,gru_bwd] [--B 256] [--iters 50]
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import numpy as np
import torch

from models import _native as nat
from models import ops
from models.ops import GCNGraph, Incidence, check, ptr


GRAPH = True  # time iters launches captured in one HIP graph (host launch cost out of the loop)


def timeit(fn, iters):
    """Mean device time per call (us): `iters` back-to-back calls captured in one HIP graph
    and replayed (so Python / ctypes launch overhead cannot starve the GPU between these
    short kernels); eager launches with --eager."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(iters):
                    fn()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / (3 * iters)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def stamps_summary(lib, launch):
    """One eager launch of the LG_NM3_STAMPS lab forward, then its per-wave timeline: start /
    end skew, tiles per wave and the three phases per tile (rows waited for and accumulated,
    transform, epilogue + stores), in microseconds at the clock derived from the stamps."""
    import ctypes
    lib.lg_lab_nm3_stamps_clear.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    torch.cuda.synchronize()
    check(lib.lg_lab_nm3_stamps_clear(), "stamps clear")
    torch.cuda.synchronize()
    launch()
    torch.cuda.synchronize()
    n = 8192 * 24
    buf = np.zeros(n, dtype=np.uint64)
    check(lib.lg_lab_nm3_stamps(buf.ctypes.data, n), "stamps read")
    st = buf.reshape(8192, 24).astype(np.int64)
    st = st[st[:, 0] != 0]
    rt0, rt1, c0, c1 = st[:, 0], st[:, 22], st[:, 1], st[:, 21]
    ghz = float(np.median((c1 - c0) / np.maximum(rt1 - rt0, 1))) * 0.1  # memrealtime is 100 MHz
    us = lambda cyc: cyc / (ghz * 1e3)
    t0 = rt0.min()
    start = (rt0 - t0) / 100.0
    end = (rt1 - t0) / 100.0
    tiles = np.array([sum(1 for t in range(6) if r[5 + 3 * t] != 0) for r in st])
    ph = {"wait_acc": [], "transform": [], "epilogue": [], "staging": us(st[:, 2] - st[:, 1]).tolist()}
    for r in st:
        prev = r[2]
        for t in range(6):
            if r[5 + 3 * t] == 0:
                break
            ph["wait_acc"].append(us(r[3 + 3 * t] - prev))
            ph["transform"].append(us(r[4 + 3 * t] - r[3 + 3 * t]))
            ph["epilogue"].append(us(r[5 + 3 * t] - r[4 + 3 * t]))
            prev = r[5 + 3 * t]
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (10, 50, 90, 99)]
    xcc = (st[:, 23] >> 32) & 0xF
    return {"waves": int(len(st)), "clock_GHz": round(ghz, 3), "span_us": round(float(end.max()), 3),
            "start_us_p10_50_90_99": q(start), "end_us_p10_50_90_99": q(end),
            "life_us_mean": round(float((end - start).mean()), 3),
            "tiles_hist": {int(k): int(v) for k, v in zip(*np.unique(tiles, return_counts=True))},
            **{f"{k}_us_p10_50_90_99": q(v) for k, v in ph.items() if len(v)},
            "end_by_xcc_us": [round(float(end[xcc == i].max()), 3) if (xcc == i).any() else None for i in range(8)]}


def bwd_stamps_summary(lib, launch):
    """k_gcn_bwd_nm3 per-wave timeline (LG_NM3_STAMPS build): W staging, each tile's duration
    (end stamp to end stamp; the first from the staging barrier), tiles per wave, the wave ends
    and the latest end per XCD, in microseconds."""
    import ctypes
    lib.lg_lab_nm3_stamps_clear.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    torch.cuda.synchronize()
    check(lib.lg_lab_nm3_stamps_clear(), "stamps clear")
    torch.cuda.synchronize()
    launch()
    torch.cuda.synchronize()
    n = 8192 * 24
    buf = np.zeros(n, dtype=np.uint64)
    check(lib.lg_lab_nm3_stamps(buf.ctypes.data, n), "stamps read")
    st = buf.reshape(8192, 24).astype(np.int64)
    st = st[st[:, 0] != 0]
    rt0, rt1, c0, c1 = st[:, 0], st[:, 22], st[:, 1], st[:, 21]
    ghz = float(np.median((c1 - c0) / np.maximum(rt1 - rt0, 1))) * 0.1
    us = lambda cyc: cyc / (ghz * 1e3)
    t0 = rt0.min()
    start, end = (rt0 - t0) / 100.0, (rt1 - t0) / 100.0
    tiles = np.array([int((r[3:19] != 0).sum()) for r in st])
    dur, first, last = [], [], []
    for r in st:
        prev = r[2]
        for t in range(16):
            if r[3 + t] == 0:
                break
            d = us(r[3 + t] - prev)
            dur.append(d)
            if t == 0:
                first.append(d)
            prev = r[3 + t]
        if r[3] != 0:
            last.append(us(r[21] - prev))
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (10, 50, 90, 99)]
    xcc = (st[:, 23] >> 32) & 0xF
    return {"waves": int(len(st)), "clock_GHz": round(ghz, 3), "span_us": round(float(end.max()), 3),
            "start_us_p10_50_90_99": q(start), "end_us_p10_50_90_99": q(end),
            "staging_us_p10_50_90_99": q(us(st[:, 2] - st[:, 1])),
            "tile_us_p10_50_90_99": q(dur), "first_tile_us_p10_50_90_99": q(first) if first else None,
            "epilogue_us_p10_50_90_99": q(last) if last else None,
            "tiles_hist": {int(k): int(v) for k, v in zip(*np.unique(tiles, return_counts=True))},
            "end_by_tiles_p50": {int(k): round(float(np.median(end[tiles == k])), 3) for k in np.unique(tiles)},
            "end_by_xcc_us": [round(float(end[xcc == i].max()), 3) if (xcc == i).any() else None for i in range(8)]}


def gru_stamps_summary(lib, launch, nst=48, steps=8):
    """k_gru_bwd2 per-step timeline (stamps build): for 8 mid-kernel steps of every wave, the
    clocks at the step's start (a), before its barrier (b), after it (c) and once dh is formed
    (d).  Medians over waves and steps, in clock cycles: a->b (elementwise part, refill, the
    deferred dW, rescale), b->c (barrier wait), c->d (dh product), d->next a, the step period."""
    lib.lg_lab_gru_stamps_clear.restype = ctypes.c_int
    lib.lg_lab_gru_stamps.restype = ctypes.c_int
    lib.lg_lab_gru_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    check(lib.lg_lab_gru_stamps_clear(), "gru stamps clear")
    launch()
    torch.cuda.synchronize()
    n = 256 * 8 * nst
    buf = np.zeros(n, dtype=np.uint64)
    check(lib.lg_lab_gru_stamps(buf.ctypes.data, n), "gru stamps read")
    a = buf.reshape(256 * 8, nst)[:, :6 * steps].reshape(-1, steps, 6).astype(np.float64)
    a = a[(a > 0).all(axis=(1, 2))]  # waves that stamped every step (slot order: t descending)
    if not len(a):
        return {"waves": 0}
    d = {"waves": int(len(a)),
         "start_to_gates_done": a[:, :, 4] - a[:, :, 0],
         "gates_done_to_refill_issued": a[:, :, 5] - a[:, :, 4],
         "refill_to_barrier": a[:, :, 1] - a[:, :, 5],
         "elementwise_dw_to_barrier": np.diff(a[:, :, 0:2], axis=2)[..., 0],
         "barrier_wait": np.diff(a[:, :, 1:3], axis=2)[..., 0],
         "dh_product": np.diff(a[:, :, 2:4], axis=2)[..., 0],
         "dh_to_next_step": a[:, 1:, 0] - a[:, :-1, 3],
         "step_period": a[:, 1:, 0] - a[:, :-1, 0]}
    out = {"waves": d.pop("waves")}
    for k, v in d.items():
        out[k + "_cyc_p10_50_90"] = [round(float(np.percentile(v, p)), 1) for p in (10, 50, 90)]
    return out


def pc_stamps_summary(lib, launch, waves_per_wg=12, prod=4):
    """Per-wave timeline of one eager k_gcn_fwd_pc launch (LG_NM3_STAMPS build): producers and
    consumers separately — start / end, tiles handed over / stored, the per-tile interval, and
    the tail (last end minus the median end), the end by tile count and by XCC."""
    import ctypes
    lib.lg_lab_nm3_stamps_clear.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    torch.cuda.synchronize()
    check(lib.lg_lab_nm3_stamps_clear(), "stamps clear")
    torch.cuda.synchronize()
    launch()
    torch.cuda.synchronize()
    n = 8192 * 24
    buf = np.zeros(n, dtype=np.uint64)
    check(lib.lg_lab_nm3_stamps(buf.ctypes.data, n), "stamps read")
    st = buf.reshape(8192, 24).astype(np.int64)
    rows = np.nonzero(st[:, 0] != 0)[0]
    st = st[rows]
    role = np.where((rows % waves_per_wg) < prod, "prod", "cons")
    rt0, rt1, c0, c1 = st[:, 0], st[:, 22], st[:, 1], st[:, 21]
    ghz = float(np.median((c1 - c0) / np.maximum(rt1 - rt0, 1))) * 0.1
    us = lambda cyc: cyc / (ghz * 1e3)
    t0 = rt0.min()
    start = (rt0 - t0) / 100.0
    end = (rt1 - t0) / 100.0
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (10, 50, 90, 99, 100)] if len(a) else []
    xcc = (st[:, 23] >> 32) & 0xF
    out = {"waves": int(len(st)), "clock_GHz": round(ghz, 3), "span_us": round(float(end.max()), 3)}
    for r in ("prod", "cons"):
        m = role == r
        sr = st[m]
        tiles = (sr[:, 3:19] != 0).sum(1)
        gaps = []
        for row, nt in zip(sr, tiles):
            prev = row[2]
            for t in range(min(nt, 16)):
                gaps.append(us(row[3 + t] - prev))
                prev = row[3 + t]
        e = end[m]
        out[r] = {"start_us_p10_50_90_99_max": q(start[m]), "end_us_p10_50_90_99_max": q(e),
                  "tail_us": round(float(e.max() - np.median(e)), 3),
                  "staging_us_p50": round(float(np.median(us(sr[:, 2] - sr[:, 1]))), 3),
                  "tiles_hist": {int(k): int(v) for k, v in zip(*np.unique(tiles, return_counts=True))},
                  "tile_us_p10_50_90_99_max": q(gaps),
                  "end_by_tiles_p50": {int(k): round(float(np.median(e[tiles == k])), 3) for k in np.unique(tiles)},
                  "end_by_xcc_max": [round(float(e[xcc[m] == i].max()), 3) if (xcc[m] == i).any() else None
                                     for i in range(8)]}
    return out


def pc_probe_summary(lib, launch, waves_per_wg=12, prod=4, reps=5):
    """Product-speed timeline of k_gcn_fwd_pc (LG_PC_PROBE build: per wave only start, after-W-
    staging and end clocks plus its tile count, stored once at the wave's end).  The launch is
    run `reps` times back to back (the last one is read), so it starts the way it does in a
    step: behind another kernel.  Per role: start / staging-done / end (us from the first wave's
    start), the tail (last end minus median end), the end by tile count and by XCC."""
    lib.lg_lab_nm3_stamps_clear.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.restype = ctypes.c_int
    lib.lg_lab_nm3_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    torch.cuda.synchronize()
    for _ in range(reps):
        launch()
    torch.cuda.synchronize()
    check(lib.lg_lab_nm3_stamps_clear(), "stamps clear")
    torch.cuda.synchronize()
    launch()
    torch.cuda.synchronize()
    n = 8192 * 24
    buf = np.zeros(n, dtype=np.uint64)
    check(lib.lg_lab_nm3_stamps(buf.ctypes.data, n), "stamps read")
    st = buf.reshape(8192, 24).astype(np.int64)
    rows = np.nonzero(st[:, 0] != 0)[0]
    st = st[rows]
    role = np.where((rows % waves_per_wg) < prod, "prod", "cons")
    rt0, rt1, c0, c1, c2 = st[:, 0], st[:, 22], st[:, 1], st[:, 2], st[:, 21]
    ghz = float(np.median((c2 - c0) / np.maximum(rt1 - rt0, 1))) * 0.1
    t0 = rt0.min()
    start = (rt0 - t0) / 100.0
    end = (rt1 - t0) / 100.0
    staged = start + (c1 - c0) / (ghz * 1e3)
    q = lambda a: [round(float(np.percentile(a, p)), 3) for p in (0, 10, 50, 90, 99, 100)] if len(a) else []
    xcc = (st[:, 23] >> 32) & 0xF
    out = {"waves": int(len(st)), "clock_GHz": round(ghz, 3), "span_us": round(float(end.max()), 3),
           "percentiles": [0, 10, 50, 90, 99, 100]}
    for r in ("prod", "cons"):
        m = role == r
        e, tiles = end[m], st[m, 3]
        out[r] = {"start_us": q(start[m]), "staged_us": q(staged[m]), "end_us": q(e),
                  "tail_us": round(float(e.max() - np.median(e)), 3),
                  "tiles_hist": {int(k): int(v) for k, v in zip(*np.unique(tiles, return_counts=True))},
                  "end_by_tiles_p50": {int(k): round(float(np.median(e[tiles == k])), 3) for k in np.unique(tiles)},
                  "end_by_xcc_max": [round(float(e[xcc[m] == i].max()), 3) if (xcc[m] == i).any() else None
                                     for i in range(8)]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="gcn_fwd,gcn_fwd_train,gcn_bwd,gcn_fwd_nm,gcn_fwd_nm_train,gcn_bwd_nm,spmm,"
                                       "edge_fwd,edge_bwd,gru_fwd,gru_bwd")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--graph", default="ltown", choices=["ltown", "selfonly", "ring"],
                    help="lab graphs on L-TOWN-A's 661 nodes: selfonly = no edges (one gathered block per "
                         "tile), ring = a cycle (three blocks per tile, neighbours adjacent)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--lab", default="", help="comma list of extra lg_gcn_fwd flag bits (kernel lab switches)")
    ap.add_argument("--edgelab", default="", help="comma list of lg_edge_head_fwd lab bits (1 nomfma, 2 noload, "
                                                   "4 nosplit; LEAKGNN_LIB=lib/lab build only)")
    ap.add_argument("--edgebwdlab", default="", help="comma list of streamed EdgeHead backward lab bits (1 no dW1 "
                                                      "MFMA, 2 no dfeat MFMA, 4 no scatter; LEAKGNN_LIB=lib/lab only)")
    ap.add_argument("--nmlab", default="", help="comma list of lg_gcn_fwd_nm schedules: v1 or bpc<n> (train mode)")
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of a replayed HIP graph")
    ap.add_argument("--stamps", action="store_true", help="per-wave timeline of each --nmlab train launch "
                                                           "(LEAKGNN_LIB=lib/lab_stamps build only)")
    ap.add_argument("--probe", action="store_true", help="product-speed start/end timeline of each --nmlab train "
                                                          "launch of k_gcn_fwd_pc (LEAKGNN_LIB=lib/probe build only)")
    args = ap.parse_args()
    global GRAPH
    GRAPH = not args.eager
    lib = nat.load_library()
    dev = torch.device("cuda:0")
    g = np.load(REPO / "tests/golden/graph_ltown_a.npz")
    ei = torch.from_numpy(g["edge_index"])
    N, D, B = 661, 64, args.B
    if args.graph == "selfonly":
        ei = torch.zeros(2, 0, dtype=torch.long)
    elif args.graph == "ring":
        a = torch.arange(N)
        b = (a + 1) % N
        ei = torch.stack([torch.cat([a, b]), torch.cat([b, a])])
    graph = GCNGraph.build(ei, N, dev)
    inc = Incidence.build(torch.from_numpy(g["pipe_ends"]), N, dev)
    P = inc.num_pipes
    def cs():  # launch stream = torch's current stream at CALL time (graph capture switches it)
        return torch.cuda.current_stream().cuda_stream
    x = torch.randn(B, N, D, device=dev)
    y = torch.empty_like(x)
    W = torch.randn(D, D, device=dev) / 8
    bias = torch.randn(D, device=dev)
    res = {}
    E1 = graph.nnz_cap
    fwd_bytes = 8 * B * N * D + 4 * (N + 1) + 8 * E1
    which = args.which.split(",")
    if "gcn_fwd" in which:
        f = lambda: check(lib.lg_gcn_fwd(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(W), ptr(bias),
                                         ptr(y), B, N, D, E1, nat.LG_F_BIAS | nat.LG_F_RELU, 0.0, 0, 0, cs()), "fwd")
        t = timeit(f, args.iters)
        res["gcn_fwd"] = {"us": t, "GBps": fwd_bytes / t / 1e3}
    if "gcn_fwd_train" in which:
        f = lambda: check(lib.lg_gcn_fwd(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(W), ptr(bias),
                                         ptr(y), B, N, D, E1, nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT, 0.1,
                                         123, 1, cs()), "fwd")
        t = timeit(f, args.iters)
        res["gcn_fwd_train"] = {"us": t, "GBps": fwd_bytes / t / 1e3}
    for lab in [int(v) for v in args.lab.split(",") if v]:
        f = lambda: check(lib.lg_gcn_fwd(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(W), ptr(bias),
                                         ptr(y), B, N, D, E1, nat.LG_F_BIAS | nat.LG_F_RELU | lab, 0.0, 0, 0, cs()), "fwd")
        res[f"gcn_fwd_lab{lab >> 20}"] = {"us": timeit(f, args.iters)}
    # node-major kernels (x, y as [N][B][D]; same bytes)
    for name, fl in (("gcn_fwd_nm", 0), ("gcn_fwd_nm_train", nat.LG_F_DROPOUT)):
        if name in which:
            f = lambda fl=fl: check(lib.lg_gcn_fwd_nm(ptr(graph.nodetab), ptr(graph.pairs), ptr(x), ptr(W), ptr(bias),
                                                      ptr(y), B, N, D, E1, nat.LG_F_BIAS | nat.LG_F_RELU | fl, 0.1, 123,
                                                      1, cs()), name)
            t = timeit(f, args.iters)
            res[name] = {"us": t, "GBps": fwd_bytes / t / 1e3}
    ymask = torch.empty(N * ((B + 15) // 16) * 64, device=dev, dtype=torch.int16)
    for lab in [v for v in args.nmlab.split(",") if v]:
        bits, with_mask = 0, False
        for tok in lab.split("+"):  # dflt | x3 | nm3 | f32 | bf16 | pc | mask
            bits |= {"f32": nat.LG_F_F32_MFMA, "bf16": nat.LG_F_BF16, "pc": nat.LG_F_PC, "x3": nat.LG_F_BF16X3,
                     "nm3": nat.LG_F_NM3, "dflt": 0}.get(tok, 0)
            with_mask |= tok == "mask"  # the last layer's form: [y > 0] bits written beside y
        for mode, fl in (("eval", 0), ("train", nat.LG_F_DROPOUT)):
            f = lambda fl=fl, bits=bits, wm=with_mask: check(lib.lg_gcn_fwd_nm_bits(
                ptr(graph.nodetab), ptr(graph.pairs), ptr(x), ptr(W), ptr(bias), ptr(y), B, N, D, E1,
                nat.LG_F_BIAS | nat.LG_F_RELU | fl | bits, 0.1, 123, 1, cs(), ptr(ymask) if wm else None), "nmlab")
            t = timeit(f, args.iters)
            res[f"gcn_fwd_nm_{lab}_{mode}"] = {"us": t, "GBps": fwd_bytes / t / 1e3}
            if args.probe and mode == "train" and hasattr(lib, "lg_lab_nm3_stamps"):
                res[f"probe_{lab}"] = pc_probe_summary(lib, f)
            if args.stamps and mode == "train" and hasattr(lib, "lg_lab_nm3_stamps"):
                pcs = not (bits & (nat.LG_F_NM3 | nat.LG_F_F32_MFMA)) and not (bits & nat.LG_F_BF16 and not bits & nat.LG_F_PC)
                res[f"stamps_{lab}"] = pc_stamps_summary(lib, f) if pcs else stamps_summary(lib, f)
    # gcn_bwd_nm: the training step's layer-2 backward (output mask as the forward's ymask
    # bits); gcn_bwd_nm_y: the same with the mask gathered from y
    for name, fl, nbias in (("gcn_bwd_nm", nat.LG_F_MASK_IN | nat.LG_F_MASK_OUT, False),
                            ("gcn_bwd_nm_y", nat.LG_F_MASK_IN | nat.LG_F_MASK_OUT, False),
                            ("gcn_bwd_nm_l0", nat.LG_F_MASK_OUT, True),
                            ("gcn_bwd_nm_l0s", nat.LG_F_MASK_OUT | nat.LG_F_DX_SENSOR_ROWS, True),
                            ):
        if name not in which:
            continue
        dy = torch.randn_like(x)
        yy = torch.relu(torch.randn_like(x))
        dx = torch.empty_like(x)
        dW = torch.empty(D, D, device=dev)
        db = torch.empty(D, device=dev)
        slot = torch.full((N,), -1, dtype=torch.int32, device=dev)
        slot[:29] = torch.arange(29, dtype=torch.int32, device=dev)
        dnb = torch.empty(D, device=dev)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=dev, dtype=torch.uint8)
        bits = None
        if name == "gcn_bwd_nm":  # the mask bits of yy = dropout(relu(layer(x))) from the forward
            bits = torch.empty(N * ((B + 15) // 16) * 64, device=dev, dtype=torch.int16)
            check(lib.lg_gcn_fwd_nm_bits(ptr(graph.nodetab), ptr(graph.pairs), ptr(x), ptr(W), ptr(bias), ptr(yy), B,
                                         N, D, E1, nat.LG_F_BIAS | nat.LG_F_RELU | nat.LG_F_DROPOUT, 0.1, 123, 2,
                                         cs(), ptr(bits)), "fwd bits")
        f = lambda fl=fl, nbias=nbias, dy=dy, yy=yy, dx=dx, dW=dW, db=db, slot=slot, dnb=dnb, ws=ws, bits=bits: check(
            lib.lg_gcn_bwd_nm_bits(ptr(graph.nodetab_t), ptr(graph.pairs_t), ptr(dy), ptr(yy), ptr(x), ptr(W),
                                   ptr(dx), ptr(dW), ptr(db), ptr(slot) if nbias else None,
                                   ptr(dnb) if nbias else None, B, N, D, fl, 1.0, 1.0, ptr(ws), ws.numel(), cs(),
                                   ptr(bits) if bits is not None else None), name)
        t = timeit(f, args.iters)
        if bits is not None:
            byts = 12 * B * N * D + bits.numel() * 2
        else:
            byts = (16 if fl & nat.LG_F_MASK_IN else 12) * B * N * D
        res[name] = {"us": t, "GBps": byts / t / 1e3}
        if args.stamps and hasattr(lib, "lg_lab_nm3_stamps"):
            res[name]["stamps"] = bwd_stamps_summary(lib, f)
    if "node_init" in which:  # sensor projection + node init (x0 = B*N*D fp32 written, node-major)
        S5 = 29
        slot = torch.full((N,), -1, dtype=torch.int32, device=dev)
        slot[:S5] = torch.arange(S5, dtype=torch.int32, device=dev)
        sidx = torch.arange(S5, dtype=torch.int64, device=dev)
        hs = torch.randn(B, S5, D, device=dev)
        Wp = torch.randn(D, D + 1, device=dev) / 8
        x0 = torch.empty(N, B, D, device=dev)
        f = lambda: check(lib.lg_node_init_proj_fwd(ptr(slot), ptr(sidx), ptr(hs), ptr(Wp), ptr(bias), ptr(x0), B, N,
                                                    S5, D, D, nat.LG_F_DROPOUT | nat.LG_F_NODE_MAJOR, 0.1, 123, 0,
                                                    cs()), "node_init")
        t = timeit(f, args.iters)
        res["node_init"] = {"us": t, "GBps": 4 * B * N * D / t / 1e3}
    if any(k in which for k in ("node_init_bits", "gcn_fwd_x0", "gcn_bwd_x0")):  # the compressed node init path
        S5 = 29
        slot = torch.full((N,), -1, dtype=torch.int32, device=dev)
        slot[:S5] = torch.arange(S5, dtype=torch.int32, device=dev)
        sidx = torch.arange(S5, dtype=torch.int64, device=dev)
        hs = torch.randn(B, S5, D, device=dev)
        Wp = torch.randn(D, D + 1, device=dev) / 8
        xs0 = torch.empty(S5, B, D, device=dev)
        nbits = N * ((B + 15) // 16) * 64
        x0b = torch.empty(nbits, device=dev, dtype=torch.int16)
        for nm_, S_, sl_ in (("node_init_bits", S5, slot), ("node_init_bits_s0", 0, torch.full_like(slot, -1))):
            f = lambda S_=S_, sl_=sl_: check(lib.lg_node_init_bits_fwd(ptr(sl_), ptr(sidx), ptr(hs), ptr(Wp), ptr(bias),
                                                                       ptr(xs0), ptr(x0b), B, N, S_, D, D, nat.LG_F_DROPOUT,
                                                                       0.1, 123, 0, cs()), nm_)
            t = timeit(f, args.iters)
            res[nm_] = {"us": t, "GBps": (nbits * 2 + 4 * S_ * B * D) / t / 1e3}
        f()
        mk = ops.SensorMarks.build(graph, slot)
        fx = lambda: check(lib.lg_gcn_fwd_nm_x0(ptr(mk.nodetab_s), ptr(mk.pairs_s), ptr(xs0), ptr(x0b), ptr(bias), ptr(W),
                                                ptr(bias), ptr(y), B, N, S5, D, nat.LG_F_BIAS | nat.LG_F_RELU |
                                                nat.LG_F_DROPOUT, 0.1, 123, 1, cs()), "fwd x0")
        t = timeit(fx, args.iters)
        res["gcn_fwd_x0"] = {"us": t, "GBps": (4 * B * N * D + nbits * 2 + 4 * S5 * B * D) / t / 1e3}
        if args.probe and hasattr(lib, "lg_lab_nm3_stamps"):
            res["probe_x0"] = pc_probe_summary(lib, fx)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        dW, db, dnb = torch.empty(D, D, device=dev), torch.empty(D, device=dev), torch.empty(D, device=dev)
        ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=dev, dtype=torch.uint8)
        fb = lambda: check(lib.lg_gcn_bwd_nm_x0(ptr(graph.nodetab_t), ptr(graph.pairs_t), ptr(mk.pos_slot_t), ptr(dy),
                                                ptr(xs0), ptr(x0b), ptr(bias), ptr(W), ptr(dx), ptr(dW), ptr(db),
                                                ptr(slot), ptr(dnb), B, N, S5, D,
                                                nat.LG_F_MASK_OUT | nat.LG_F_DX_SENSOR_ROWS | nat.LG_F_DROPOUT, 0.1,
                                                1.0 / 0.9, ptr(ws), ws.numel(), cs()), "bwd x0")
        t = timeit(fb, args.iters)
        res["gcn_bwd_x0"] = {"us": t, "GBps": (4 * B * N * D) / t / 1e3}
    if "c5_fwd" in which or "c5_bwd" in which or "c5_fwd_wm" in which:  # BASELINE configs[4]: one 100k-node graph, B = 1, GCNConv's launches
        from models.synth import synthetic_pipe_graph
        ei5, _ = synthetic_pipe_graph(100_000, 150_000, seed=0)
        N5 = 100_000
        g5 = GCNGraph.build(ei5, N5, dev)
        x5 = torch.randn(N5, D, device=dev)
        y5 = torch.empty_like(x5)
        b5 = 8 * N5 * D + 4 * (N5 + 1) + 8 * (int(ei5.shape[1]) + N5)  # 54.8 MB
        # c5_fwd / c5_bwd: the row-tile kernels (lg_gcn_{fwd,bwd}_rows); *_wm: window-major (the product's)
        f = lambda: check(lib.lg_gcn_fwd_rows(ptr(g5.nodetab), ptr(g5.pairs), ptr(x5), ptr(W), ptr(bias), ptr(y5), N5,
                                              D, nat.LG_F_BIAS, cs()), "c5 fwd")
        fwm = lambda: check(lib.lg_gcn_fwd(ptr(g5.rowptr), ptr(g5.col), ptr(g5.w), ptr(x5), ptr(W), ptr(bias), ptr(y5),
                                           1, N5, D, g5.col.numel(), nat.LG_F_BIAS, 0.0, 0, 0, cs()), "c5 fwd wm")
        if "c5_fwd" in which:
            t = timeit(f, args.iters)
            res["c5_fwd"] = {"us": t, "GBps": b5 / t / 1e3}
            if args.stamps and hasattr(lib, "lg_lab_nm3_stamps"):
                res["stamps_c5_fwd"] = stamps_summary(lib, f)
        if "c5_fwd" in which or "c5_fwd_wm" in which:
            t = timeit(fwm, args.iters)
            res["c5_fwd_wm"] = {"us": t, "GBps": b5 / t / 1e3}
        if "c5_copy" in which:  # the floor: x -> y of the same bytes (torch copy_ and the library's copy)
            t = timeit(lambda: y5.copy_(x5), args.iters)
            res["c5_copy_torch"] = {"us": t, "GBps": 8 * N5 * D / t / 1e3}
            t = timeit(lambda: check(lib.lg_stream_copy(ptr(x5), ptr(y5), 4 * N5 * D, cs()), "copy"), args.iters)
            res["c5_copy_lg"] = {"us": t, "GBps": 8 * N5 * D / t / 1e3}
        if "c5_spmm" in which:
            t = timeit(lambda: check(lib.lg_spmm(ptr(g5.rowptr), ptr(g5.col), ptr(g5.w), ptr(x5), ptr(y5), 1, N5, D,
                                                 g5.col.numel(), cs()), "c5 spmm"), args.iters)
            res["c5_spmm"] = {"us": t, "GBps": b5 / t / 1e3}
        if "c5_bwd" in which:
            dy5 = torch.randn_like(x5)
            dx5 = torch.empty_like(x5)
            dW5, db5 = torch.empty(D, D, device=dev), torch.empty(D, device=dev)
            ws5 = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=dev, dtype=torch.uint8)
            wsr = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=dev, dtype=torch.uint8)
            f = lambda: check(lib.lg_gcn_bwd_rows(ptr(g5.nodetab_t), ptr(g5.pairs_t), ptr(dy5), ptr(x5), ptr(W),
                                                  ptr(dx5), ptr(dW5), ptr(db5), N5, D, ptr(wsr), wsr.numel(), cs()), "c5 bwd")
            t = timeit(f, args.iters)
            res["c5_bwd"] = {"us": t, "GBps": (b5 + 4 * N5 * D) / t / 1e3}
            fwm = lambda: check(lib.lg_gcn_bwd(ptr(g5.rowptr_t), ptr(g5.col_t), ptr(g5.w_t), ptr(dy5), None, ptr(x5),
                                               ptr(W), ptr(dx5), ptr(dW5), ptr(db5), None, None, 1, N5, D,
                                               g5.col_t.numel(), 0, 1.0, 1.0, ptr(ws5), ws5.numel(), cs()), "c5 bwd wm")
            t = timeit(fwm, args.iters)
            res["c5_bwd_wm"] = {"us": t, "GBps": (b5 + 4 * N5 * D) / t / 1e3}
    if "copy" in which:  # torch device copy of the same bytes: x (B*N*D fp32) -> y
        f = lambda: y.copy_(x)
        t = timeit(f, args.iters)
        res["copy"] = {"us": t, "GBps": 8 * B * N * D / t / 1e3}
    if "spmm" in which:
        f = lambda: check(lib.lg_spmm(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(y), B, N, D, E1,
                                      cs()), "spmm")
        t = timeit(f, args.iters)
        res["spmm"] = {"us": t, "GBps": fwd_bytes / t / 1e3}
    if "gcn_bwd" in which:
        dy = torch.randn_like(x)
        yy = torch.relu(torch.randn_like(x))
        dx = torch.empty_like(x)
        dW = torch.empty(D, D, device=dev)
        db = torch.empty(D, device=dev)
        ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=dev, dtype=torch.uint8)
        f = lambda: check(lib.lg_gcn_bwd(ptr(graph.rowptr_t), ptr(graph.col_t), ptr(graph.w_t), ptr(dy), ptr(yy),
                                         ptr(x), ptr(W), ptr(dx), ptr(dW), ptr(db), None, None, B, N, D, E1,
                                         nat.LG_F_MASK_IN | nat.LG_F_MASK_OUT, 1.0, 1.0, ptr(ws), ws.numel(), cs()), "bwd")
        t = timeit(f, args.iters)
        res["gcn_bwd"] = {"us": t, "GBps": (16 * B * N * D) / t / 1e3}
    if "edge_fwd" in which or "edge_bwd" in which or "edge_bwd_stream" in which:
        W1 = torch.randn(128, 3 * D, device=dev) / 16
        b1 = torch.randn(128, device=dev)
        W2 = torch.randn(1, 128, device=dev) / 8
        b2 = torch.randn(1, device=dev)
        lo = torch.empty(B, P, device=dev)
        hid = torch.empty(B * P, 128, device=dev)
        f = lambda: check(lib.lg_edge_head_fwd(ptr(inc.ends), ptr(x), ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(lo), P,
                                               ptr(hid), B, N, P, D, 128, nat.LG_F_DROPOUT, 0.1, 5, 101, cs()), "edge fwd")
        if "edge_fwd" in which:
            t = timeit(f, args.iters)
            res["edge_fwd"] = {"us": t, "TFLOPs": 2 * B * P * 3 * D * 128 / t / 1e6}
            labs = [(f"edge_fwd_eval_lab{v}", v << 28, None) for v in (int(x) for x in args.edgelab.split(",") if x)]
            for name, fl, hp in [("edge_fwd_x3", nat.LG_F_DROPOUT | nat.LG_F_BF16X3, hid),
                                 ("edge_fwd_nohid", nat.LG_F_DROPOUT, None), ("edge_fwd_eval", 0, None)] + labs:
                g = lambda fl=fl, hp=hp: check(lib.lg_edge_head_fwd(ptr(inc.ends), ptr(x), ptr(W1), ptr(b1), ptr(W2),
                                                                    ptr(b2), ptr(lo), P, ptr(hp) if hp is not None else None, B, N, P, D, 128, fl, 0.1,
                                                                    5, 101, cs()), name)
                t = timeit(g, args.iters)
                res[name] = {"us": t, "TFLOPs": 2 * B * P * 3 * D * 128 / t / 1e6}
        else:
            f()
        if "edge_bwd" in which or "edge_bwd_stream" in which:  # edge_bwd_stream alone: only the streamed launch
            only_stream = "edge_bwd" not in which
            dl = torch.randn(B, P, device=dev)
            dpipe = torch.empty(B, P, 2, D, device=dev)
            dW1, db1, dW2, db2 = (torch.empty_like(t) for t in (W1, b1, W2, b2))
            ws = torch.empty(int(lib.lg_edge_head_bwd_workspace_bytes(B, P, D, 128)), device=dev, dtype=torch.uint8)
            f = lambda: check(lib.lg_edge_head_bwd(ptr(inc.ends), ptr(x), ptr(W1), ptr(W2), ptr(hid), ptr(dl), P,
                                                   ptr(dpipe), ptr(dW1), ptr(db1), ptr(dW2), ptr(db2), B, N, P, D, 128,
                                                   nat.LG_F_DROPOUT, 0.1, ptr(ws), ws.numel(), cs()), "edge bwd")
            if not only_stream:
                t = timeit(f, args.iters)
                res["edge_bwd"] = {"us": t, "TFLOPs": 2 * 2 * B * P * 3 * D * 128 / t / 1e6}
            # with the node scatter fused, node-major h as in the step: per window (ABI 19) and
            # streamed per tile through the pipe schedule (ABI 22)
            xn = x.transpose(0, 1).contiguous()
            dl1 = torch.randn(B, P + 1, device=dev)
            dpool = torch.randn(B, D, device=dev)
            dh = torch.empty_like(xn)
            sched, hdr = inc.schedule(D)
            hdr_c = (ctypes.c_int32 * 16)(*hdr)
            labs = [(f"edge_bwd_stream_lab{v}", sched, hdr_c, v << 28)
                    for v in (int(x) for x in args.edgebwdlab.split(",") if x)]
            runs = [("edge_bwd_scat", None, None, 0), ("edge_bwd_stream", sched, hdr_c, 0)] + labs
            for name, sp, hp, lb in (runs[1:2] if only_stream else runs):
                g = lambda sp=sp, hp=hp, lb=lb: check(lib.lg_edge_head_bwd_scatter(
                    ptr(inc.ends), ptr(xn), ptr(W1), ptr(W2), ptr(hid), ptr(dl1), P + 1, ptr(dpipe), ptr(dW1), ptr(db1),
                    ptr(dW2), ptr(db2), ptr(inc.rowptr), ptr(inc.item), ptr(sp) if sp is not None else None, hp,
                    ptr(dpool), ptr(dh), B, N, P, D, 128, nat.LG_F_DROPOUT | nat.LG_F_NODE_MAJOR | lb, 0.1, ptr(ws),
                    ws.numel(), cs()), name)
                t = timeit(g, args.iters)
                res[name] = {"us": t, "TFLOPs": 2 * 2 * B * P * 3 * D * 128 / t / 1e6}
            if not only_stream:
                g = lambda: check(lib.lg_pipe_scatter_bwd(ptr(inc.rowptr), ptr(inc.item), ptr(dpipe), ptr(dpool),
                                                          ptr(dh), B, N, P, D, nat.LG_F_NODE_MAJOR, cs()), "pipe scatter")
                t = timeit(g, args.iters)
                res["pipe_scatter"] = {"us": t, "GBps": (B * P * 2 * D * 4 + B * N * D * 4) / t / 1e3}
    if "gru_fwd" in which or "gru_bwd" in which:
        S, L = 29, 36
        r = torch.randn(B, L, S, device=dev)
        tf = torch.randn(B, L, 9, device=dev)
        wih = torch.randn(192, 10, device=dev) / 4
        whh = torch.randn(192, 64, device=dev) / 8
        bih, bhh = torch.randn(192, device=dev) / 4, torch.randn(192, device=dev) / 4
        hs = torch.empty(L, B * S, 64, device=dev)
        gt = torch.empty(L, B * S, 4, 64, device=dev)
        hl = torch.empty(B * S, 64, device=dev)
        f = lambda: check(lib.lg_gru_fwd(ptr(r), ptr(tf), ptr(wih), ptr(whh), ptr(bih), ptr(bhh), ptr(hs), ptr(gt),
                                         ptr(hl), B, L, S, 10, 64, cs()), "gru fwd")
        t = timeit(f, args.iters)
        flops = 2 * B * S * L * 192 * (64 + 10)
        res["gru_fwd"] = {"us": t, "TFLOPs": flops / t / 1e6}
        f = lambda: check(lib.lg_gru_fwd(ptr(r), ptr(tf), ptr(wih), ptr(whh), ptr(bih), ptr(bhh), None, None,
                                         ptr(hl), B, L, S, 10, 64, cs()), "gru fwd eval")
        res["gru_fwd_eval"] = {"us": timeit(f, args.iters)}
        f = lambda: check(lib.lg_gru_fwd(ptr(r), ptr(tf), ptr(wih), ptr(whh), ptr(bih), ptr(bhh), ptr(hs), None,
                                         ptr(hl), B, L, S, 10, 64, cs()), "gru fwd hs only")
        res["gru_fwd_hs"] = {"us": timeit(f, args.iters)}
        if "gru_bwd" in which:
            dh = torch.randn(B * S, 64, device=dev)
            dws = [torch.empty_like(t) for t in (wih, whh, bih, bhh)]
            ws = torch.empty(int(lib.lg_gru_bwd_workspace_bytes(B, S, 10, 64)), device=dev, dtype=torch.uint8)
            f = lambda: check(lib.lg_gru_bwd(ptr(r), ptr(tf), ptr(wih), ptr(whh), ptr(hs), ptr(gt), ptr(dh), None,
                                             ptr(dws[0]), ptr(dws[1]), ptr(dws[2]), ptr(dws[3]), B, L, S, 10, 64,
                                             ptr(ws), ws.numel(), cs()), "gru bwd")
            t = timeit(f, args.iters)
            res["gru_bwd"] = {"us": t, "TFLOPs": 2 * flops / t / 1e6}
            if args.stamps and hasattr(lib, "lg_lab_gru_stamps"):
                res["stamps_gru_bwd"] = gru_stamps_summary(lib, f)
    if "tcn" in which:
        # frozen-predictor residual builder, B segments of l_pred + l_det = 72 steps
        from models import tcn_plan
        from models import utils as mutils
        from models.predictor import NormalPredictorTCN
        torch.manual_seed(0)
        m = NormalPredictorTCN(29, 9).eval().to(dev)
        seg, tseg = torch.randn(B, 72, 29, device=dev), torch.randn(B, 72, 9, device=dev)
        plan = tcn_plan.plan_for(36, 36)
        conv_flops = sum(cp.rows for cp in plan.convs) * B * 2 * 128 * 384
        with torch.no_grad():
            f = lambda: tcn_plan.tcn_residual(m, seg, tseg, 36, 36)
            t = timeit(f, args.iters)
            res["tcn_residual"] = {"us": t, "conv_TFLOPs": conv_flops / t / 1e6, "segments_per_s": B / t * 1e6}
            # one conv layer alone (the widest: rows 252)
            li = max(range(8), key=lambda i: plan.convs[i].rows)
            cp = plan.convs[li]
            rows_prev = plan.convs[li - 1].rows
            xin = torch.randn(B * rows_prev, 128, device=dev)
            blk_in = torch.randn(B * plan.convs[li - 2].rows, 128, device=dev) if li % 2 == 1 else None
            out = torch.empty(B * cp.rows, 128, device=dev)
            dp = tcn_plan._DevicePlan(plan, dev)
            packed = tcn_plan._packed_weights(m, dev)
            blk = m.tcn[li // 2]
            conv, norm = (blk.conv1.conv, blk.norm1) if li % 2 == 0 else (blk.conv2.conv, blk.norm2)
            f = lambda: check(lib.lg_tcn_conv_fwd(ptr(xin), ptr(blk_in), ptr(dp.tables[li]), ptr(packed[li]),
                                                  ptr(conv.bias), ptr(norm.weight), ptr(norm.bias), 1e-5, ptr(out), B,
                                                  rows_prev, plan.convs[li - 2].rows if li % 2 == 1 else 0, cp.rows,
                                                  128, cs()), "tcn conv")
            t = timeit(f, args.iters)
            res[f"tcn_conv_l{li}"] = {"us": t, "TFLOPs": B * cp.rows * 2 * 128 * 384 / t / 1e6}
            mutils.RESIDUAL_FAST_PATH = False
            f = lambda: mutils.build_residual_sequence_from_segment(m, seg, tseg, 36, 36)
            t = timeit(f, max(3, args.iters // 10))
            res["tcn_residual_stock"] = {"us": t, "segments_per_s": B / t * 1e6}
            mutils.RESIDUAL_FAST_PATH = True
    for k, v in res.items():
        print(k, json.dumps({a: round(b, 2) if isinstance(b, float) else b for a, b in v.items()}))


if __name__ == "__main__":
    main()
