#!/usr/bin/env python3
"""Benchmark: LeakDetector training steps on batched L-TOWN-A windows (BASELINE.json
metric "windowed graphs/sec fwd+bwd on L-TOWN-A at 1/2/4/8 GPU; %HBM roofline").

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
  torchrun --nproc-per-node N ... bench.py --gpus N        (one rank per GPU, RCCL)

A step = one full detector training step over one batch of B windows per rank:
forward (GRU encoder, node init, 2x fused GCN layer, pipe gather, EdgeHead,
pool, NoLeakHead) + cross-entropy + backward + gradient all-reduce (N>1) +
clip_grad_norm_(1.0) + AdamW step — train mode, dropout 0.1, fp32.  Inputs are
synthetic residual windows of the reference shape (B, 36, 29) with time features,
resident in HBM before timing (the frozen-predictor residual build is a separate
model and is not part of the detector step).  Weak scaling: B windows per rank.

Roofline: the dominant HIP kernel is the fused GCN layer (lg_gcn_fwd, the
scatter-aggregate).  Its algorithmic bytes per launch follow SURVEY §8(d):
8*B*N*D + 4*(N+1) + 8*E'  (read x once, write y once, single-graph CSR), timed with
HIP events on the launch stream over the timed steps.  `traffic` is the measured HBM
traffic of one such launch: two child `rocprofv3 --pmc` passes (FETCH_SIZE, then
WRITE_SIZE; kernel trace only) over tools/kbench.py's identical train-mode launch,
corrected as MI355X_MICROARCH.md prescribes for gfx950 (2 x FETCH_SIZE + WRITE_SIZE,
KiB).  The plain propagate (lg_spmm, K6 alone) is timed beside it on the same graph.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "leak-det-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
LTA_INP = REPO / "leak-det-gnn_amd" / "data" / "L-TOWN-A.inp"
SENSORS = ['n54', 'n105', 'n114', 'n163', 'n188', 'n229', 'n288', 'n296', 'n332', 'n342', 'n410', 'n415', 'n429',
           'n458', 'n469', 'n495', 'n506', 'n516', 'n519', 'n549', 'n613', 'n636', 'n644', 'n679', 'n722', 'n726',
           'n740', 'n752', 'n769']  # reference configs/sim_LTA.yaml:21


def all_pipe_ids(inp: Path):
    from models.utils import parse_epanet_inp
    sec = parse_epanet_inp(inp)
    return sorted({ln.split()[0] for ln in sec["PIPES"]})  # dataset order: sorted pipe ids (datasets.py:353)


def sampled_pipe_ids(ratio: float, seed: int = 198):
    """The reference example's leak-set pipes (cmd.sh:10: --pipe_sample_ratio 0.5 --seed 198):
    leak_generation.py:90-99's pick over the .inp's pipe order, sorted (models/synth.pick_pipes)."""
    from models.synth import pick_pipes
    from models.utils import parse_epanet_inp
    return pick_pipes([ln.split()[0] for ln in parse_epanet_inp(LTA_INP)["PIPES"]], ratio, seed)


def time_features(B: int, L: int, gen: torch.Generator) -> torch.Tensor:
    """(B, L, 9): hour sin/cos + day-of-week one-hot at 5-min steps (datasets.py:49-59)."""
    start = torch.randint(0, 7 * 288, (B, 1), generator=gen)
    t = start + torch.arange(L).view(1, L)
    minutes = (t % 288) * 5
    ang = 2 * np.pi * (minutes.float() / 60.0) / 24.0
    dow = (t // 288) % 7
    return torch.cat([ang.sin().unsqueeze(-1), ang.cos().unsqueeze(-1),
                      torch.nn.functional.one_hot(dow, 7).float()], dim=-1)


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> dict:
    """The host cores this process may run on: os.cpu_count(), the affinity mask, and the
    cgroup CPU quota (cpu.max; on the GPU box the pod's share is far below the machine's
    core count, and threads past the quota only queue behind it).  `threads` = the affinity
    count, capped by the quota when one is set."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(np.ceil(quota))))
    return {"threads": threads, "cpu_count": total, "affinity": aff,
            "cgroup_quota_cpus": round(quota, 2) if quota is not None else None}


def cpu_baseline(batch: int, budget_s: float, threads: int) -> dict:
    """The oracle's CPU restatement of the same step timed on the host cores (reported only,
    BASELINE.md plan): eval-mode forward and train-mode fwd+CE+bwd, median of >= 10 timed
    steps after 3 warm-ups each (more while within the budget)."""
    from oracle.detector_ref import LeakDetectorRef
    torch.set_num_threads(threads)
    pipes = all_pipe_ids(LTA_INP)
    torch.manual_seed(0)
    m = LeakDetectorRef(LTA_INP, SENSORS, pipes)
    gen = torch.Generator().manual_seed(1234)
    r = torch.randn(batch, 36, 29, generator=gen)
    tf = time_features(batch, 36, gen)
    lab = torch.randint(0, len(pipes) + 1, (batch,), generator=gen)

    def train_step():
        m.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(r, tf), lab).backward()

    def eval_fwd():
        with torch.no_grad():
            m(r, tf)

    def timed(fn, mode):
        m.train(mode == "train")
        for _ in range(3):
            fn()
        ts = []
        t_end = time.perf_counter() + budget_s / 2
        while len(ts) < 10 or (time.perf_counter() < t_end and len(ts) < 30):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), len(ts)

    tr, ntr = timed(train_step, "train")
    ev, nev = timed(eval_fwd, "eval")
    share = cpu_share()
    return {"value": round(batch / tr, 2), "unit": "windows/s", "cores": threads, "kind": "port",
            "host_cpus": share,
            "cpu_model": cpu_model(), "eval_forward_windows_per_s": round(batch / ev, 2),
            "train_ms_per_step": round(tr * 1e3, 1), "eval_ms_per_step": round(ev * 1e3, 1),
            "sample": f"median of {ntr} train-mode fwd+CE+bwd steps (value) and {nev} eval-mode forwards, each "
                      f"after 3 warm-ups, B={batch} L-TOWN-A windows (oracle/detector_ref.py on torch CPU, "
                      f"{threads} threads, {cpu_model()})"}


def pmc_traffic(which: str, kname: str, batch: int) -> dict | None:
    """Per-launch HBM bytes of one kbench launch from rocprofv3 PMC counters.

    Runs as child processes (never exec): one counter per pass, kernel trace only.
    Returns None when rocprofv3 is unavailable or a pass fails.
    """
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            cmd = [prof, "--pmc", counter, "--kernel-trace", "-d", d, "-o", "pmc", "--output-format", "csv", "--",
                   sys.executable, str(REPO / "tools" / "kbench.py"), "--which", which, "--B", str(batch),
                   "--iters", "20", "--eager"]
            try:
                subprocess.run(cmd, env=env, cwd=str(REPO), timeout=300, check=True, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
            except (subprocess.SubprocessError, OSError):
                return None
            per = {}
            for f in Path(d).rglob("*counter_collection.csv"):
                for r in csv.DictReader(open(f)):
                    if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
                        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            if not per:
                return None
            vals[counter] = sum(per.values()) / len(per)
    return {"bytes": (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0, "FETCH_SIZE_KiB": vals["FETCH_SIZE"],
            "WRITE_SIZE_KiB": vals["WRITE_SIZE"]}


def short_kernel_name(name: str) -> str:
    """k_gcn_fwd_pc<64, true, ...>(...) -> k_gcn_fwd_pc; (anonymous namespace)::k_ce_fwd(...) -> k_ce_fwd"""
    n = name.replace("(anonymous namespace)::", "")  # also inside the argument list
    return n.split("<")[0].split("(")[0].strip().split(" ")[-1]


def small_kernels_us(breakdown: dict | None) -> dict:
    """kernels_us entries of the step's small launches, from the step trace (per step, us)."""
    if not breakdown:
        return {}
    by = breakdown["by_name_us"]
    pick = {"ce_fwd": ["k_ce_fwd", "k_ce_mean"], "ce_bwd": ["k_ce_bwd"], "adam": ["k_adam", "k_adam_norm", "k_adam_update"],
            "seed": ["k_seed_advance"], "slab_reduce": ["k_slab_reduce"], "sensor_proj_bwd": ["k_sensor_proj_bwd"]}
    # launches that a fused kernel absorbed (round 5) are absent from the trace: not reported
    return {k: round(sum(by.get(n, 0.0) for n in v), 2) for k, v in pick.items() if any(n in by for n in v)}


# step work that runs inside another kernel since round 5 (kernels_us has no entry for it)
FUSED_INTO = {"node_init": "k_gru_fwd (lg_gru_node_init_fwd epilogue + bits workgroups)",
              "sensor_proj_bwd": "k_gru_bwd2 (lg_gru_node_init_bwd prologue / epilogue)",
              "pool_head_bwd": "k_edge_bwd (lg_heads_bwd_scatter prologue)",
              "seed": "k_adam (lg_clip_adamw_seeds)"}


def step_breakdown(batch: int, ms_per_step: float, steps: int = 20) -> dict | None:
    """Every kernel of the captured step as it runs in the graph replays (tools/step_trace.py
    under a child `rocprofv3 --kernel-trace`).  The replays between two k_gru_fwd launches are
    one step each; the later half (steady state) is used:
      kernels          the median replay's kernels in launch order, with their durations;
      kernels_mean_us  per launch position (name#occurrence: k_gcn_fwd_pc#1 is the second
                       k_gcn_fwd_pc of the step, layer 1) the mean duration over the replays;
      sum_us / replay_span_us / step_gap_us
                       the median replay's kernel sum, its span (first kernel start to the next
                       replay's first kernel start) and span minus sum (the gaps between kernels,
                       including the one between replays);
      replay_gap_us    median over replays of the next replay's first kernel start minus this
                       replay's last kernel end: the device idles there while the host submits
                       the next graph launch;
      step_minus_kernels_us  ms_per_step (the bench's own, unprofiled clock) minus the sum."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        cmd = [prof, "--kernel-trace", "-d", d, "-o", "trace", "--output-format", "csv", "--", sys.executable,
               str(REPO / "tools" / "step_trace.py"), "--B", str(batch), "--steps", str(steps)]
        try:
            subprocess.run(cmd, env=env, cwd=str(REPO), timeout=300, check=True, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
        except (subprocess.SubprocessError, OSError):
            return None
        rows = []
        for f in Path(d).rglob("*kernel_trace.csv"):
            rows += list(csv.DictReader(open(f)))
    if not rows:
        return None
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_gru_fwd" in r["Kernel_Name"]]
    if len(marks) < 4:
        return None
    reps, gaps = [], []
    for a, b in zip(marks[len(marks) // 2:-1], marks[len(marks) // 2 + 1:]):  # the later half: steady state
        ks = [(short_kernel_name(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
              for r in rows[a:b]]
        span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
        gaps.append((int(rows[b]["Start_Timestamp"]) - int(rows[b - 1]["End_Timestamp"])) / 1e3)
        reps.append((sum(t for _, t in ks), span, ks))
    n0 = len(reps[0][2])
    same = [r for r in reps if len(r[2]) == n0]
    pos = []
    seen: dict = {}
    for n, _ in reps[0][2]:
        pos.append(f"{n}#{seen.get(n, 0)}")
        seen[n] = seen.get(n, 0) + 1
    mean_pos = {p: round(float(np.mean([r[2][i][1] for r in same])), 2) for i, p in enumerate(pos)}
    reps.sort(key=lambda x: x[0])
    tot, span, ks = reps[len(reps) // 2]
    agg: dict = {}
    for n, t in ks:
        agg[n] = round(agg.get(n, 0.0) + t, 2)
    return {"source": "rocprofv3 --kernel-trace over tools/step_trace.py (the same captured step), median replay",
            "kernels": [[n, round(t, 2)] for n, t in ks], "kernels_mean_us": mean_pos, "replays": len(same),
            "by_name_us": agg, "launches": len(ks),
            "sum_us": round(tot, 1), "replay_span_us": round(span, 1), "step_us": round(ms_per_step * 1e3, 1),
            "step_gap_us": round(span - tot, 1), "replay_gap_us": round(float(np.median(gaps)), 2),
            "step_minus_kernels_us": round(ms_per_step * 1e3 - tot, 1),
            "accounted_frac": round(tot / (ms_per_step * 1e3), 4)}


# kernels_us names -> launch position in the captured step (step_breakdown kernels_mean_us)
STEP_POSITIONS = {"gru_fwd": "k_gru_fwd#0", "node_init": "k_node_init_bits#0", "gcn_fwd_l0": "k_gcn_fwd_pc#0",
                  "gcn_fwd": "k_gcn_fwd_pc#1", "edge_fwd": "k_edge_fwd#0", "pool_head": "k_pool_head_fwd#0",
                  "pool_head_bwd": "k_pool_head_bwd#0", "edge_bwd": "k_edge_bwd#0", "gcn_bwd": "k_gcn_bwd_nm3#0",
                  "gcn_bwd_l0": "k_gcn_bwd_nm3#1", "linear_dw": "k_sensor_proj_bwd#0", "gru_bwd": "k_gru_bwd2#0"}


def in_step_kernels_us(breakdown: dict | None) -> dict:
    """kernels_us from the captured step's trace: each named kernel's mean in-graph duration
    (us) at its launch position, plus the small launches' per-step sums."""
    if not breakdown:
        return {}
    mp = breakdown["kernels_mean_us"]
    out = {k: mp[v] for k, v in STEP_POSITIONS.items() if v in mp}
    out.update(small_kernels_us(breakdown))
    return out


def stream_copy_peak(dev, nbytes: int = 2 << 30, iters: int = 10) -> dict:
    """Measured copy bandwidth on this box: device copy of an nbytes fp32 buffer (past the
    256 MiB Infinity Cache), read + write bytes over HIP-event time."""
    x = torch.ones(nbytes // 4, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        y.copy_(x)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / iters
    # the library's non-temporal b128 copy kernel over the same buffers (lg_stream_copy)
    from models import _native as nat
    from models.ops import check, ptr, stream_of
    lib = nat.load_library()
    st = stream_of(x)
    for _ in range(3):
        check(lib.lg_stream_copy(ptr(x), ptr(y), nbytes, st), "lg_stream_copy")
    a.record()
    for _ in range(iters):
        check(lib.lg_stream_copy(ptr(x), ptr(y), nbytes, st), "lg_stream_copy")
    b.record()
    torch.cuda.synchronize()
    ms_hip = a.elapsed_time(b) / iters
    del x, y
    torch.cuda.empty_cache()
    torch_gbps, hip_gbps = 2 * nbytes / (ms * 1e-3) / 1e9, 2 * nbytes / (ms_hip * 1e-3) / 1e9
    return {"GBps": round(max(torch_gbps, hip_gbps), 1), "torch_copy_GBps": round(torch_gbps, 1),
            "hip_copy_GBps": round(hip_gbps, 1), "bytes_moved": 2 * nbytes,
            "method": f"the faster of torch copy_ and lg_stream_copy (non-temporal b128) of a {nbytes >> 20} MiB "
                      f"fp32 buffer (read + write), HIP events, mean of {iters}"}


def time_propagate(graph, B: int, N: int, D: int, dev, iters: int = 50) -> float:
    """Mean device time (ms) of lg_spmm (K6 alone) on [B, N, D], HIP events on the launch stream."""
    from models import _native as nat
    from models.ops import check, ptr
    lib = nat.load_library()
    x = torch.randn(B, N, D, device=dev)
    y = torch.empty_like(x)
    st = torch.cuda.current_stream(dev)

    def f():
        check(lib.lg_spmm(ptr(graph.rowptr), ptr(graph.col), ptr(graph.w), ptr(x), ptr(y), B, N, D, graph.nnz_cap,
                          st.cuda_stream), "lg_spmm")
    for _ in range(5):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(iters):
        f()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 dense fp32
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 (v_mfma_f32_16x16x32_bf16)


def gru_mfma_report(kms: dict, B: int, S: int, L: int = 36, H: int = 64) -> dict:
    """The GRU kernels' MFMA pipe share: the recurrent products (and the whole backward) run
    on bf16 MFMA with 3-way split operands (six products per fp32 product), the forward's x
    part (K = 12 padded) on fp32 MFMA.  `mfma_busy_est` = sum over instruction kinds of
    issued FLOP / that kind's dense peak, divided by the kernel time: the share of the
    chip's MFMA pipe time the kernel's MFMAs occupy (1.0 = MFMA-bound)."""
    ns = B * S * L
    work = {"gru_fwd": (6 * 2 * ns * 3 * H * H, 2 * ns * 3 * H * 12),
            "gru_bwd": (6 * 2 * ns * 3 * H * (H + H + 16), 0)}
    eq = {"gru_fwd": 2 * ns * 3 * H * (H + 10), "gru_bwd": 2 * 2 * ns * 3 * H * (H + 10)}
    out = {}
    for k, (bf, f32) in work.items():
        t = kms.get(k)
        if not t:
            continue
        sec = t * 1e-3
        out[k] = {"fp32_equiv_tflops": round(eq[k] / sec / 1e12, 2),
                  "mfma_busy_est": round((bf / (BF16_MFMA_PEAK_TFLOPS * 1e12) + f32 / (FP32_MFMA_PEAK_TFLOPS * 1e12)) / sec, 4),
                  "us": round(t * 1e3, 2)}
    return out


class ResidualDetector(torch.nn.Module):
    """The reference's training forward from raw segments (train_detector.py:302-310):
    residual build with the frozen predictor under no_grad, then the detector."""

    def __init__(self, predictor, detector, l_pred: int = 36, l_det: int = 36):
        super().__init__()
        self.predictor, self.detector, self.l_pred, self.l_det = predictor, detector, l_pred, l_det

    def forward(self, seg, tseg):
        from models import utils as mutils
        with torch.no_grad():
            residual = mutils.build_residual_sequence_from_segment(self.predictor, seg, tseg, self.l_pred,
                                                                   self.l_det, device=seg.device)
        return self.detector(residual, tseg[:, self.l_pred:, :])


def e2e_training(model, opt, label, B: int, steps: int, dev) -> dict:
    """Detector training steps INCLUDING the frozen-predictor residual build from raw
    (B, 72, 29) segments (train_detector.py:296-317 loop order; SURVEY §8 d: reported
    separately from graphs/s), the whole step replayed as one HIP graph like the headline
    step.  Residual build = the HIP shared-window TCN path; the stock per-window module
    path (what the reference runs) is timed beside it."""
    from models import tcn_plan
    from models import utils as mutils
    from models.graph_step import CapturedTrainStep
    from models.predictor import NormalPredictorTCN
    torch.manual_seed(7)
    predictor = NormalPredictorTCN(len(SENSORS), 9).to(dev).eval()
    for p in predictor.parameters():
        p.requires_grad_(False)
    gen = torch.Generator().manual_seed(4321)
    seg = torch.randn(B, 72, len(SENSORS), generator=gen).to(dev)
    tseg = time_features(B, 72, gen).to(dev)
    e2e = ResidualDetector(predictor, model).to(dev)
    step = CapturedTrainStep(e2e, CrossEntropyLoss(), opt, (seg, tseg), label, clip=None, warmup=3)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    e2e_s = (time.perf_counter() - t0) / steps
    with torch.no_grad():
        fast_ms = _event_ms(lambda: tcn_plan.tcn_residual(predictor, seg, tseg, 36, 36), 20)
        mutils.RESIDUAL_FAST_PATH = False
        try:
            stock_ms = _event_ms(lambda: mutils.build_residual_sequence_from_segment(predictor, seg, tseg, 36, 36), 3)
        finally:
            mutils.RESIDUAL_FAST_PATH = True
    plan = tcn_plan.plan_for(36, 36)
    conv_flop = sum(cp.rows for cp in plan.convs) * B * 2 * 128 * 384
    conv_ms = _conv_ms(predictor, plan, B, dev)
    conv_tf = conv_flop / (conv_ms * 1e-3) / 1e12
    return {"value": round(B / e2e_s, 2), "unit": "windows/s", "ms_per_step": round(e2e_s * 1e3, 4),
            "step": "residual build (frozen TCN, 36 windows of 36 steps per segment) + detector fwd+CE+bwd+AdamW, "
                    "one HIP-graph replay per step",
            "residual_ms": round(fast_ms, 4), "residual_ms_stock_module": round(stock_ms, 4),
            "residual_speedup": round(stock_ms / fast_ms, 2),
            "tcn_conv": {"kernel": "lg_tcn_conv_fwd x8 (shared-window rows)", "bound": "mfma",
                         "achieved": round(conv_tf, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(conv_tf / FP32_MFMA_PEAK_TFLOPS, 4), "flop_per_call": conv_flop,
                         "ms_per_call": round(conv_ms, 4)}}


def c4_leg(dev, steps: int, warmup: int, rank: int, world: int) -> dict:
    """BASELINE configs[3]: the detector training step on the synthetic 10k-node / 15k-pipe
    network (30k edge columns, written as an EPANET .inp), node_hidden = sensor_hidden = 32,
    64 windows per rank (global 512 at 8 GPUs), one HIP-graph replay per step, weak scaling.
    Returns windows/s over all ranks (max time over ranks) and the C4 GCN forward roofline."""
    from models import ops
    from models.detector import LeakDetector
    from models.graph_step import CapturedTrainStep
    from models.synth import pick_sensors, write_synthetic_inp
    N, P, D, B = 10_000, 15_000, 32, 64
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        inp = Path(d) / "c4.inp"
        node_ids, pipe_ids = write_synthetic_inp(inp, N, P, seed=0)
        sensors = pick_sensors(node_ids, 29, seed=0)
        torch.manual_seed(0)
        m = LeakDetector(inp, sensors, pipe_ids, sensor_hidden=D, node_hidden=D).to(dev).train()
    from models.optim import ClipAdamW
    opt = ClipAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)  # clip_grad_norm_(1.0) + AdamW
    gen = torch.Generator().manual_seed(99 + rank)
    r = torch.randn(B, 36, 29, generator=gen).to(dev)
    tf = time_features(B, 36, gen).to(dev)
    lab = torch.randint(0, P + 1, (B,), generator=gen).to(dev)
    step = CapturedTrainStep(m, CrossEntropyLoss(), opt, (r, tf), lab, clip=None, warmup=3)
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    timer = ops.KernelTimer(["gcn_fwd"])
    ops.set_kernel_timer(timer)
    timer.enabled = True
    for _ in range(5):
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(r, tf), lab).backward()
    timer.enabled = False
    ops.set_kernel_timer(None)
    fwd_ms = timer.mean_ms("gcn_fwd")
    E1 = int(m.edge_index_single.shape[1]) + N
    byts = 8 * B * N * D + 4 * (N + 1) + 8 * E1
    gbs = byts / (fwd_ms * 1e-3) / 1e9
    return {"metric": "windowed graphs/sec fwd+bwd, synthetic 10k nodes / 30k edge columns (BASELINE configs[3])",
            "value": round(B * world * steps / el, 2), "unit": "windows/s", "ms_per_step": round(el * 1e3 / steps, 4),
            "windows_per_rank": B, "global_batch": B * world, "feat": D, "pipes": P, "scaling": "weak",
            "roofline_gcn_fwd": {"kernel": "lg_gcn_fwd_nm (train mode)", "bound": "hbm",
                                 "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": byts,
                                 "avg_launch_us": round(fwd_ms * 1e3, 2)}}


def c5_leg(dev, iters: int = 20) -> dict:
    """BASELINE configs[4], "the HBM-roofline stress of scatter-aggregate": ONE synthetic pipe
    graph of 100,000 nodes / 300,000 edge columns (150,000 pipes, models/synth.py, seed 0),
    D = 64, B = 1: GCNConv(64, 64) forward and backward through the product's module (its
    D = 64 path: the node-table row tiles lg_gcn_fwd_rows / lg_gcn_bwd_rows), x ~ N(0, 1) seed 0.  Roofline bytes per forward
    call from SURVEY §8(d): 8 B N D + 4 (N + 1) + 8 E' = 54.8 MB (E' = E + N); backward:
    read dy (gathered) and x, write dx: 12 B N D + CSR bytes.  HIP events on the launch
    stream (the library's kernel timer), mean over `iters` calls after warm-up."""
    from models import ops
    from models.gcn import GCNConv
    from models.synth import synthetic_pipe_graph
    N, P, D = 100_000, 150_000, 64
    ei, _ = synthetic_pipe_graph(N, P, seed=0)
    torch.manual_seed(0)
    conv = GCNConv(D, D).to(dev)
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(N, D, generator=gen).to(dev).requires_grad_(True)
    dy = torch.randn(N, D, generator=gen).to(dev)
    eid = ei.to(dev)
    for _ in range(3):
        conv(x, eid).backward(dy)
    torch.cuda.synchronize()
    timer = ops.KernelTimer(["gcn_fwd", "gcn_bwd"])
    ops.set_kernel_timer(timer)
    timer.enabled = True
    for _ in range(iters):
        x.grad = None
        conv(x, eid).backward(dy)
    torch.cuda.synchronize()
    timer.enabled = False
    ops.set_kernel_timer(None)
    fwd_ms, bwd_ms = timer.mean_ms("gcn_fwd"), timer.mean_ms("gcn_bwd")
    E1 = int(ei.shape[1]) + N
    csr = 4 * (N + 1) + 8 * E1
    fwd_bytes, bwd_bytes = 8 * N * D + csr, 12 * N * D + csr
    fg, bg = fwd_bytes / (fwd_ms * 1e-3) / 1e9, bwd_bytes / (bwd_ms * 1e-3) / 1e9
    return {"metric": "GCNConv fwd / bwd on one synthetic 100k-node / 300k-edge-column graph (BASELINE configs[4])",
            "nodes": N, "edge_columns": int(ei.shape[1]), "feat": D, "windows": 1, "scaling": "replicas only",
            "path": "models.gcn.GCNConv (lg_gcn_fwd_rows / lg_gcn_bwd_rows: 16-node tiles off the node table)",
            "roofline": {"kernel": "lg_gcn_fwd_rows -> k_gcn_fwd_rows (K5+K6+K7 fused)", "bound": "hbm",
                         "achieved": round(fg, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fg / HBM_PEAK_GBS, 4),
                         "bytes_per_launch": fwd_bytes, "avg_launch_us": round(fwd_ms * 1e3, 2)},
            "roofline_bwd": {"kernel": "lg_gcn_bwd_rows -> k_gcn_bwd_rows (dx, dW, db)", "bound": "hbm",
                             "achieved": round(bg, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bg / HBM_PEAK_GBS, 4),
                             "bytes_per_launch": bwd_bytes, "avg_launch_us": round(bwd_ms * 1e3, 2)}}


def CrossEntropyLoss():
    """nn.CrossEntropyLoss() on the fused HIP op (models/loss.py; same defaults)."""
    from models.loss import CrossEntropyLoss as _CE
    return _CE()


def tier_leg(dev, steps: int, warmup: int, rank: int, world: int, mlp_dtype: str, batch: int,
             pipe_ratio: float = 1.0) -> dict:
    """BASELINE configs[2] as written — "bf16 node-MLP on MFMA" (SURVEY §8 d C3: bf16 for the
    K5 GCN transforms and the K9 EdgeHead MLP, fp32 accumulate): the same L-TOWN-A training
    step with LeakDetector(mlp_dtype=...), captured, timed like the main line; plus the
    in-step durations of the kernels whose products change.  pipe_ratio 0.5: the same step
    with the reference example's leak set (cmd.sh:10 --pipe_sample_ratio 0.5: P = 382 of the
    764 pipes, models/synth.pick_pipes), SURVEY §8(d) C3's "also report P=382"."""
    from models import ops
    from models.detector import LeakDetector
    from models.graph_step import CapturedTrainStep
    pipes = all_pipe_ids(LTA_INP) if pipe_ratio >= 1.0 else sampled_pipe_ids(pipe_ratio)
    P, B = len(pipes), batch
    torch.manual_seed(0)
    m = LeakDetector(LTA_INP, SENSORS, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1,
                     use_time=True, mlp_dtype=mlp_dtype).to(dev).train()
    from models.optim import ClipAdamW
    opt = ClipAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)  # clip_grad_norm_(1.0) + AdamW
    gen = torch.Generator().manual_seed(1234 + rank)
    r = torch.randn(B, 36, len(SENSORS), generator=gen).to(dev)
    tf = time_features(B, 36, gen).to(dev)
    lab = torch.randint(0, P + 1, (B,), generator=gen).to(dev)
    step = CapturedTrainStep(m, CrossEntropyLoss(), opt, (r, tf), lab, clip=None, warmup=3)
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    names = ["gcn_fwd", "gcn_bwd", "gcn_bwd_l0", "edge_fwd", "edge_bwd"]
    timer = ops.KernelTimer(names)
    ops.set_kernel_timer(timer)
    timer.enabled = True
    for _ in range(5):
        opt.zero_grad(set_to_none=True)
        torch.nn.functional.cross_entropy(m(r, tf), lab).backward()
    timer.enabled = False
    ops.set_kernel_timer(None)
    kms = {k: timer.mean_ms(k) for k in names}
    what = ("bf16 node-MLP on MFMA" if mlp_dtype == "bf16" else "fp32 node-MLP") + (f", P = {P}" if pipe_ratio < 1 else "")
    return {"metric": f"windowed graphs/sec fwd+bwd on L-TOWN-A (BASELINE configs[2]: {what})",
            "value": round(B * world * steps / el, 2), "unit": "windows/s", "ms_per_step": round(el * 1e3 / steps, 4),
            "mlp_dtype": mlp_dtype, "windows_per_rank": B, "scaling": "weak", "pipes": P,
            "parity": "logits within 2e-2 of the fp32 oracle (tests/test_gpu_configs.py::test_bf16_tier_b256)"
            if mlp_dtype == "bf16" else "fp32 bars",
            "kernels_us_eager": {k: round(v * 1e3, 2) for k, v in kms.items() if v is not None}}


def _event_ms(fn, iters: int) -> float:
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def _conv_ms(predictor, plan, B: int, dev) -> float:
    """Summed HIP-event time of the 8 conv launches of one residual build."""
    from models import _native as nat
    from models import tcn_plan
    lib = nat.load_library()
    dp = tcn_plan._DevicePlan(plan, dev)
    packed = tcn_plan._packed_weights(predictor, dev)
    bufs = [(torch.randn(B * plan.seg_len, 128, device=dev), plan.seg_len)]
    for cp in plan.convs:
        bufs.append((torch.empty(B * cp.rows, 128, device=dev), cp.rows))
    st = torch.cuda.current_stream(dev).cuda_stream

    def run():
        for li, cp in enumerate(plan.convs):
            blk = predictor.tcn[li // 2]
            conv, norm = (blk.conv1.conv, blk.norm1) if li % 2 == 0 else (blk.conv2.conv, blk.norm2)
            prev, rp = bufs[li]
            bi, rb = bufs[li - 1] if li % 2 == 1 else (None, 0)
            nat.check(lib.lg_tcn_conv_fwd(nat.ptr(prev), nat.ptr(bi), nat.ptr(dp.tables[li]), nat.ptr(packed[li]),
                                          nat.ptr(conv.bias), nat.ptr(norm.weight), nat.ptr(norm.bias), 1e-5,
                                          nat.ptr(bufs[li + 1][0]), B, rp, rb, cp.rows, 128, st), "lg_tcn_conv_fwd")
    return _event_ms(run, 20)


def _free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`--gpus N` without torchrun's environment: start N ranks (one process per GPU)
    under torch.distributed.run as a CHILD process, before this process touches the GPU,
    and return its exit code.  Rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve())] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _timed_max(fn, steps: int, sync, world: int) -> float:
    """Seconds of `steps` calls of fn between barrier + sync fences, max over ranks."""
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def exchange_fields(t_full: float, t_nocomm: float, t_ar: float, steps: int, world: int, how: str) -> dict:
    """The multi-rank step's exchange cost.  allreduce_us: the gradient all-reduce alone, per
    step; exchange_exposed_us: what the exchange adds to the step (with it minus without,
    the rest identical); weak_scaling_eff: the step without the exchange over the step with
    it — per-rank throughput at this world size relative to the same step with nothing to
    wait for (the driver computes the cross-run efficiency from its own N=1 line)."""
    if world == 1:
        return {"allreduce_us": 0.0, "exchange_exposed_us": 0.0, "weak_scaling_eff": 1.0, "exchange": how}
    return {"allreduce_us": round(t_ar * 1e6 / steps, 2),
            "exchange_exposed_us": round(max(0.0, t_full - t_nocomm) * 1e6 / steps, 2),
            "weak_scaling_eff": round(min(1.0, t_nocomm / t_full), 4), "exchange": how}


def dry_run(args, rank: int, world: int) -> None:
    """`--dry-run`: the multi-rank launch / barrier / max-over-ranks timing / JSON path on
    CPU (gloo), with the step reduced to the detector's gradient all-reduce (60,418 fp32
    values in one bucket).  For CI without a GPU; never a measurement."""
    import torch.distributed as dist
    from models.ddp import init_distributed
    init_distributed(backend="gloo")
    grad = torch.ones(60418) * (rank + 1)
    a = torch.randn(192, 192)

    def compute():  # stand-in for the detector step (a fixed CPU workload)
        for _ in range(4):
            a.matmul(a)

    def full():
        compute()
        dist.all_reduce(grad)

    for _ in range(args.warmup):
        full()
    nosync = lambda: None  # noqa: E731
    t_full = _timed_max(full, args.steps, nosync, world)
    t_nocomm = _timed_max(compute, args.steps, nosync, world)
    t_ar = _timed_max(lambda: dist.all_reduce(grad), args.steps, nosync, world)
    if rank == 0:
        out = {"metric": "windowed graphs/sec fwd+bwd on L-TOWN-A", "value": None, "unit": "windows/s",
               "n_gpus": world, "ranks_seen": dist.get_world_size(), "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(t_full * 1e3 / max(args.steps, 1), 4),
               "dry_run": True, "backend": "gloo",
               "config": {"workload": "gradient all-reduce (60,418 fp32) after a fixed CPU matmul stand-in step",
                          "parallelism": f"dp{world}"}}
        out.update(exchange_fields(t_full, t_nocomm, t_ar, max(args.steps, 1), world, "one bucket, blocking (gloo)"))
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="windows per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=24.0, help="seconds of CPU-baseline sampling")
    ap.add_argument("--no-c4", action="store_true", help="skip the configs[3] (C4) leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the configs[4] (C5) leg")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--eager", action="store_true", help="launch the step eagerly instead of replaying its HIP graph")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo launch-path check (no GPU, no measurement)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="node-MLP tier of the main line: fp32 (split-bf16 MFMA, fp32 parity) or bf16 (configs[2])")
    ap.add_argument("--no-tier-leg", action="store_true", help="skip the leg of the other node-MLP tier")
    ap.add_argument("--no-p382", action="store_true", help="skip the P = 382 leg (cmd.sh:10's pipe_sample_ratio 0.5)")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world_env = int(env_world or 1)
    if world_env != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; launch one rank per GPU")
    if args.dry_run:
        from models.ddp import dist_env
        rank, _, world = dist_env()
        dry_run(args, rank, world)
        return
    if torch.cuda.device_count() < args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} GPU(s) visible")

    from models import ops
    from models.ddp import GradAllReduce, init_distributed, reseed_rank
    from models.detector import LeakDetector

    rank, local_rank, world = init_distributed()
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    pipes = all_pipe_ids(LTA_INP)
    P, B = len(pipes), args.batch

    torch.manual_seed(0)
    model = LeakDetector(LTA_INP, SENSORS, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1,
                         use_time=True, mlp_dtype=args.dtype).to(dev).train()
    # clip_grad_norm_(1.0) + AdamW(lr 1e-3, wd 1e-4) as ONE launch (models/optim.py: the same
    # arithmetic as the reference's pair, device-side step counter so it lives in the step graph)
    from models.optim import ClipAdamW
    opt = ClipAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    allreduce = GradAllReduce(model.parameters())
    reseed_rank(0, rank, world)  # same weights on every rank, per-rank dropout seeds from here on
    N = len(model.node_names)
    E1 = int(model.edge_index_single.shape[1]) + N  # E' = E + N self loops

    gen = torch.Generator().manual_seed(1234 + rank)
    residual = torch.randn(B, 36, len(SENSORS), generator=gen).to(dev)
    tfeat = time_features(B, 36, gen).to(dev)
    label = torch.randint(0, P + 1, (B,), generator=gen).to(dev)
    loss_fn = CrossEntropyLoss()

    def step():
        logits = model(residual, tfeat)
        loss = loss_fn(logits, label)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        allreduce()
        opt.step()  # clip_grad_norm_(1.0) + AdamW
        return loss

    eager_step = step
    if not args.eager:
        # the whole step as ONE replayed HIP graph (models/graph_step.py; dropout re-drawn per replay;
        # the capture runs its own 3 eager steps first)
        from models.graph_step import CapturedTrainStep
        step = CapturedTrainStep(model, loss_fn, opt, (residual, tfeat), label, clip=None, warmup=3)
    # the W untimed warm-up steps are steps of the timed kind: graph replays.  (Until round 5 they
    # were eager steps before the capture, so the timed region began with the graph's first
    # replays, whose one-time device-side cost, ~0.3 ms, the driver's K = 20 amortised over
    # fewer steps than the builder's K = 50: VERDICT r05 weak 8.)
    for _ in range(args.warmup):
        step()
    timer = ops.KernelTimer(["gcn_fwd", "gcn_fwd_l0", "gcn_bwd", "gcn_bwd_l0", "node_init", "gru_fwd", "gru_bwd",
                             "edge_fwd", "edge_bwd", "pipe_scatter", "pool_head", "pool_head_bwd", "linear_dw"])
    ops.set_kernel_timer(timer)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # pass 1: wall clock of exactly K steps (no event instrumentation inside)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    # the exchange's cost: the same captured step with the collectives skipped, and the
    # gradient all-reduce alone (two buckets as the step issues them, or one eagerly)
    if world > 1:
        cuda_sync = torch.cuda.synchronize
        if hasattr(step, "comm"):
            step.comm = False
            t_nocomm = _timed_max(step, args.steps, cuda_sync, world)
            step.comm = True
            bucks = [b for b, _ in step.buckets]
            how = ("head bucket async under the trunk backward, trunk bucket blocking"
                   if len(bucks) == 2 else "one bucket, blocking")
        else:
            t_nocomm, bucks, how = elapsed, [allreduce.flat], "one bucket, blocking (eager)"
        t_ar = _timed_max(lambda: [dist.all_reduce(b) for b in bucks], args.steps, cuda_sync, world)
        xchg = exchange_fields(elapsed, t_nocomm, t_ar, args.steps, world, how)
    else:
        xchg = exchange_fields(elapsed, elapsed, 0.0, args.steps, 1, "none (one rank)")
    # pass 2: per-kernel HIP-event durations over the same number of steps (eager launches:
    # the events bracket each library call on its stream)
    timer.enabled = True
    for _ in range(args.steps):
        eager_step()
    barrier()
    timer.enabled = False
    ops.set_kernel_timer(None)
    kms = {k: timer.mean_ms(k) for k in timer.names}
    # BASELINE configs[3] (C4) at every world size: 64 windows per rank, weak scaling
    c4 = None if args.no_c4 else c4_leg(dev, max(10, args.steps // 2), 3, rank, world)
    c5 = None if (args.no_c5 or rank != 0) else c5_leg(dev)  # replicas only: rank 0 reports it
    other = "bf16" if args.dtype == "fp32" else "fp32"
    tier = None if args.no_tier_leg else tier_leg(dev, args.steps, 3, rank, world, other, B)

    if rank != 0:
        dist.destroy_process_group()
        return

    ms_per_step = elapsed * 1e3 / args.steps
    value = B * world * args.steps / elapsed
    D = 64
    csr_bytes = 4 * (N + 1) + 8 * E1
    fwd_bytes = 8 * B * N * D + csr_bytes           # read x once, write y once
    # layer-L-1 backward: read dy, x and the forward's [y > 0] bits (B*N*D/8 bytes); write dx
    bwd_bytes = 12 * B * N * D + N * ((B + 15) // 16) * 128 + csr_bytes
    pmc = world == 1 and not args.no_pmc
    # the kernels as they run in the timed (captured) step: rocprofv3 kernel trace of the same
    # step graph's replays; the eager pass-2 event timings are reported beside as *_eager
    breakdown = step_breakdown(B, elapsed * 1e3 / args.steps) if (pmc and not args.eager) else None
    kin = in_step_kernels_us(breakdown)
    timing = "in-graph (captured step replays, rocprofv3 kernel trace: step_kernels)" if kin else \
        "eager launches, HIP event pairs (pass 2)"
    fwd_ms = kin["gcn_fwd"] * 1e-3 if "gcn_fwd" in kin else kms["gcn_fwd"]
    bwd_ms = kin["gcn_bwd"] * 1e-3 if "gcn_bwd" in kin else kms["gcn_bwd"]
    achieved = fwd_bytes / (fwd_ms * 1e-3) / 1e9
    bwd_gbs = bwd_bytes / (bwd_ms * 1e-3) / 1e9
    graph = model._device_state(dev)[0]
    prop_ms = time_propagate(graph, B, N, D, dev)
    prop_gbs = fwd_bytes / (prop_ms * 1e-3) / 1e9
    copy = stream_copy_peak(dev)
    traffic = pmc_traffic("gcn_fwd_nm_train", "k_gcn_fwd_pc", B) if pmc else None
    traffic_bwd = pmc_traffic("gcn_bwd_nm", "k_gcn_bwd_nm", B) if pmc else None
    gru_rep = gru_mfma_report({k: (kin[k] * 1e-3 if k in kin else kms.get(k)) for k in ("gru_fwd", "gru_bwd")},
                              B, len(SENSORS))
    p382 = None if (args.no_p382 or args.batch != 256) else tier_leg(dev, args.steps, 3, rank, world, args.dtype, B,
                                                                     pipe_ratio=0.5)
    src = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the same launch, 2*FETCH+WRITE (gfx950)"
    out = {
        "metric": "windowed graphs/sec fwd+bwd on L-TOWN-A", "value": round(value, 2), "unit": "windows/s",
        "n_gpus": world, "ranks_seen": dist.get_world_size() if world > 1 else 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic residual windows (B,36,29) + time features, random-init weights",
        "config": {"workload": "L-TOWN-A detector training step (BASELINE configs[2])", "graph": "L-TOWN-A",
                   "nodes": N, "edge_columns": E1 - N, "pipes": P, "windows_per_rank": B,
                   "global_batch": B * world, "feat": D, "gnn_layers": 2, "parallelism": f"dp{world}",
                   "step": "fwd+CE+bwd+allreduce+clip+AdamW, train mode (clip_grad_norm_ + AdamW in one launch, "
                           "models/optim.py)",
                   "launch": "eager" if args.eager else "hipgraph (one replay per step, dropout re-drawn on device)"},
        "roofline": {"kernel": "lg_gcn_fwd_nm_bits -> k_gcn_fwd_pc, layer 1 (fused gather-aggregate by producer "
                               "waves, fp16x2 MFMA transform + bias/ReLU/dropout by consumer waves, train mode; layer 0 "
                               "reads the compressed node init: kernels_us.gcn_fwd_l0)", "bound": "hbm",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": round(traffic["bytes"]) if traffic else None,
                     "traffic_source": src if traffic else None,
                     "bytes_per_launch": fwd_bytes, "avg_launch_us": round(fwd_ms * 1e3, 2), "timing": timing,
                     "avg_launch_us_eager": round(kms["gcn_fwd"] * 1e3, 2),
                     "frac_of_measured_copy": round(achieved / copy["GBps"], 4)},
        "roofline_bwd": {"kernel": "lg_gcn_bwd_nm_bits (layer 2: gather of dy * [y > 0] over the transposed CSR, "
                                   "[y > 0] from the forward's mask bits; dx = t W, dW, db, masked by [x > 0])",
                         "bound": "hbm",
                         "achieved": round(bwd_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(bwd_gbs / HBM_PEAK_GBS, 4),
                         "traffic": round(traffic_bwd["bytes"]) if traffic_bwd else None,
                         "traffic_source": src if traffic_bwd else None,
                         "bytes_per_launch": bwd_bytes, "avg_launch_us": round(bwd_ms * 1e3, 2), "timing": timing,
                         "avg_launch_us_eager": round(kms["gcn_bwd"] * 1e3, 2)},
        "roofline_propagate": {"kernel": "lg_spmm (K6 alone, same graph and shape)", "bound": "hbm",
                               "achieved": round(prop_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(prop_gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(prop_ms * 1e3, 2)},
        "stream_copy": copy,
        **xchg,
        "gru_mfma": gru_rep,
        "kernels_us": kin or None,
        "kernels_us_eager": {k: round(v * 1e3, 2) for k, v in kms.items() if v is not None},
        "kernels_fused": FUSED_INTO,
        "step_gap_us": breakdown["step_gap_us"] if breakdown else None,
        "replay_gap_us": breakdown["replay_gap_us"] if breakdown else None,
        "step_kernels": breakdown,
        "final_loss": round(final_loss, 4),
    }
    if c4 is not None:
        out["c4"] = c4
    if c5 is not None:
        if pmc:
            tr = pmc_traffic("c5_fwd", "k_gcn_fwd_rows", 1)
            out_c5 = c5["roofline"]
            out_c5["traffic"] = round(tr["bytes"]) if tr else None
            out_c5["traffic_source"] = src if tr else None
        out["c5"] = c5
    if tier is not None:
        out["mlp_tier"] = tier
    if p382 is not None:
        out["p382"] = p382
    if world == 1:
        out["e2e_training"] = e2e_training(model, opt, label, B, max(5, args.steps // 2), dev)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(B, args.cpu_budget, threads=cpu_share()["threads"])
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
