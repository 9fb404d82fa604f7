"""The bench's captured training step, replayed K times (GPU child process of bench.py under
`rocprofv3 --kernel-trace`): the same model, batch and step graph as bench.py's headline leg,
so the trace holds every kernel of a replay — the named HIP kernels AND the small launches
(CE, slab reductions, Adam, the seed advance) — for bench.py's `step_kernels_us` /
`step_gap_us` (per-step accounting of ms_per_step).

  rocprofv3 --kernel-trace -d D -o trace --output-format csv -- python tools/step_trace.py [--B 256] [--steps 20]
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import bench
    from models.detector import LeakDetector
    from models.graph_step import CapturedTrainStep
    from models.optim import ClipAdamW
    dev = torch.device("cuda:0")
    pipes = bench.all_pipe_ids(bench.LTA_INP)
    torch.manual_seed(0)
    model = LeakDetector(bench.LTA_INP, bench.SENSORS, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2,
                         dropout=0.1, use_time=True).to(dev).train()
    opt = ClipAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    gen = torch.Generator().manual_seed(1234)
    B = args.B
    residual = torch.randn(B, 36, len(bench.SENSORS), generator=gen).to(dev)
    tfeat = bench.time_features(B, 36, gen).to(dev)
    label = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(dev)
    step = CapturedTrainStep(model, bench.CrossEntropyLoss(), opt, (residual, tfeat), label, clip=None, warmup=3)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
