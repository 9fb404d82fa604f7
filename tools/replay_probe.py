"""Where the time between captured-step replays goes (GPU).

The bench's captured training step (tools/step_trace.py's model and batch), timed K times
three ways, each bracketed by a device sync:
  torch   : CUDAGraph.replay() per step (what CapturedTrainStep does);
  lg1     : lg_graph_replay(exec, 1) per step (hipGraphLaunch of the same executable, no
            torch prologue);
  lgK     : lg_graph_replay(exec, K) in one call (host loop in C).
Also the host time of the K calls alone (no sync), i.e. whether the host keeps ahead of the
device.  Prints one JSON line.

  python tools/replay_probe.py [--B 256] [--steps 200]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import bench
    from models import _native as nat
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
    B, K = args.B, args.steps
    residual = torch.randn(B, 36, len(bench.SENSORS), generator=gen).to(dev)
    tfeat = bench.time_features(B, 36, gen).to(dev)
    label = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(dev)
    step = CapturedTrainStep(model, bench.CrossEntropyLoss(), opt, (residual, tfeat), label, clip=None, warmup=3)
    lib = nat.load_library()
    ex = step.graph_a.raw_cuda_graph_exec()
    st = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    out = {"B": B, "steps": K}

    def run(name, fn, n_calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_calls):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"ms_per_step": round((t2 - t0) * 1e3 / K, 4), "host_ms_per_step": round((t1 - t0) * 1e3 / K, 4)}

    for rep in range(2):
        run(f"torch{rep}", step, K)
        run(f"lg1_{rep}", lambda: nat.check(lib.lg_graph_replay(ex, 1, st), "lg_graph_replay"), K)
        run(f"lgK_{rep}", lambda: nat.check(lib.lg_graph_replay(ex, K, st), "lg_graph_replay"), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
