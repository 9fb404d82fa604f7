"""torch.profiler op -> kernel map of one detector training step (GPU).  Diagnostic only.

  python tools/step_profile.py [--batch 256] > gpurun_out/step_profile.txt
"""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    from models.ddp import GradAllReduce
    from models.detector import LeakDetector
    dev = torch.device("cuda:0")
    pipes = bench.all_pipe_ids(bench.LTA_INP)
    torch.manual_seed(0)
    model = LeakDetector(bench.LTA_INP, bench.SENSORS, pipes).to(dev).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    allreduce = GradAllReduce(model.parameters())
    gen = torch.Generator().manual_seed(1)
    B = args.batch
    r = torch.randn(B, 36, 29, generator=gen).to(dev)
    tf = bench.time_features(B, 36, gen).to(dev)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(dev)

    def step():
        loss = torch.nn.functional.cross_entropy(model(r, tf), lab)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        allreduce()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=60,
                                                            max_name_column_width=60, max_shapes_column_width=60))


if __name__ == "__main__":
    main()
