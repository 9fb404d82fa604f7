"""Which host op launches each torch (non-libleakgnn) kernel of the detector training step:
torch.profiler over a few eager steps, kernels grouped by the innermost aten op around them."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]
import torch
from torch.profiler import ProfilerActivity, profile

import bench
from models.detector import LeakDetector
from models.optim import ClipAdamW

dev = torch.device("cuda", 0)
pipes = bench.all_pipe_ids(bench.LTA_INP)
torch.manual_seed(0)
m = LeakDetector(bench.LTA_INP, bench.SENSORS, pipes, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1,
                 use_time=True).to(dev).train()
opt = ClipAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
gen = torch.Generator().manual_seed(1)
B = 256
r = torch.randn(B, 36, 29, generator=gen).to(dev)
tf = bench.time_features(B, 36, gen).to(dev)
lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(dev)
loss_fn = bench.CrossEntropyLoss()
one = torch.ones((), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss = loss_fn(m(r, tf), lab)
    loss.backward(one)
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()
import json
import tempfile
path = tempfile.mktemp(suffix=".json")
prof.export_chrome_trace(path)
tr = json.load(open(path))["traceEvents"]
ops = {}
for e in tr:
    if e.get("cat") == "cpu_op" and "External id" in e.get("args", {}):
        ops.setdefault(e["args"]["External id"], []).append(e)
for e in sorted((e for e in tr if e.get("cat") == "kernel"), key=lambda e: e["ts"]):
    if "anonymous namespace" in e["name"]:
        print(f"   ours {e['name'][:60]}")
        continue
    ext = e.get("args", {}).get("External id")
    names = [o["name"] for o in ops.get(ext, [])]
    print(f"GLUE {e['name'][:60]:60s} {e.get('dur')} us <- {names}")
