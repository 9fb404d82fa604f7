"""`--profile N` of the training CLIs (tracing): torch.profiler around the first N
training steps after one warm-up step, CPU activity plus the GPU's (ROCm / roctracer) when
the model runs there; the trace goes to <out_dir>/<name>_trace.json (chrome://tracing,
Perfetto) and a per-op table to <name>_ops.txt.  The reference has no tracing; this is the
operator-level view beside bench.py's per-kernel HIP-event times and rocprofv3."""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import torch


class StepProfiler:
    """profiler.step() after every training step; inactive when steps == 0."""

    def __init__(self, out_dir: Path, name: str, steps: int, device: torch.device):
        self.steps = int(steps)
        self.out_dir, self.name = Path(out_dir), name
        self.prof: Optional[torch.profiler.profile] = None
        self.done = False
        if self.steps > 0:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(
                activities=acts, schedule=torch.profiler.schedule(wait=0, warmup=1, active=self.steps, repeat=1),
                on_trace_ready=self._write, record_shapes=False)
            self.prof.__enter__()

    def _write(self, prof) -> None:
        self.out_dir.mkdir(parents=True, exist_ok=True)
        prof.export_chrome_trace(str(self.out_dir / f"{self.name}_trace.json"))
        sort = "self_cuda_time_total" if any(e.device_type.name == "CUDA" for e in prof.events()) else "self_cpu_time_total"
        (self.out_dir / f"{self.name}_ops.txt").write_text(prof.key_averages().table(sort_by=sort, row_limit=40))
        self.done = True

    def step(self) -> None:
        if self.prof is None or self.done:
            return
        self.prof.step()
        if self.done:
            self.close()

    def close(self) -> None:
        if self.prof is not None:
            p, self.prof = self.prof, None
            p.__exit__(None, None, None)
