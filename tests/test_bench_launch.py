"""bench.py's multi-rank launch path on CPU (gloo): `--gpus N` without torchrun's
environment starts N ranks itself, and a --gpus / WORLD_SIZE mismatch is refused."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_gpus2_self_launch_dry_run():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--dry-run"], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["dry_run"] is True
    assert d["steps"] == 3 and d["config"]["parallelism"] == "dp2"
    # the exchange fields the driver's multi-GPU line carries (bench.py exchange_fields)
    assert d["allreduce_us"] > 0 and d["exchange_exposed_us"] >= 0
    assert 0 < d["weak_scaling_eff"] <= 1 and isinstance(d["exchange"], str)


def test_exchange_fields_single_rank_and_arithmetic():
    sys.path.insert(0, str(REPO))
    import bench
    one = bench.exchange_fields(1.0, 1.0, 0.0, 10, 1, "none")
    assert one["allreduce_us"] == 0.0 and one["weak_scaling_eff"] == 1.0
    two = bench.exchange_fields(1.2, 1.0, 0.3, 100, 2, "x")
    assert two["allreduce_us"] == 3000.0 and two["exchange_exposed_us"] == 2000.0
    assert abs(two["weak_scaling_eff"] - 1.0 / 1.2) < 1e-4


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dry-run"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
