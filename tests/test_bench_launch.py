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


def test_short_kernel_name_and_small_kernel_entries():
    """rocprofv3 kernel names -> the names the step accounting sums (bench.small_kernels_us),
    including names whose argument list carries anonymous-namespace types."""
    sys.path.insert(0, str(REPO))
    import bench
    names = {"void (anonymous namespace)::k_slab_reduce<24>((anonymous namespace)::Segs)": "k_slab_reduce",
             "void (anonymous namespace)::k_adam_update(float*, float const*, (anonymous namespace)::AdamArgs)":
                 "k_adam_update",
             "void (anonymous namespace)::k_gcn_fwd_pc<64, true, false>((anonymous namespace)::PcX0)": "k_gcn_fwd_pc",
             "k_ce_fwd(float const*, long)": "k_ce_fwd"}
    for full, short in names.items():
        assert bench.short_kernel_name(full) == short
    by = {"k_slab_reduce": 12.5, "k_adam_update": 3.0, "k_adam_norm": 1.0, "k_ce_fwd": 2.0, "k_ce_mean": 0.5}
    got = bench.small_kernels_us({"by_name_us": by})
    assert got["slab_reduce"] == 12.5 and got["adam"] == 4.0 and got["ce_fwd"] == 2.5 and "seed" not in got  # fused launches: no entry
