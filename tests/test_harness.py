"""Caller-harness counterparts (SURVEY §8 b) and the data pipeline (§8 f rank 3) against
fixtures produced by the reference's own models/datasets.py, train_detector.py split
functions and window_evaluator.py (oracle/make_golden.py: harness_fixture) on a seeded
synthetic data set in the reference on-disk format, regenerated here by models/synth.py.

Bars: sampled indices / ids / labels / buckets / timestamps exact; window arrays and the
standardizer bit-exact (same float32 arithmetic); evaluator metrics exact for counts and
rates and within 1e-9 relative for the distance means.
"""
from __future__ import annotations

import json
import math

import numpy as np
import pytest
import torch

from helpers import GOLD, LTA_INP, lta_ids

SENSORS = json.loads((GOLD / "harness.json").read_text())["sensors"]


@pytest.fixture(scope="module")
def fx():
    return json.loads((GOLD / "harness.json").read_text()), np.load(GOLD / "harness.npz")


@pytest.fixture(scope="module")
def data(tmp_path_factory, fx):
    from models.synth import write_synthetic_leak_set, write_synthetic_normal_set
    info, _ = fx
    d = tmp_path_factory.mktemp("synthds")
    write_synthetic_normal_set(d / "normal", SENSORS, n_windows=12, T=577, seed=0)
    write_synthetic_leak_set(d / "leak", SENSORS, info["pipes"], scenes_per_pipe=2, n_noleak=6, T=400, seed=0)
    return d


def test_standardizer_and_predictor_samples(fx, data):
    from models.datasets import NormalPredictorDataset, compute_sensor_stats_from_normal
    info, arrs = fx
    st = compute_sensor_stats_from_normal(data / "normal")
    assert np.array_equal(st.mean, arrs["std_mean"]) and np.array_equal(st.std, arrs["std_std"])
    ds = NormalPredictorDataset(data / "normal", steps_per_epoch=50, seed=42, standardizer=st)
    for i, ref in enumerate(info["normal_samples"]):
        s = ds[i]
        assert (s["scene_id"], s["t"]) == (ref["scene_id"], ref["t"]), i
        for k in ("x", "x_time", "y"):
            assert np.array_equal(s[k].numpy(), arrs[f"normal.{i}.{k}"]), (i, k)


def test_detector_dataset_samples(fx, data):
    from models.datasets import AbruptLeakDetectorDataset, SensorStandardizer
    info, arrs = fx
    st = SensorStandardizer(arrs["std_mean"], arrs["std_std"])
    ds = AbruptLeakDetectorDataset(data / "leak", steps_per_epoch=64, seed=123, standardizer=st, sensor_ids=SENSORS)
    assert ds.leak_scene_ids == info["leak_scene_ids"]
    assert ds.noleak_scene_ids == info["noleak_scene_ids"]   # the "failed" manifest row is filtered out
    assert ds.get_pipe_ids_in_order() == info["pipe_ids_in_order"]
    assert {sid: {b: int(v.size) for b, v in bt.items()} for sid, bt in ds._bucket_times.items()} == \
        info["bucket_sizes"]
    buckets = set()
    for i, ref in enumerate(info["leak_samples"]):
        s = ds[i]
        got = {k: (str(v) if k in ("scenario_id", "bucket", "t", "pipe_id") else int(v))
               for k, v in s.items() if k not in ("noisy_seg", "time_seg")}
        assert got == ref, i
        assert np.array_equal(s["noisy_seg"].numpy(), arrs[f"leak.{i}.noisy_seg"]), i
        assert np.array_equal(s["time_seg"].numpy(), arrs[f"leak.{i}.time_seg"]), i
        buckets.add(ref["bucket"])
    assert buckets == {"early", "late", "pre", "noleak"}  # every sampling bucket is exercised


def test_trainer_splits(fx):
    from models.train_detector import split_leak_scenids, split_normal_scenids
    info, _ = fx
    fake = [f"{k:06d}_p{k % 12}_abrupt_r{k // 12 + 1}" for k in range(50)]
    assert [list(x) for x in split_leak_scenids(fake, 42, ratio=(0.8, 0.1, 0.1))] == info["split_leak"]
    assert [list(x) for x in split_normal_scenids([f"w{k}" for k in range(23)], 53)] == info["split_normal"]


def _fixed_detector(arrs):
    class FixedLogitsDetector(torch.nn.Module):
        def forward(self, residual, tfeat):
            dev = residual.device
            A, Bm, c = (torch.from_numpy(arrs[f"eval.{k}"]).to(dev) for k in ("A", "Bm", "c"))
            return 3.0 * torch.tanh(residual.mean(1) @ A + tfeat.mean(1) @ Bm) + c
    return FixedLogitsDetector()


def _tcn():
    from models.predictor import NormalPredictorTCN
    p = np.load(GOLD / "predictor.npz")
    m = NormalPredictorTCN(num_sensors=29, time_dim=9).eval()
    m.load_state_dict({k[4:]: torch.from_numpy(p[k]) for k in p.files if k.startswith("tcn.")})
    return m


def _check_metrics(got: dict, ref: dict):
    assert set(got) == set(ref), set(got) ^ set(ref)
    for k, v in ref.items():
        g = got[k]
        if math.isinf(v):
            assert math.isinf(g), k
        else:
            assert abs(g - v) <= 1e-9 * max(1.0, abs(v)), (k, g, v)


def test_window_evaluator_matches_reference(fx, data):
    from torch.utils.data import DataLoader
    from models.datasets import AbruptLeakDetectorDataset, SensorStandardizer
    from models.window_evaluator import DetectorEvaluator
    info, arrs = fx
    st = SensorStandardizer(arrs["std_mean"], arrs["std_std"])
    eds = AbruptLeakDetectorDataset(data / "leak", steps_per_epoch=48, seed=7, standardizer=st, sensor_ids=SENSORS)
    ev = DetectorEvaluator(_tcn(), _fixed_detector(arrs), torch.device("cpu"), l_pred=36, l_det=36, topk=5,
                           metric_groups=("basic", "binary", "bucket", "atd", "success", "accuracy_i"),
                           inp_path=LTA_INP, pipe_ids_in_order=info["pipe_ids_in_order"])
    _check_metrics(ev.evaluate(DataLoader(eds, batch_size=16)), info["eval_metrics"])


# ------------------------------------------------------------------ event-level evaluator
def _event_cases():
    return json.loads((GOLD / "event.json").read_text())


def _run_event_case(case, root, arrs, device, predictor):
    from models.datasets import SensorStandardizer
    from models.event_evaluator import evaluate_dataset_event_level
    c = dict(case["args"])
    bias = np.float32(c.pop("noleak_bias", 0.0))
    cc = arrs["eval.c"].copy()
    cc[-1] += bias
    A, Bm, cv = (torch.from_numpy(v).to(device) for v in (arrs["eval.A"], arrs["eval.Bm"], cc))

    class StandIn(torch.nn.Module):  # oracle/make_golden.py FixedLogitsDetector
        def forward(self, residual, tfeat):
            return 3.0 * torch.tanh(residual.mean(1) @ A + tfeat.mean(1) @ Bm) + cv

    std = SensorStandardizer(mean=arrs["std_mean"], std=arrs["std_std"])
    out = root / "out"
    summary = evaluate_dataset_event_level(root, LTA_INP, device, predictor.to(device), StandIn(), 36, 36, std,
                                           SENSORS, _event_cases()["pipes"], sample_seed=42, out_dir=out, **c)
    events = [json.loads(ln) for ln in (out / "per_event.jsonl").read_text().splitlines() if ln]
    return summary, events


def _check_events(got, ref):
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        atd_g, atd_r = g.pop("atd_m"), r.pop("atd_m")
        assert g == r
        assert (atd_g is None) == (atd_r is None) and (atd_r is None or abs(atd_g - atd_r) <= 1e-9 * max(1.0, atd_r))


@pytest.fixture(scope="module")
def event_data(tmp_path_factory):
    from models.synth import write_synthetic_leak_set
    d = tmp_path_factory.mktemp("eventds") / "leak"
    write_synthetic_leak_set(d, SENSORS, _event_cases()["pipes"], scenes_per_pipe=2, n_noleak=6, T=400, seed=0)
    return d


def test_event_evaluator_matches_reference(fx, event_data):
    """Batched evaluator (one residual pass + one detector call per scenario) == the
    reference's per-stride-step loop on CPU: selection order, tau, alarm time, predicted
    pipe, ATD and every summary metric, over four argument sets (stride 1-3, aggregation
    0.5-12 h, with and without no-leak scenarios, alarms that come late or never)."""
    _, arrs = fx
    cases = _event_cases()["cases"]
    # the fixture covers events whose aggregated logits fall back to no-leak
    assert any(e["is_leak_true"] and not e["is_leak_pred"] for c in cases for e in c["events"])
    for case in cases:
        summary, events = _run_event_case(case, event_data, arrs, torch.device("cpu"), _tcn())
        _check_metrics(summary, case["summary"])
        _check_events(events, [dict(e) for e in case["events"]])


def test_event_trigger_and_aggregation_helpers():
    """List-API helpers (`event_evaluator.py:327-342`) on hand-made records."""
    import pandas as pd
    from models.event_evaluator import aggregate_sum_logits, trigger_argmax
    t = pd.date_range("2024-01-01", periods=6, freq="5min")
    lg = [torch.tensor([0.0, 1.0]), torch.tensor([0.0, 2.0]), torch.tensor([3.0, 1.0]), torch.tensor([1.0, 0.5]),
          torch.tensor([0.25, 4.0]), torch.tensor([9.0, 0.0])]
    rec = list(zip(t, lg))
    assert trigger_argmax(rec, noleak_class=1) == 2
    assert trigger_argmax(rec[:2], noleak_class=1) is None
    assert trigger_argmax([], noleak_class=1) is None
    s = aggregate_sum_logits(rec, 2, pd.Timedelta(minutes=15))  # rows 2, 3, 4 (gap 15 min stops)
    assert torch.equal(s, lg[2] + lg[3] + lg[4])
    assert torch.equal(aggregate_sum_logits(rec, 5, pd.Timedelta(minutes=15)), lg[5])
    assert torch.equal(aggregate_sum_logits(rec, 3, pd.Timedelta(0)), lg[3])


def test_train_predictor_cpu_plumbing(data, tmp_path):
    """configs[0]: train_predictor on the CPU, 1 epoch, batch 1 (the reference's plumbing
    run), reference flags; the checkpoint's standardizer stats are plain floats that the
    reference loaders' np.asarray(std, dtype=float32) accepts after a weights_only load."""
    from models import train_predictor
    out = tmp_path / "out"
    train_predictor.main(["--normal_root", str(data / "normal"), "--out_dir", str(out), "--epochs", "1",
                          "--steps_per_epoch", "4", "--val_steps", "2", "--test_steps", "2", "--batch_size", "1",
                          "--device", "cpu", "--log_every", "2"])
    ck = torch.load(out / "predictor_best.ckpt", map_location="cpu", weights_only=True)
    mean = np.asarray(ck["standardizer_mean"], dtype=np.float32)
    std = np.asarray(ck["standardizer_std"], dtype=np.float32)
    assert mean.shape == std.shape == (len(ck["sensor_ids"]),) and (std > 0).all()
    assert (out / "predictor_last.ckpt").is_file() and (out / "predictor_meta.json").is_file()


def test_train_predictor_profile_switch(data, tmp_path):
    """--profile N (SURVEY §5 tracing): torch.profiler over N training steps after one warm-up
    step writes a chrome trace and a per-op table next to the checkpoints (CPU run here; the
    detector CLI has the same switch, exercised on the GPU in test_gpu_harness)."""
    import json as _json
    from models import train_predictor
    out = tmp_path / "out"
    train_predictor.main(["--normal_root", str(data / "normal"), "--out_dir", str(out), "--epochs", "1",
                          "--steps_per_epoch", "6", "--val_steps", "2", "--test_steps", "2", "--batch_size", "1",
                          "--device", "cpu", "--log_every", "100", "--profile", "3"])
    trace = _json.loads((out / "predictor_trace.json").read_text())
    names = {e.get("name", "") for e in trace["traceEvents"]}
    assert any("ProfilerStep" in n for n in names), "no profiler steps in the trace"
    assert sum(1 for n in names if n.startswith("ProfilerStep#")) == 3
    assert "aten::" in (out / "predictor_ops.txt").read_text()
