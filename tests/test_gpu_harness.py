"""GPU side of the harness (SURVEY §8 b, f-3): the HBM-resident batch path equals the
reference-style DataLoader path, and train_predictor / train_detector run end to end on
the synthetic data set with the reference CLI flags."""
from __future__ import annotations

import json

import numpy as np
import pytest
import torch

from helpers import GOLD, LTA_INP

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
INFO = json.loads((GOLD / "harness.json").read_text())


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    from models.synth import write_synthetic_leak_set, write_synthetic_normal_set
    d = tmp_path_factory.mktemp("synthds_gpu")
    write_synthetic_normal_set(d / "normal", INFO["sensors"], n_windows=12, T=577, seed=0)
    write_synthetic_leak_set(d / "leak", INFO["sensors"], INFO["pipes"], scenes_per_pipe=2, n_noleak=6, T=400, seed=0)
    return d


def _same_batch(a: dict, b: dict):
    assert set(a) == set(b)
    for k in a:
        if torch.is_tensor(b[k]):
            assert torch.equal(a[k].cpu(), b[k].cpu()), k
        else:
            assert list(a[k]) == list(b[k]), k


def test_device_loader_equals_dataloader(data):
    from torch.utils.data import DataLoader
    from models.datasets import (AbruptLeakDetectorDataset, DeviceBatchLoader, NormalPredictorDataset,
                                 compute_sensor_stats_from_normal)
    st = compute_sensor_stats_from_normal(data / "normal")
    dds = AbruptLeakDetectorDataset(data / "leak", steps_per_epoch=37, seed=5, standardizer=st,
                                    sensor_ids=INFO["sensors"])
    ref = list(DataLoader(dds, batch_size=8))
    got = list(DeviceBatchLoader(dds, 8, DEV))
    assert len(ref) == len(got) == 5
    for a, b in zip(got, ref):
        assert a["noisy_seg"].device.type == "cuda"
        _same_batch(a, b)
    nds = NormalPredictorDataset(data / "normal", steps_per_epoch=20, seed=3, standardizer=st)
    for a, b in zip(DeviceBatchLoader(nds, 8, DEV), DataLoader(nds, batch_size=8)):
        _same_batch(a, b)


def test_train_predictor_and_detector_cli(data, tmp_path, capsys):
    """Reference CLI flags end to end.  The leak set here has enough scenes for non-empty
    80/10/10 splits (the reference trainer needs >= 1 scene per split)."""
    from models import train_detector, train_predictor
    from models.synth import write_synthetic_leak_set
    write_synthetic_leak_set(tmp_path / "leak", INFO["sensors"], INFO["pipes"], scenes_per_pipe=4, n_noleak=12,
                             T=300, seed=1)
    out = tmp_path / "out"
    train_predictor.main(["--normal_root", str(data / "normal"), "--out_dir", str(out), "--epochs", "1",
                          "--steps_per_epoch", "32", "--val_steps", "16", "--test_steps", "16", "--batch_size", "8",
                          "--device", "cuda", "--log_every", "2"])
    ck = torch.load(out / "predictor_best.ckpt", weights_only=True)
    assert ck["sensor_ids"] == INFO["sensors"] and ck["arch"] == "tcn"
    assert set(ck) == {"epoch", "arch", "model_state", "standardizer_mean", "standardizer_std", "sensor_ids", "args"}
    train_detector.main(["--leak_root", str(tmp_path / "leak"), "--inp_path", str(LTA_INP), "--predictor_ckpt",
                         str(out / "predictor_best.ckpt"), "--out_dir", str(out), "--epochs", "2",
                         "--steps_per_epoch", "16", "--val_steps", "16", "--test_steps", "16", "--batch_size", "8",
                         "--device", "cuda", "--log_every", "1", "--profile", "2"])
    trace = json.loads((out / "detector_trace.json").read_text())  # --profile 2: torch.profiler, GPU activity
    assert len({str(e.get("name", "")) for e in trace["traceEvents"]} & {f"ProfilerStep#{i}" for i in range(8)}) == 2
    ck = torch.load(out / "detector_best.ckpt", weights_only=True)
    assert ck["pipe_ids_in_order"] == INFO["pipe_ids_in_order"] and ck["num_classes"] == len(INFO["pipes"]) + 1
    assert set(ck) == {"epoch", "detector_state", "sensor_ids", "pipe_ids_in_order", "num_classes",
                       "predictor_ckpt", "args"}
    meta = json.loads((out / "detector_meta.json").read_text())
    assert meta["sampling_config"]["p_early"] == 0.3
    log = capsys.readouterr().out
    assert "[detector] TEST:" in log and "ATD=" in log and "loss=" in log
    losses = [float(l.split("loss=")[1].split()[0]) for l in log.splitlines() if "[detector][epoch" in l and "loss=" in l]
    assert all(np.isfinite(losses)) and len(losses) >= 2


def test_event_evaluator_gpu_matches_reference(data):
    """Event-level evaluator on the GPU (residuals from the HIP shared-window TCN over the
    whole scenario, one batched detector call) == the reference's per-step CPU loop
    (tests/golden/event.json): alarm times, predicted pipes, ATD and summary metrics."""
    from test_harness import _check_events, _check_metrics, _event_cases, _run_event_case, _tcn
    arrs = np.load(GOLD / "harness.npz")
    for case in _event_cases()["cases"]:
        summary, events = _run_event_case(case, data / "leak", arrs, DEV, _tcn())
        _check_metrics(summary, case["summary"])
        _check_events(events, [dict(e) for e in case["events"]])


def test_event_windows_batched_equal_per_window_loop(data):
    """scenario_window_logits on a LeakDetector == the reference's loop shape: per window,
    build_residual_segment on its own (l_pred + l_det) segment and a B = 1 detector call
    (`event_evaluator.py:476-492`), fp32 within 1e-5 relative of the logit scale."""
    import pandas as pd
    from models.datasets import SensorStandardizer, make_time_features
    from models.detector import LeakDetector
    from models.event_evaluator import load_sensors_csv, scenario_window_logits
    from models.utils import build_residual_sequence_from_segment
    from test_harness import _tcn
    arrs = np.load(GOLD / "harness.npz")
    sid = sorted(p.name for p in (data / "leak").iterdir() if p.is_dir() and "abrupt" in p.name)[0]
    df = load_sensors_csv(data / "leak" / sid / "sensors.csv", INFO["sensors"])
    std = SensorStandardizer(mean=arrs["std_mean"], std=arrs["std_std"])
    pressure = std.transform(df.values.astype(np.float32))
    tfeat = make_time_features(pd.to_datetime(df.index))
    torch.manual_seed(0)
    det = LeakDetector(LTA_INP, INFO["sensors"], INFO["pipes"]).to(DEV).eval()
    tcn = _tcn().to(DEV)
    logits, last = scenario_window_logits(tcn, det, pressure, tfeat, 36, 36, 5, DEV, window_batch=16)
    assert logits.shape == (len(last), len(INFO["pipes"]) + 1) and len(last) > 40
    p, tf = torch.from_numpy(pressure).to(DEV), torch.from_numpy(tfeat).to(DEV)
    with torch.no_grad():
        for w, end in enumerate(last):
            t0 = int(end) - 36 + 1
            res = build_residual_sequence_from_segment(tcn, p[t0 - 36:t0 + 36], tf[t0 - 36:t0 + 36], 36, 36)
            ref = det(res[None], tf[None, t0:t0 + 36]).float().cpu()[0]
            assert (logits[w] - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6, w


def _dp_trainer_worker(rank, world, port, argv):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from models import train_detector
    from models.detector import LeakDetector

    class NoDropout(LeakDetector):  # dropout off: masks are per-rank draws, the comparison must be exact
        def __init__(self, *a, **k):
            k["dropout"] = 0.0
            super().__init__(*a, **k)
    train_detector.LeakDetector = NoDropout
    train_detector.main(argv)


@pytest.mark.parametrize("steps,log_every", [(24, 10), (25, 1)])
def test_train_detector_data_parallel_equals_single_process(data, tmp_path, steps, log_every):
    """train_detector under a 2-rank launch (torchrun environment, gloo, both ranks on this
    GPU): each rank trains on its half of every global batch of --batch_size samples and the
    gradients are all-reduced; rank 0's checkpoint equals a single-process run's on the same
    global batches (dropout off on both sides).  steps 25: the last global batch is ONE window,
    so rank 1 gets none and must still join every collective (the step's all-reduce and, at
    --log_every 1, the logging all-reduces)."""
    import socket
    import torch.multiprocessing as mp
    from models import train_detector, train_predictor
    from models.detector import LeakDetector
    from models.synth import write_synthetic_leak_set
    write_synthetic_leak_set(tmp_path / "leak", INFO["sensors"], INFO["pipes"], scenes_per_pipe=4, n_noleak=12,
                             T=300, seed=1)
    out = tmp_path / "pred"
    train_predictor.main(["--normal_root", str(data / "normal"), "--out_dir", str(out), "--epochs", "1",
                          "--steps_per_epoch", "16", "--val_steps", "8", "--test_steps", "8", "--batch_size", "8",
                          "--device", "cuda"])

    def argv(o):
        return ["--leak_root", str(tmp_path / "leak"), "--inp_path", str(LTA_INP), "--predictor_ckpt",
                str(out / "predictor_best.ckpt"), "--out_dir", str(o), "--epochs", "1", "--steps_per_epoch", str(steps),
                "--val_steps", "8", "--test_steps", "8", "--batch_size", "8", "--device", "cuda",
                "--dist_backend", "gloo", "--log_every", str(log_every)]
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.start_processes(_dp_trainer_worker, args=(2, port, argv(tmp_path / "dp")), nprocs=2, start_method="spawn")

    class NoDropout(LeakDetector):
        def __init__(self, *a, **k):
            k["dropout"] = 0.0
            super().__init__(*a, **k)
    orig = train_detector.LeakDetector
    train_detector.LeakDetector = NoDropout
    try:
        train_detector.main(argv(tmp_path / "sp"))
    finally:
        train_detector.LeakDetector = orig
    a = torch.load(tmp_path / "dp" / "detector_last.ckpt", weights_only=True)["detector_state"]
    b = torch.load(tmp_path / "sp" / "detector_last.ckpt", weights_only=True)["detector_state"]
    assert set(a) == set(b)
    for k in b:
        d = (a[k].double() - b[k].double()).abs().max().item()
        assert d <= 2e-5 * max(b[k].abs().max().item(), 1e-3), f"{k}: {d:.3e}"


def test_train_detector_captured_cli_equals_eager_cli(data, tmp_path):
    """--capture on (every full-size batch's step one replayed HIP graph, the tail batch
    eager) writes the checkpoint the eager CLI (--capture off) writes, dropout off on both
    sides (the graph draws its masks from device seed slots); the JSONL perf log has one
    line per log interval with windows/s."""
    from models import train_detector, train_predictor
    from models.detector import LeakDetector
    from models.synth import write_synthetic_leak_set
    write_synthetic_leak_set(tmp_path / "leak", INFO["sensors"], INFO["pipes"], scenes_per_pipe=4, n_noleak=12,
                             T=300, seed=1)
    out = tmp_path / "pred"
    train_predictor.main(["--normal_root", str(data / "normal"), "--out_dir", str(out), "--epochs", "1",
                          "--steps_per_epoch", "16", "--val_steps", "8", "--test_steps", "8", "--batch_size", "8",
                          "--device", "cuda"])

    class NoDropout(LeakDetector):
        def __init__(self, *a, **k):
            k["dropout"] = 0.0
            super().__init__(*a, **k)

    def run(o, mode):
        train_detector.main(["--leak_root", str(tmp_path / "leak"), "--inp_path", str(LTA_INP), "--predictor_ckpt",
                             str(out / "predictor_best.ckpt"), "--out_dir", str(o), "--epochs", "2",
                             "--steps_per_epoch", "20", "--val_steps", "8", "--test_steps", "8", "--batch_size", "8",
                             "--device", "cuda", "--log_every", "1", "--capture", mode])
    orig = train_detector.LeakDetector
    train_detector.LeakDetector = NoDropout
    try:
        run(tmp_path / "g", "on")
        run(tmp_path / "e", "off")
    finally:
        train_detector.LeakDetector = orig
    a = torch.load(tmp_path / "g" / "detector_last.ckpt", weights_only=True)["detector_state"]
    b = torch.load(tmp_path / "e" / "detector_last.ckpt", weights_only=True)["detector_state"]
    assert set(a) == set(b)
    for k in b:
        d = (a[k].double() - b[k].double()).abs().max().item()
        assert d <= 1e-6 * max(b[k].abs().max().item(), 1e-3), f"{k}: {d:.3e}"
    recs = [json.loads(ln) for ln in (tmp_path / "g" / "detector_perf.jsonl").read_text().splitlines()]
    assert len(recs) == 6  # 2 epochs x 3 batches (8, 8, tail 4)
    assert [r["mode"] for r in recs[:3]] == ["graph"] * 3  # the graph exists from the first full batch on
    assert [r["windows"] for r in recs[:3]] == [8, 8, 4] and all(r["windows_per_s"] > 0 for r in recs)
    eager = [json.loads(ln) for ln in (tmp_path / "e" / "detector_perf.jsonl").read_text().splitlines()]
    assert {r["mode"] for r in eager} == {"eager"}
