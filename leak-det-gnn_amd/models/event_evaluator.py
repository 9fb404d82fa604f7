"""Event-level evaluator (reference `eval/event_evaluator.py`), batched per scenario.

SURVEY §8 f rank 4.  The reference walks every stride step of a scenario with a B = 1
residual build and a B = 1 detector forward, pulling each logits row to the host
(`event_evaluator.py:476-492`).  Here a scenario costs two device calls:

1. **One residual pass per scenario.**  The residual at absolute step a,
   `noisy[a] - predictor(noisy[a-l_pred:a], time[a-l_pred:a])`, does not depend on which
   window contains it (`build_residual_segment`, `event_evaluator.py:262-302`), so the
   residual of every step is computed once (`series_residual`: the series cut into
   l_det-step blocks, one batched `build_residual_sequence_from_segment` call, on the GPU
   the shared-window HIP TCN) and each window is a slice of it.  At stride 1 that is
   l_det (36x) fewer predictor windows than the reference's loop.
2. **One batched detector call** over all windows of the scenario (chunks of
   `window_batch`), one host copy of the (W, P+1) logits.

Trigger (`trigger_argmax`, `:327-331`) and aggregation (`aggregate_sum_logits`, `:334-342`)
then run on the host copy with the reference's arithmetic: first window whose argmax is
not the no-leak class; fp32 sum of that window's logits and the following ones whose end
time is < agg_window after it, accumulated row by row in window order.

Scenario selection (`:383-432`), tau from `leak_flow_m3h.csv` (`:204-223`), ATD via the
pipe-distance oracle (`:96-170`), the per-event jsonl / summary.json outputs and the
metric set (`eval/metrics.py:22-160`) follow the reference.  Pinned by
`tests/golden/event.json` (reference evaluator on the synthetic leak set, stand-in
detector): `tests/test_harness.py::test_event_evaluator_matches_reference`.
"""
from __future__ import annotations

import argparse
import json
import random
from collections import defaultdict
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
import torch.nn as nn

from .datasets import SensorStandardizer, make_time_features
from .utils import build_residual_sequence_from_segment
from .window_evaluator import PipeDistanceOracle


# ------------------------------------------------------------------ metrics (eval/metrics.py)
@dataclass
class EventResult:
    """One scenario's outcome (`eval/metrics.py:22-32`)."""
    scenario_id: str
    is_leak_true: bool
    is_leak_pred: bool
    true_pipe_id: Optional[str] = None
    pred_pipe_id: Optional[str] = None
    tau_iso: Optional[str] = None
    alarm_time_iso: Optional[str] = None
    atd_m: Optional[float] = None


def _ratio(a: float, b: float) -> float:
    return float(a / b) if b > 0 else 0.0


def compute_event_metrics(events: Sequence[EventResult], *, success_radii_m: Sequence[float] = (50.0, 100.0, 300.0),
                          localization_mode: str = "detected") -> Dict[str, float]:
    """Scenario-level detection + localisation metrics (`eval/metrics.py:39-160`)."""
    if localization_mode not in ("detected", "all_leaks"):
        raise ValueError("localization_mode must be 'detected' or 'all_leaks'.")
    events = list(events)
    leak = [e for e in events if e.is_leak_true]
    clean = [e for e in events if not e.is_leak_true]
    tp = sum(e.is_leak_pred for e in leak)
    fn = len(leak) - tp
    fp = sum(e.is_leak_pred for e in clean)
    tn = len(clean) - fp
    prec, rec = _ratio(tp, tp + fp), _ratio(tp, tp + fn)
    out: Dict[str, float] = {
        "n_events": float(len(events)), "n_leak_events": float(len(leak)), "n_noleak_events": float(len(clean)),
        "det_tp": float(tp), "det_fp": float(fp), "det_fn": float(fn), "det_tn": float(tn),
        "det_precision": float(prec), "det_recall": float(rec),
        "det_f1": _ratio(2 * prec * rec, prec + rec) if (prec + rec) > 0 else 0.0,
        "det_fp_rate": _ratio(fp, len(clean)), "det_fn_rate": _ratio(fn, len(leak)),
    }
    detected_only = localization_mode == "detected"
    loc = [e for e in leak if e.is_leak_pred] if detected_only else leak
    hit = [e for e in loc if e.is_leak_pred]
    miss = 0 if detected_only else len(loc) - len(hit)
    named = [e for e in hit if e.true_pipe_id is not None and e.pred_pipe_id is not None]
    atd = [float(e.atd_m) for e in hit if e.atd_m is not None]
    succ_total = len(loc) if not detected_only else len(hit)
    out["loc_mode"] = 1.0 if detected_only else 2.0
    out["loc_n_events"] = float(len(loc))
    out["loc_n_detected"] = float(len(hit))
    out["loc_miss_rate"] = _ratio(miss, len(loc)) if loc else 0.0
    out["loc_accuracy_exact"] = _ratio(sum(e.true_pipe_id == e.pred_pipe_id for e in named), len(named))
    out["loc_atd_mean_m"] = float(np.mean(atd)) if atd else float("inf")
    out["loc_atd_median_m"] = float(np.median(atd)) if atd else float("inf")
    for r in success_radii_m:
        out[f"loc_success_at_{int(r)}m"] = _ratio(sum(a <= float(r) for a in atd), succ_total)
    return out


# ------------------------------------------------------------------ scenario files
def read_manifest(manifest_path: str | Path) -> List[Dict]:
    """Non-empty jsonl rows (`event_evaluator.py:173-182`)."""
    with open(manifest_path, "r", encoding="utf-8") as f:
        return [json.loads(s) for s in (ln.strip() for ln in f) if s]


def load_sensors_csv(path: str | Path, sensor_ids: Sequence[str]) -> pd.DataFrame:
    """(T, S) frame in `sensor_ids` order (`:185-189`)."""
    df = pd.read_csv(path, index_col=0, parse_dates=True)
    missing = [c for c in sensor_ids if c not in df.columns]
    if missing:
        raise ValueError(f"Missing sensors in csv: {missing[:10]} ...")
    return df.loc[:, list(sensor_ids)]


def load_leak_flow_csv(path: str | Path) -> pd.Series:
    """Leak flow series; several columns are summed (`:204-211`)."""
    df = pd.read_csv(path, index_col=0, parse_dates=True)
    return df.iloc[:, 0] if df.shape[1] == 1 else df.sum(axis=1)


def find_tau_from_leak_flow(leak_flow: pd.Series, eps: float = 1e-9) -> Optional[pd.Timestamp]:
    """First timestamp with flow > eps (`:214-223`)."""
    on = np.flatnonzero(leak_flow.to_numpy(dtype=np.float64) > float(eps))
    return leak_flow.index[on[0]] if on.size else None


# ------------------------------------------------------------------ trigger + aggregation
def trigger_argmax(records: List[Tuple[pd.Timestamp, torch.Tensor]], noleak_class: int) -> Optional[int]:
    """Index of the first record whose argmax is a pipe (`:327-331`); list API kept for callers."""
    if not records:
        return None
    return first_alarm(torch.stack([lg for _, lg in records]), noleak_class)


def aggregate_sum_logits(records: List[Tuple[pd.Timestamp, torch.Tensor]], start_idx: int,
                         agg_window: pd.Timedelta) -> torch.Tensor:
    """Sum of the logits of records[start_idx:] ending < agg_window after it (`:334-342`)."""
    times = np.asarray([np.datetime64(t, "ns").astype(np.int64) for t, _ in records])
    return sum_logits_from(torch.stack([lg for _, lg in records]), times, start_idx, agg_window)


def first_alarm(logits: torch.Tensor, noleak_class: int) -> Optional[int]:
    """First row of a (W, C) logits matrix whose argmax is not `noleak_class`."""
    alarm = torch.nonzero(logits.argmax(dim=1) != int(noleak_class))
    return int(alarm[0, 0]) if alarm.numel() else None


def sum_logits_from(logits: torch.Tensor, end_ns: np.ndarray, start: int, agg_window: pd.Timedelta) -> torch.Tensor:
    """fp32 row-by-row sum of logits[start:stop) where end_ns[stop] - end_ns[start] is the
    first gap >= agg_window (window end times are increasing)."""
    gap = end_ns[start:] - end_ns[start]
    stop = start + int(np.searchsorted(gap, int(agg_window.value), side="left"))
    if stop == start:
        return logits[start]
    s = logits[start]
    for i in range(start + 1, stop):  # the reference's accumulation order, bit for bit
        s = s + logits[i]
    return s


# ------------------------------------------------------------------ batched scenario pass
@torch.no_grad()
def series_residual(predictor: nn.Module, pressure: torch.Tensor, tfeat: torch.Tensor, l_pred: int,
                    block: int) -> torch.Tensor:
    """Residual of every step a in [l_pred, T) of one series, (T - l_pred, S), in one
    predictor call: the steps are cut into blocks of `block` residual steps, each block
    is one (l_pred + block) segment of a batch (the last block is shifted left to end
    at T), and `build_residual_sequence_from_segment` runs over that batch."""
    T = pressure.shape[0]
    n = T - l_pred
    blk = max(1, min(int(block), n))
    starts = list(range(0, n, blk))
    starts[-1] = n - blk  # last block ends at T (overlaps the previous one)
    idx = torch.tensor(starts, device=pressure.device)[:, None] + torch.arange(l_pred + blk, device=pressure.device)
    res = build_residual_sequence_from_segment(predictor, pressure[idx], tfeat[idx], l_pred, blk)  # (nb, blk, S)
    out = torch.empty(n, pressure.shape[1], dtype=res.dtype, device=pressure.device)
    for i, a in enumerate(starts):
        out[a:a + blk] = res[i]
    return out


@torch.no_grad()
def scenario_window_logits(predictor: nn.Module, detector: nn.Module, pressure: np.ndarray, tfeat: np.ndarray,
                           l_pred: int, l_det: int, stride: int, device: torch.device,
                           window_batch: int = 256) -> Tuple[torch.Tensor, np.ndarray]:
    """Logits of every detection window of one scenario.

    Windows start at t0 = l_pred, l_pred + stride, ... <= T - l_det (`:476-492`); window
    t0 covers residual steps [t0, t0 + l_det) and time features tfeat[t0 : t0 + l_det].
    Returns the (W, C) logits on the host and each window's last step index t0 + l_det - 1.
    """
    T = pressure.shape[0]
    t0 = np.arange(l_pred, T - l_det + 1, max(1, int(stride)), dtype=np.int64)
    if t0.size == 0:
        return torch.empty(0, 0), t0
    p = torch.from_numpy(np.ascontiguousarray(pressure, dtype=np.float32)).to(device)
    tf = torch.from_numpy(np.ascontiguousarray(tfeat, dtype=np.float32)).to(device)
    res_all = series_residual(predictor, p, tf, l_pred, l_det)
    steps = torch.arange(l_det, device=device)
    t0_dev = torch.from_numpy(t0).to(device)
    out = []
    for c in range(0, t0.size, window_batch):
        rows = t0_dev[c:c + window_batch, None] + steps  # (w, l_det) absolute steps
        out.append(detector(res_all[rows - l_pred], tf[rows]).float())
    return torch.cat(out).cpu(), t0 + l_det - 1


# ------------------------------------------------------------------ scenario selection
def select_scenarios(rows: List[Dict], pipe_ids_in_order: Sequence[str], include_noleak: bool, max_leak_scens: int,
                     max_noleak_scens: int, sample_seed: float) -> List[Dict]:
    """Round-robin leak rows over pipes plus a sample of no-leak rows, shuffled, with the
    reference's seeded `random.Random` call sequence (`event_evaluator.py:383-432`)."""
    rng = random.Random(int(sample_seed))
    ok = [r for r in rows if r.get("status", "ok") == "ok"]
    leak = [r for r in ok if r.get("kind") == "leak"]
    clean = [r for r in ok if r.get("kind") == "no_leak"]
    by_pipe: Dict[str, List[Dict]] = defaultdict(list)
    for r in leak:
        if r.get("pipe_id") is not None:
            by_pipe[r["pipe_id"]].append(r)
    for pid in by_pipe:
        rng.shuffle(by_pipe[pid])
    cycle = [pid for pid in pipe_ids_in_order if pid in by_pipe]
    rng.shuffle(cycle)
    chosen: List[Dict] = []
    if int(max_leak_scens) >= 0:
        want = int(max_leak_scens)
        while len(chosen) < want:
            took = False
            for pid in cycle:
                if by_pipe[pid]:
                    chosen.append(by_pipe[pid].pop())
                    took = True
                    if len(chosen) >= want:
                        break
            if not took:
                break
    elif int(max_leak_scens) == -1:
        for pid in cycle:
            chosen.extend(by_pipe[pid])
    else:
        raise ValueError("Invalid max_leak_scens value.")
    extra: List[Dict] = []
    if include_noleak and clean:
        k = min(int(max_noleak_scens), len(clean))
        if k >= 0:
            extra = rng.sample(clean, k)
        elif k == -1:
            extra = clean
        else:
            raise ValueError("Invalid max_noleak_scens value.")
    picked = chosen + extra
    rng.shuffle(picked)
    return picked


# ------------------------------------------------------------------ main evaluation
def evaluate_dataset_event_level(
    dataset_root: str | Path, inp_path: str | Path, device: torch.device,
    predictor: nn.Module, detector: nn.Module, l_pred_steps: int, l_det_steps: int,
    standardizer: SensorStandardizer, sensor_ids: Sequence[str], pipe_ids_in_order: List[str],
    stride_steps: int = 1, agg_window_hours: float = 12.0,
    include_noleak: bool = True, max_leak_scens: int = 0, max_noleak_scens: int = 0, sample_seed: float = 42,
    eps_tau: float = 1e-9, success_radii_m: Sequence[float] = (50.0, 100.0, 300.0),
    out_dir: Optional[str | Path] = None, window_batch: int = 256,
) -> Dict[str, float]:
    """Same signature, outputs and files as `event_evaluator.py:348-571`."""
    dataset_root = Path(dataset_root)
    manifest = dataset_root / "manifest.jsonl"
    if not manifest.exists():
        raise FileNotFoundError(f"manifest.jsonl not found under {dataset_root}")
    pipe_to_idx = {pid: i for i, pid in enumerate(pipe_ids_in_order)}
    noleak_class = len(pipe_ids_in_order)
    num_classes = noleak_class + 1
    print(f"[event-eval] dataset_root={dataset_root}")
    print(f"[event-eval] pipes={len(pipe_ids_in_order)} num_classes={num_classes} include_noleak={include_noleak}")
    print(f"[event-eval] l_pred_steps={l_pred_steps} l_det_steps={l_det_steps} stride_steps={stride_steps} "
          f"agg_window={agg_window_hours}h")
    dist = PipeDistanceOracle.build(inp_path, pipe_ids_in_order)
    agg_window = pd.Timedelta(hours=float(agg_window_hours))
    out_path = Path(out_dir) if out_dir is not None else None
    if out_path is not None:
        out_path.mkdir(parents=True, exist_ok=True)
        (out_path / "per_event.jsonl").unlink(missing_ok=True)

    picked = select_scenarios(read_manifest(manifest), pipe_ids_in_order, include_noleak, max_leak_scens,
                              max_noleak_scens, sample_seed)
    events: List[EventResult] = []
    for idx, r in enumerate(picked, start=1):
        sid, kind = r.get("scenario_id"), r.get("kind")
        if not include_noleak and kind == "no_leak":
            continue
        sdir = dataset_root / str(sid)
        if not (sdir / "sensors.csv").exists():
            print(f"[event-eval][warn] missing sensors.csv for {sid}, skip.")
            continue
        df = load_sensors_csv(sdir / "sensors.csv", sensor_ids)
        if len(df) < l_pred_steps + l_det_steps:
            print(f"[event-eval][warn] too short ({len(df)} rows) for {sid}, skip.")
            continue
        tfeat = make_time_features(pd.to_datetime(df.index))
        pressure = standardizer.transform(df.values.astype(np.float32))
        leak_true = kind == "leak"
        true_pid = r.get("pipe_id") if leak_true else None
        if leak_true and true_pid not in pipe_to_idx:
            print(f"[event-eval][warn] pipe_id {true_pid} not in label space, skip {sid}.")
            continue
        tau = None
        if leak_true:
            if (sdir / "leak_flow_m3h.csv").exists():
                tau = find_tau_from_leak_flow(load_leak_flow_csv(sdir / "leak_flow_m3h.csv"), eps=eps_tau)
            else:
                print(f"[event-eval][warn] missing leak_flow_m3h.csv for leak scenario {sid}.")
        tau_iso = tau.isoformat() if tau is not None else None

        logits, last = scenario_window_logits(predictor, detector, pressure, tfeat, l_pred_steps, l_det_steps,
                                              stride_steps, device, window_batch)
        if logits.numel() and logits.shape[1] != num_classes:
            raise RuntimeError(f"Detector logits dim {logits.shape[1]} != expected num_classes {num_classes}")
        trig = first_alarm(logits, noleak_class) if logits.numel() else None
        if trig is None:
            ev = EventResult(str(sid), bool(leak_true), False, true_pid, None, tau_iso, None, None)
        else:
            ends = df.index[last]
            summed = sum_logits_from(logits, ends.asi8, trig, agg_window)
            pred_idx = int(torch.argmax(summed))
            pred_leak = pred_idx != noleak_class
            pred_pid = pipe_ids_in_order[pred_idx] if pred_leak else None
            atd = float(dist.pipe_distance(pipe_to_idx[true_pid], pred_idx)) if (pred_leak and leak_true) else None
            ev = EventResult(str(sid), bool(leak_true), bool(pred_leak), true_pid, pred_pid, tau_iso,
                             ends[trig].isoformat(), atd)
        events.append(ev)
        if idx % 25 == 0 or idx == len(picked):
            print(f"[event-eval] processed {idx}/{len(picked)} scenarios...")
        if out_path is not None:
            with open(out_path / "per_event.jsonl", "a", encoding="utf-8") as f:
                f.write(json.dumps(asdict(ev), ensure_ascii=False) + "\n")

    summary = compute_event_metrics(events, success_radii_m=success_radii_m, localization_mode="detected")
    print("[event-eval] SUMMARY")
    for k in ("n_events", "n_leak_events", "n_noleak_events", "det_precision", "det_recall", "det_f1",
              "det_fp_rate", "det_fn_rate", "loc_n_events", "loc_n_detected", "loc_accuracy_exact",
              "loc_atd_mean_m", "loc_atd_median_m", "loc_success_at_50m", "loc_success_at_100m",
              "loc_success_at_300m"):
        if k in summary:
            v = summary[k]
            print(f"  {k}: {v:.6f}" if isinstance(v, float) and abs(v) < 1e6 else f"  {k}: {v}")
    if out_path is not None:
        with open(out_path / "summary.json", "w", encoding="utf-8") as f:
            json.dump(summary, f, ensure_ascii=False, indent=2)
        print(f"[event-eval] saved: {out_path / 'summary.json'} , {out_path / 'per_event.jsonl'}")
    return summary


def main() -> None:
    """CLI with the reference's flags (`event_evaluator.py:574-626`)."""
    from .detector import LeakDetector
    from .predictor import NormalPredictorGRU, NormalPredictorTCN
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset_root", type=str, required=True)
    ap.add_argument("--inp_path", type=str, required=True)
    ap.add_argument("--predictor_ckpt", type=str, required=True)
    ap.add_argument("--detector_ckpt", type=str, required=True)
    ap.add_argument("--device", type=str, default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--l_pred_hours", type=float, default=3.0)
    ap.add_argument("--l_det_hours", type=float, default=3.0)
    ap.add_argument("--step_minutes", type=float, default=5.0)
    ap.add_argument("--stride_minutes", type=float, default=5.0)
    ap.add_argument("--agg_window_hours", type=float, default=12.0)
    ap.add_argument("--include_noleak", action="store_true")
    ap.add_argument("--max_leak_scens", type=int, default=0)
    ap.add_argument("--max_noleak_scens", type=int, default=0)
    ap.add_argument("--sample_seed", type=int, default=42)
    ap.add_argument("--out_dir", type=str, default=None)
    ap.add_argument("--window_batch", type=int, default=256, help="windows per detector call")
    args = ap.parse_args()
    device = torch.device(args.device)
    per_hour = int(round(60.0 / float(args.step_minutes)))
    l_pred = int(round(float(args.l_pred_hours) * per_hour))
    l_det = int(round(float(args.l_det_hours) * per_hour))
    stride = max(1, int(round(float(args.stride_minutes) / float(args.step_minutes))))
    # weights_only load; LEAKGNN_TRUST_CKPT=1 opts in to a trusted foreign checkpoint
    from .train_detector import _load_ckpt
    pck = _load_ckpt(args.predictor_ckpt, torch.device("cpu"))
    dck = _load_ckpt(args.detector_ckpt, torch.device("cpu"))
    S = len(pck["sensor_ids"])
    pred_cls = NormalPredictorGRU if pck.get("arch", "tcn") == "gru" else NormalPredictorTCN
    predictor = pred_cls(num_sensors=S, time_dim=9)
    predictor.load_state_dict(pck["model_state"])
    predictor.to(device).eval()
    detector = LeakDetector(args.inp_path, dck["sensor_ids"], dck["pipe_ids_in_order"], sensor_hidden=64,
                            node_hidden=64, gnn_layers=2, dropout=0.1, use_time=True)
    detector.load_state_dict(dck["detector_state"])
    detector.to(device).eval()
    if list(pck["sensor_ids"]) != list(dck["sensor_ids"]):
        raise ValueError("predictor and detector checkpoints disagree on sensor_ids")
    def _stat(v):  # lists (this build), numpy arrays (reference) or tensors on any device
        return np.asarray(v.detach().cpu() if torch.is_tensor(v) else v, dtype=np.float32)

    std = SensorStandardizer(mean=_stat(pck["standardizer_mean"]), std=_stat(pck["standardizer_std"]))
    evaluate_dataset_event_level(
        args.dataset_root, args.inp_path, device, predictor, detector, l_pred, l_det, std, dck["sensor_ids"],
        dck["pipe_ids_in_order"], stride_steps=stride, agg_window_hours=args.agg_window_hours,
        include_noleak=bool(args.include_noleak), max_leak_scens=int(args.max_leak_scens),
        max_noleak_scens=int(args.max_noleak_scens), sample_seed=float(args.sample_seed), out_dir=args.out_dir,
        window_batch=args.window_batch)


if __name__ == "__main__":
    main()
