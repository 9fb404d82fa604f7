"""WDN datasets (reference models/datasets.py) with a device-resident batch path.

Reference-compatible API (same constructor arguments, same sample dicts, same numpy RNG
draws, so a given (seed, idx) yields the identical sample):
  make_time_features                         datasets.py:49-59
  SensorStandardizer                         datasets.py:62-70
  compute_sensor_stats_from_normal           datasets.py:72-111
  ScenarioStore (LRU CSV loader)             datasets.py:126-194
  NormalPredictorDataset                     datasets.py:200-257
  DetectorSamplingConfig                     datasets.py:263-279
  AbruptLeakDetectorDataset                  datasets.py:282-543

MI355X path (SURVEY §8 f rank 3): ``DeviceBatchLoader`` keeps every scenario of a
dataset resident in HBM as one (scenes, T, S) tensor (+ time features), draws each
sample's (scene, time, label) with the dataset's own per-index RNG on the host, and
forms a whole batch of windows with ONE device gather — no per-sample CSV/LRU work and
no host-to-device copy of windows per step.  It yields the same batch dicts a
``torch.utils.data.DataLoader(ds, batch_size, shuffle=False)`` would, with the tensors
already on the device.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch
from torch.utils.data import Dataset


# ----------------------------------------------------------------------------- utils
def _read_manifest_jsonl(path: Path) -> List[Dict[str, Any]]:
    """datasets.py:24-32: one JSON object per non-empty line."""
    rows: List[Dict[str, Any]] = []
    with path.open("r", encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if line:
                rows.append(json.loads(line))
    return rows


def _filter_ok(rows: Iterable[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """datasets.py:35-40: keep rows whose status (default "ok") is "ok"."""
    return [r for r in rows if str(r.get("status", "ok")).lower() == "ok"]


def _ensure_sensor_order(df: pd.DataFrame, sensor_ids: Sequence[str]) -> pd.DataFrame:
    """datasets.py:43-47."""
    missing = [c for c in sensor_ids if c not in df.columns]
    if missing:
        raise ValueError(f"Missing sensors in csv: {missing[:10]} (and {len(missing) - 10} more)")
    return df.loc[:, list(sensor_ids)]


def make_time_features(dt_index: pd.DatetimeIndex) -> np.ndarray:
    """(T, 9) float32: hour sin/cos + day-of-week one-hot (datasets.py:49-59)."""
    hour = dt_index.hour.astype(np.float32) + (dt_index.minute.astype(np.float32) / 60.0) + (
        dt_index.second.astype(np.float32) / 3600.0)
    hour = np.asarray(hour, dtype=np.float32)
    angle = (2.0 * np.pi) * (hour / 24.0)
    hour_sin = np.sin(angle).astype(np.float32)
    hour_cos = np.cos(angle).astype(np.float32)
    dow = dt_index.dayofweek.to_numpy()
    dow_oh = np.eye(7, dtype=np.float32)[dow]
    return np.concatenate([hour_sin[:, None], hour_cos[:, None], dow_oh], axis=1).astype(np.float32)


@dataclass(frozen=True)
class SensorStandardizer:
    mean: np.ndarray  # (S,)
    std: np.ndarray   # (S,)

    def transform(self, x: np.ndarray) -> np.ndarray:
        return (x - self.mean) / self.std

    def inverse_transform(self, x: np.ndarray) -> np.ndarray:
        return (x * self.std) + self.mean


def compute_sensor_stats_from_normal(normal_root: str | Path, sensor_ids: Optional[Sequence[str]] = None,
                                     use_gt: bool = True, max_scenes: Optional[int] = None) -> SensorStandardizer:
    """Per-sensor mean / std over all rows of the no-leak scenes (datasets.py:72-111):
    float64 sums, var = E[x^2] - mean^2 clipped at 1e-12, std floored at 1e-3."""
    normal_root = Path(normal_root)
    manifest = _filter_ok(_read_manifest_jsonl(normal_root / "manifest.jsonl"))
    if max_scenes is not None:
        manifest = manifest[:max_scenes]
    fname = "sensors_gt.csv" if use_gt else "sensors.csv"
    if sensor_ids is None:
        df0 = pd.read_csv(normal_root / manifest[0]["window_id"] / fname, index_col=0, parse_dates=True)
        sensor_ids = list(df0.columns)
    s = len(sensor_ids)
    sum_ = np.zeros((s,), dtype=np.float64)
    sumsq = np.zeros((s,), dtype=np.float64)
    count = 0
    for row in manifest:
        df = pd.read_csv(normal_root / row["window_id"] / fname, index_col=0, parse_dates=True)
        x = _ensure_sensor_order(df, sensor_ids).to_numpy(dtype=np.float64)
        sum_ += x.sum(axis=0)
        sumsq += (x * x).sum(axis=0)
        count += x.shape[0]
    mean = (sum_ / max(count, 1)).astype(np.float32)
    var = (sumsq / max(count, 1) - mean.astype(np.float64) ** 2).clip(min=1e-12)
    std = np.maximum(np.sqrt(var).astype(np.float32), 1e-3).astype(np.float32)
    return SensorStandardizer(mean=mean, std=std)


# ------------------------------------------------------------------- scenario store
@dataclass
class _LoadedSeries:
    noisy: np.ndarray            # (T, S) float32
    gt: np.ndarray               # (T, S) float32
    time_feat: np.ndarray        # (T, 9) float32
    timestamps: pd.DatetimeIndex
    sensor_ids: List[str]


class ScenarioStore:
    """Lazy CSV loader with an LRU cache of float32 arrays (datasets.py:126-194)."""

    def __init__(self, root: Path, sensor_ids: Optional[Sequence[str]] = None,
                 standardizer: Optional[SensorStandardizer] = None, cache_size: int = 32) -> None:
        self.root = Path(root)
        self.sensor_ids = list(sensor_ids) if sensor_ids is not None else None
        self.standardizer = standardizer
        self.cache_size = int(cache_size)
        self._cache: Dict[str, _LoadedSeries] = {}
        self._lru: List[str] = []

    def _cache_put(self, key: str, val: _LoadedSeries) -> None:
        if key in self._cache:
            return
        self._cache[key] = val
        self._lru.append(key)
        if len(self._lru) > self.cache_size:
            self._cache.pop(self._lru.pop(0), None)

    def get(self, scene_id: str) -> _LoadedSeries:
        if scene_id in self._cache:
            try:
                self._lru.remove(scene_id)
            except ValueError:
                pass
            self._lru.append(scene_id)
            return self._cache[scene_id]
        df_noisy = pd.read_csv(self.root / scene_id / "sensors.csv", index_col=0, parse_dates=True)
        df_gt = pd.read_csv(self.root / scene_id / "sensors_gt.csv", index_col=0, parse_dates=True)
        if self.sensor_ids is None:
            self.sensor_ids = list(df_noisy.columns)
        df_noisy = _ensure_sensor_order(df_noisy, self.sensor_ids)
        df_gt = _ensure_sensor_order(df_gt, self.sensor_ids)
        ts = df_noisy.index
        if not ts.equals(df_gt.index):
            raise ValueError(f"Timestamps mismatch between sensors.csv and sensors_gt.csv in {scene_id}")
        x_noisy = df_noisy.to_numpy(dtype=np.float32)
        x_gt = df_gt.to_numpy(dtype=np.float32)
        if self.standardizer is not None:
            x_noisy = self.standardizer.transform(x_noisy)
            x_gt = self.standardizer.transform(x_gt)
        loaded = _LoadedSeries(noisy=x_noisy, gt=x_gt, time_feat=make_time_features(ts), timestamps=ts,
                               sensor_ids=list(self.sensor_ids))
        self._cache_put(scene_id, loaded)
        return loaded


# ------------------------------------------------------------ predictor dataset
class NormalPredictorDataset(Dataset):
    """(x, x_time, y) windows from no-leak scenes (datasets.py:200-257): per index,
    rng = default_rng(seed + idx); scene = rng.choice(scene_ids);
    t = rng.integers(l_in - 1, T - h - 1 + 1); x = noisy[t-l_in+1 .. t], y = gt[t+1 .. t+h]."""

    def __init__(self, normal_root: str | Path, l_in_steps: int = 36, horizon_steps: int = 1,
                 steps_per_epoch: int = 50000, seed: int = 42, sensor_ids: Optional[Sequence[str]] = None,
                 standardizer: Optional[SensorStandardizer] = None, cache_size: int = 32) -> None:
        super().__init__()
        self.normal_root = Path(normal_root)
        self.l_in = int(l_in_steps)
        self.h = int(horizon_steps)
        self.steps_per_epoch = int(steps_per_epoch)
        self.seed = int(seed)
        manifest = _filter_ok(_read_manifest_jsonl(self.normal_root / "manifest.jsonl"))
        self.scene_ids = [r["window_id"] for r in manifest]
        self.store = ScenarioStore(self.normal_root, sensor_ids=sensor_ids, standardizer=standardizer,
                                   cache_size=cache_size)
        self._sensor_ids = self.store.get(self.scene_ids[0]).sensor_ids
        self._T: Dict[str, int] = {}

    def get_sensor_node_ids(self):
        return self._sensor_ids

    def __len__(self) -> int:
        return self.steps_per_epoch

    def draw(self, idx: int) -> tuple:
        """(scene_id, t) of sample idx — the reference's RNG draws, nothing loaded."""
        rng = np.random.default_rng(self.seed + idx)
        scene_id = rng.choice(self.scene_ids)
        T = self._scene_len(scene_id)
        t_min, t_max = self.l_in - 1, T - self.h - 1
        if t_max < t_min:
            raise ValueError(f"Scene too short for l_in={self.l_in}, h={self.h}: {scene_id} (T={T})")
        return str(scene_id), int(rng.integers(t_min, t_max + 1))

    def _scene_len(self, scene_id: str) -> int:
        if scene_id not in self._T:  # a scene's length is fixed: read it once
            self._T[scene_id] = self.store.get(scene_id).noisy.shape[0]
        return self._T[scene_id]

    def __getitem__(self, idx: int) -> Dict[str, Any]:
        scene_id, t = self.draw(idx)
        data = self.store.get(scene_id)
        return {
            "scene_id": scene_id,
            "t": str(data.timestamps[t]),
            "x": torch.from_numpy(data.noisy[t - self.l_in + 1: t + 1]),
            "x_time": torch.from_numpy(data.time_feat[t - self.l_in + 1: t + 1]),
            "y": torch.from_numpy(data.gt[t + 1: t + 1 + self.h]),
        }


# ------------------------------------------------------------- detector dataset
@dataclass(frozen=True)
class DetectorSamplingConfig:
    """datasets.py:263-279."""
    p_early: float = 0.30
    p_late: float = 0.30
    p_pre: float = 0.20
    p_noleak: float = 0.20
    early_hours: float = 6.0
    pre_hours: float = 2.0
    q0: float = 1e-6

    def validate(self) -> None:
        s = self.p_early + self.p_late + self.p_pre + self.p_noleak
        if abs(s - 1.0) > 1e-6:
            raise ValueError(f"Bucket probs must sum to 1.0, got {s}")


class AbruptLeakDetectorDataset(Dataset):
    """(L_pred + L_det)-step segments ending at t with a softmax label over P+1 classes
    (datasets.py:282-543).  Buckets: early [tau, tau+6h) and late (>= tau+6h) positives,
    pre-leak [tau-2h, tau) and no-leak negatives; tau = first step with leak flow > q0."""

    def __init__(self, leak_root: str | Path, l_pred_steps: int = 36, l_det_steps: int = 36,
                 steps_per_epoch: int = 80000, seed: int = 123, sensor_ids: Optional[Sequence[str]] = None,
                 standardizer: Optional[SensorStandardizer] = None, step_min: int = 5,
                 sampling: DetectorSamplingConfig = DetectorSamplingConfig(), cache_size: int = 32,
                 include_leak_types: tuple = ("abrupt",)) -> None:
        super().__init__()
        self.leak_root = Path(leak_root)
        self.l_pred = int(l_pred_steps)
        self.l_det = int(l_det_steps)
        self.seg_len = self.l_pred + self.l_det
        self.steps_per_epoch = int(steps_per_epoch)
        self.seed = int(seed)
        self.include_leak_types = tuple(include_leak_types)
        sampling.validate()
        self.sampling = sampling
        self.cfg = sampling

        manifest = _filter_ok(_read_manifest_jsonl(self.leak_root / "manifest.jsonl"))
        leak_rows, noleak_rows = [], []
        for r in manifest:  # datasets.py:325-336
            kind = str(r.get("kind", "")).lower()
            leak_type = str(r.get("leak_type", None)).lower()
            pipe_id = r.get("pipe_id", None)
            if kind == "leak" and leak_type is not None and pipe_id is not None:
                if leak_type in self.include_leak_types:
                    leak_rows.append(r)
            else:
                noleak_rows.append(r)
        self.leak_scene_ids = [r["scenario_id"] for r in leak_rows]
        self.noleak_scene_ids = [r["scenario_id"] for r in noleak_rows]
        pipe_ids = sorted({str(r["pipe_id"]) for r in leak_rows})
        self.pipe_ids_in_order = pipe_ids
        self.pipe_to_idx = {pid: i for i, pid in enumerate(pipe_ids)}
        self.num_pipes = len(pipe_ids)
        self.no_leak_class = self.num_pipes
        self.store = ScenarioStore(self.leak_root, sensor_ids=sensor_ids, standardizer=standardizer,
                                   cache_size=cache_size)

        self._bucket_times: Dict[str, Dict[str, np.ndarray]] = {}
        self._pipe_idx: Dict[str, int] = {}
        self._T: Dict[str, int] = {}
        self.step_min = step_min
        steps_per_hour = 60.0 / self.step_min
        early_steps = int(round(self.sampling.early_hours * steps_per_hour))
        pre_steps = int(round(self.sampling.pre_hours * steps_per_hour))
        if early_steps <= 0 or pre_steps <= 0:
            raise ValueError(f"Unreasonable values of early_steps ({early_steps}) or pre_steps ({pre_steps}).")
        empty = np.array([], dtype=np.int64)
        t_min = self.seg_len - 1
        for r in leak_rows:  # datasets.py:369-423
            sid, pid = r["scenario_id"], str(r["pipe_id"])
            self._pipe_idx[sid] = self.pipe_to_idx[pid]
            T = self.store.get(sid).noisy.shape[0]
            self._T[sid] = T
            df_q = pd.read_csv(self.leak_root / sid / "leak_flow_m3h.csv", index_col=0, parse_dates=True)
            q = df_q[pid].to_numpy(dtype=np.float32)
            if len(q) != T:
                raise ValueError(f"Length mismatch leak_flow vs sensors in {sid}: {len(q)} vs {T}")
            active = q > float(self.sampling.q0)
            tau = int(np.argmax(active)) if np.any(active) else T
            t_max = T - 1
            if t_max < t_min:
                self._bucket_times[sid] = {"early": empty, "late": empty, "pre": empty}
                continue

            def _range_to_idx(a: int, b: int) -> np.ndarray:
                a2, b2 = max(a, t_min), min(b, t_max + 1)
                return np.arange(a2, b2, dtype=np.int64) if b2 > a2 else empty

            self._bucket_times[sid] = {
                "early": _range_to_idx(tau, min(tau + early_steps, T)),
                "late": _range_to_idx(min(tau + early_steps, T), T),
                "pre": _range_to_idx(max(tau - pre_steps, 0), tau),
            }
        self._noleak_times: Dict[str, np.ndarray] = {}
        for sid in self.noleak_scene_ids:  # datasets.py:426-435
            T = self.store.get(sid).noisy.shape[0]
            self._T[sid] = T
            self._noleak_times[sid] = np.arange(t_min, T, dtype=np.int64) if T - 1 >= t_min else empty
        self.leak_scene_ids = [s for s in self.leak_scene_ids
                               if sum(v.size for v in self._bucket_times.get(s, {}).values()) > 0]
        self.noleak_scene_ids = [s for s in self.noleak_scene_ids if self._noleak_times[s].size > 0]
        if not self.leak_scene_ids:
            raise RuntimeError("No usable abrupt leak scenarios found. Check manifest filters and scene lengths.")
        if not self.noleak_scene_ids:
            raise RuntimeError("No usable no-leak scenarios found. Check manifest or scene lengths.")
        s = self.sampling
        self._cum = np.array([s.p_early, s.p_early + s.p_late, s.p_early + s.p_late + s.p_pre, 1.0],
                             dtype=np.float64)
        self._sensor_ids = self.store.get(self.leak_scene_ids[0]).sensor_ids
        self._idx_to_pipe = {j: pid for pid, j in self.pipe_to_idx.items()}

    def get_sensor_node_ids(self):
        return self._sensor_ids

    def get_pipe_ids_in_order(self):
        return list(self.pipe_ids_in_order)

    def get_pipe_to_idx(self):
        return dict(self.pipe_to_idx)

    def __len__(self) -> int:
        return self.steps_per_epoch

    def _choose_bucket(self, rng: np.random.Generator) -> str:
        u = float(rng.random())
        if u < self._cum[0]:
            return "early"
        if u < self._cum[1]:
            return "late"
        if u < self._cum[2]:
            return "pre"
        return "noleak"

    def draw(self, idx: int) -> Dict[str, Any]:
        """The sampling decisions of sample idx (datasets.py:483-517): same RNG calls in
        the same order as the reference, no array access."""
        rng = np.random.default_rng(self.seed + idx)
        for _ in range(10):
            bucket = self._choose_bucket(rng)
            if bucket == "noleak":
                sid = rng.choice(self.noleak_scene_ids)
                times = self._noleak_times[sid]
                if times.size == 0:
                    continue
                t = int(rng.choice(times))
                label, pipe_idx, pipe_id = self.no_leak_class, -1, None
            else:
                sid = rng.choice(self.leak_scene_ids)
                times = self._bucket_times[sid][bucket]
                if times.size == 0:
                    continue
                t = int(rng.choice(times))
                pipe_idx = int(self._pipe_idx[sid])
                pipe_id = self._idx_to_pipe.get(pipe_idx)
                label = pipe_idx if bucket in ("early", "late") else self.no_leak_class
            return {"scenario_id": str(sid), "bucket": bucket, "t": t, "label": int(label),
                    "pipe_index": int(pipe_idx), "pipe_id": str(pipe_id) if pipe_id is not None else "NOLEAK"}
        raise RuntimeError("Failed to sample a valid (scenario, time) after multiple attempts. Check data lengths/buckets.")

    def _sample_dict(self, d: Dict[str, Any], data: _LoadedSeries) -> Dict[str, Any]:
        t = d["t"]
        return {
            "scenario_id": d["scenario_id"], "bucket": d["bucket"], "t": str(data.timestamps[t]),
            "label": d["label"], "pipe_index": d["pipe_index"], "pipe_id": d["pipe_id"],
            "num_classes": int(self.num_pipes + 1), "l_pred": int(self.l_pred), "l_det": int(self.l_det),
        }

    def __getitem__(self, idx: int) -> Dict[str, Any]:
        d = self.draw(idx)
        data = self.store.get(d["scenario_id"])
        t = d["t"]
        out = self._sample_dict(d, data)
        out["noisy_seg"] = torch.from_numpy(data.noisy[t - self.seg_len + 1: t + 1])
        out["time_seg"] = torch.from_numpy(data.time_feat[t - self.seg_len + 1: t + 1])
        return out


# ------------------------------------------------------------- device batch path
class _DeviceBank:
    """All scenes of a store as (scenes, T_max, C) device tensors + host timestamps."""

    def __init__(self, store: ScenarioStore, scene_ids: Sequence[str], device: torch.device,
                 with_gt: bool = False) -> None:
        self.index = {sid: i for i, sid in enumerate(scene_ids)}
        series = [store.get(sid) for sid in scene_ids]
        T = max(s.noisy.shape[0] for s in series)
        S = series[0].noisy.shape[1]

        def pack(arrs, C):
            buf = np.zeros((len(arrs), T, C), dtype=np.float32)
            for i, a in enumerate(arrs):
                buf[i, : a.shape[0]] = a
            return torch.from_numpy(buf).to(device)

        self.noisy = pack([s.noisy for s in series], S)
        self.time_feat = pack([s.time_feat for s in series], 9)
        self.gt = pack([s.gt for s in series], S) if with_gt else None
        self.timestamps = [s.timestamps for s in series]
        self.device = device

    def windows(self, src: torch.Tensor, scene: List[int], first: List[int], length: int) -> torch.Tensor:
        """src[scene[i], first[i] : first[i] + length] for every i, as one (n, length, C) gather."""
        sc = torch.tensor(scene, dtype=torch.long, device=self.device).view(-1, 1)
        tt = torch.tensor(first, dtype=torch.long, device=self.device).view(-1, 1) + torch.arange(
            length, device=self.device).view(1, -1)
        return src[sc, tt]


class DeviceBatchLoader:
    """Batches of ``ds`` (AbruptLeakDetectorDataset or NormalPredictorDataset) in index
    order, windows gathered on ``device`` from HBM-resident scenes.  Equivalent to
    DataLoader(ds, batch_size, shuffle=False) + .to(device) of the tensor fields."""

    def __init__(self, ds, batch_size: int, device: torch.device, shard: Tuple[int, int] = (0, 1)) -> None:
        self.ds = ds
        self.batch_size = int(batch_size)
        self.device = torch.device(device)
        self.rank, self.world = int(shard[0]), int(shard[1])  # data parallel: this rank's slice of each batch
        if isinstance(ds, AbruptLeakDetectorDataset):
            ids = list(dict.fromkeys(list(ds.leak_scene_ids) + list(ds.noleak_scene_ids)))
            self.bank = _DeviceBank(ds.store, ids, self.device)
        elif isinstance(ds, NormalPredictorDataset):
            self.bank = _DeviceBank(ds.store, list(ds.scene_ids), self.device, with_gt=True)
        else:
            raise TypeError(f"unsupported dataset {type(ds).__name__}")

    def __len__(self) -> int:
        return (len(self.ds) + self.batch_size - 1) // self.batch_size

    def _detector_batch(self, idxs: range) -> Dict[str, Any]:
        ds, bank = self.ds, self.bank
        draws = [ds.draw(i) for i in idxs]
        scene = [bank.index[d["scenario_id"]] for d in draws]
        first = [d["t"] - ds.seg_len + 1 for d in draws]
        n = len(draws)
        return {
            "scenario_id": [d["scenario_id"] for d in draws],
            "bucket": [d["bucket"] for d in draws],
            "t": [str(bank.timestamps[s][d["t"]]) for s, d in zip(scene, draws)],
            "noisy_seg": bank.windows(bank.noisy, scene, first, ds.seg_len),
            "time_seg": bank.windows(bank.time_feat, scene, first, ds.seg_len),
            "label": torch.tensor([d["label"] for d in draws], dtype=torch.long, device=self.device),
            "pipe_index": torch.tensor([d["pipe_index"] for d in draws], dtype=torch.long, device=self.device),
            "pipe_id": [d["pipe_id"] for d in draws],
            "num_classes": torch.full((n,), ds.num_pipes + 1, dtype=torch.long, device=self.device),
            "l_pred": torch.full((n,), ds.l_pred, dtype=torch.long, device=self.device),
            "l_det": torch.full((n,), ds.l_det, dtype=torch.long, device=self.device),
        }

    def _predictor_batch(self, idxs: range) -> Dict[str, Any]:
        ds, bank = self.ds, self.bank
        draws = [ds.draw(i) for i in idxs]
        scene = [bank.index[s] for s, _ in draws]
        first = [t - ds.l_in + 1 for _, t in draws]
        return {
            "scene_id": [s for s, _ in draws],
            "t": [str(bank.timestamps[sc][t]) for sc, (_, t) in zip(scene, draws)],
            "x": bank.windows(bank.noisy, scene, first, ds.l_in),
            "x_time": bank.windows(bank.time_feat, scene, first, ds.l_in),
            "y": bank.windows(bank.gt, scene, [t + 1 for _, t in draws], ds.h),
        }

    def __iter__(self) -> Iterator[Dict[str, Any]]:
        make = self._detector_batch if isinstance(self.ds, AbruptLeakDetectorDataset) else self._predictor_batch
        for b0 in range(0, len(self.ds), self.batch_size):
            yield make(shard_slice(range(b0, min(b0 + self.batch_size, len(self.ds))), self.rank, self.world))


def shard_slice(idxs: range, rank: int, world: int) -> range:
    """Contiguous slice `rank` of `world` of one global batch's sample indices (sizes
    differ by at most one on a ragged last batch).  Samples are seeded by seed + index
    (datasets.py:236,490), so the union over ranks is the single-process batch."""
    n = len(idxs)
    lo = idxs.start + (n * rank) // world
    hi = idxs.start + (n * (rank + 1)) // world
    return range(lo, hi)


class ShardBatchSampler:
    """batch_sampler for torch's DataLoader: this rank's shard_slice of every global batch."""

    def __init__(self, n: int, batch_size: int, rank: int, world: int) -> None:
        self.n, self.bs, self.rank, self.world = int(n), int(batch_size), int(rank), int(world)

    def __len__(self) -> int:
        return (self.n + self.bs - 1) // self.bs

    def __iter__(self):
        for b0 in range(0, self.n, self.bs):
            yield list(shard_slice(range(b0, min(b0 + self.bs, self.n)), self.rank, self.world))
