"""Train + evaluate the normal-state predictor on no-leak data (reference
models/train_predictor.py): same CLI flags (:95-109), split (:46-56), loop order
(:196-222) and checkpoint schema (:236-244).

  python -m models.train_predictor --normal_root DATA --out_dir OUT [--arch tcn|gru] ...

Differences that do not change results: batches come from datasets.DeviceBatchLoader
(scenes resident in HBM, one gather per batch; --loader torch restores the
DataLoader path), and checkpoints store the standardizer as plain lists of floats: they
load with torch.load(weights_only=True), and the reference's loaders
(train_detector.py / event_evaluator.py: np.asarray(std_mean, dtype=np.float32) after a
load with map_location=cuda) accept them on any device.
"""
from __future__ import annotations

import argparse
import json
import math
import random
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from .datasets import DeviceBatchLoader, NormalPredictorDataset, ShardBatchSampler, compute_sensor_stats_from_normal
from .predictor import NormalPredictorGRU, NormalPredictorTCN
from .utils import now


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def pick_device(device: str) -> torch.device:
    if device == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


def split_ids(ids: List[str], seed: int, ratios=(0.8, 0.1, 0.1)) -> Tuple[List[str], List[str], List[str]]:
    """train_predictor.py:46-56."""
    assert abs(sum(ratios) - 1.0) < 1e-6
    rng = random.Random(seed)
    ids = list(ids)
    rng.shuffle(ids)
    n = len(ids)
    n_train, n_val = int(n * ratios[0]), int(n * ratios[1])
    return ids[:n_train], ids[n_train:n_train + n_val], ids[n_train + n_val:]


def make_loader(ds, batch_size: int, device: torch.device, kind: str, num_workers: int = 0,
                shard: Tuple[int, int] = (0, 1)):
    """Batches of `batch_size` samples in index order; with shard = (rank, world) each rank
    gets its contiguous slice of every global batch (data parallelism)."""
    if kind == "device" and device.type == "cuda":
        return DeviceBatchLoader(ds, batch_size, device, shard=shard)
    if shard[1] > 1:
        return DataLoader(ds, batch_sampler=ShardBatchSampler(len(ds), batch_size, *shard), num_workers=num_workers,
                          pin_memory=(device.type == "cuda"))
    return DataLoader(ds, batch_size=batch_size, num_workers=num_workers, pin_memory=(device.type == "cuda"))


@torch.no_grad()
def evaluate_predictor(model: nn.Module, loader, device: torch.device, standardizer_mean: torch.Tensor,
                       standardizer_std: torch.Tensor) -> Dict[str, float]:
    """MAE / RMSE in original units (train_predictor.py:58-92), sums kept on the device."""
    model.eval()
    mae_sum = torch.zeros((), dtype=torch.float64, device=device)
    mse_sum = torch.zeros((), dtype=torch.float64, device=device)
    n = 0
    for batch in loader:
        x, x_time = batch["x"].to(device), batch["x_time"].to(device)
        y = batch["y"].to(device)[:, 0, :]
        y_hat = model(x, x_time)
        err = (y_hat * standardizer_std + standardizer_mean) - (y * standardizer_std + standardizer_mean)
        mae_sum += err.abs().sum().double()
        mse_sum += (err * err).sum().double()
        n += y.numel()
    return {"mae": float(mae_sum.item() / max(n, 1)), "rmse": float(math.sqrt(mse_sum.item() / max(n, 1)))}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--normal_root", type=str, required=True, help="Path to normal dataset root")
    ap.add_argument("--out_dir", type=str, required=True, help="Output directory for checkpoints/logs")
    ap.add_argument("--arch", type=str, default="tcn", choices=["tcn", "gru"])
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--steps_per_epoch", type=int, default=100000)
    ap.add_argument("--val_steps", type=int, default=8000)
    ap.add_argument("--test_steps", type=int, default=8000)
    ap.add_argument("--batch_size", type=int, default=256)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--weight_decay", type=float, default=1e-4)
    ap.add_argument("--grad_clip", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--device", type=str, default="auto", help="auto|cuda|cpu|cuda:0 ...")
    ap.add_argument("--num_workers", type=int, default=0)
    ap.add_argument("--log_every", type=int, default=50)
    ap.add_argument("--loader", type=str, default="device", choices=["device", "torch"])
    ap.add_argument("--profile", type=int, default=0,
                    help="torch.profiler over this many training steps (after one warm-up step): "
                         "<out_dir>/predictor_trace.json + predictor_ops.txt (models/profiling.py)")
    args = ap.parse_args(argv)

    out_dir = Path(args.out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    set_seed(args.seed)
    device = pick_device(args.device)
    print(f"{now()} [predictor] device={device} seed={args.seed}")
    print(f"{now()} [predictor] loading normal data from: {args.normal_root}")

    stdzr = compute_sensor_stats_from_normal(Path(args.normal_root))
    mean = torch.tensor(stdzr.mean, dtype=torch.float32, device=device)
    std = torch.tensor(stdzr.std, dtype=torch.float32, device=device)
    base_ds = NormalPredictorDataset(normal_root=args.normal_root, steps_per_epoch=1, seed=args.seed,
                                     standardizer=stdzr)
    sensor_ids = base_ds.get_sensor_node_ids()
    train_ids, val_ids, test_ids = split_ids(base_ds.scene_ids, args.seed, ratios=(0.8, 0.1, 0.1))
    print(f"{now()} [predictor] scenes: total={len(base_ds.scene_ids)} train={len(train_ids)} "
          f"val={len(val_ids)} test={len(test_ids)}")

    def mk(steps, seed, ids):
        ds = NormalPredictorDataset(normal_root=args.normal_root, l_in_steps=36, horizon_steps=1,
                                    steps_per_epoch=steps, seed=seed, sensor_ids=sensor_ids, standardizer=stdzr,
                                    cache_size=1024)
        ds.scene_ids = ids
        return make_loader(ds, args.batch_size, device, args.loader, args.num_workers)

    train_loader = mk(args.steps_per_epoch, args.seed, train_ids)
    val_loader = mk(args.val_steps, args.seed + 1, val_ids)
    test_loader = mk(args.test_steps, args.seed + 2, test_ids)

    S = len(sensor_ids)
    model = (NormalPredictorTCN(num_sensors=S, time_dim=9) if args.arch == "tcn"
             else NormalPredictorGRU(num_sensors=S, time_dim=9)).to(device)
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=args.weight_decay,
                            fused=(device.type == "cuda"))
    loss_fn = nn.MSELoss()
    best_rmse = float("inf")
    best_path, last_path = out_dir / "predictor_best.ckpt", out_dir / "predictor_last.ckpt"
    meta = {"arch": args.arch, "num_sensors": S, "time_dim": 9, "l_in_steps": 36, "horizon_steps": 1,
            "sensor_ids": sensor_ids, "standardizer": {"mean": stdzr.mean.tolist(), "std": stdzr.std.tolist()},
            "split": {"train_ids": train_ids, "val_ids": val_ids, "test_ids": test_ids}}
    (out_dir / "predictor_meta.json").write_text(json.dumps(meta, indent=2, ensure_ascii=False), encoding="utf-8")

    print(f"{now()} [predictor] start training: epochs={args.epochs}, steps/epoch={args.steps_per_epoch}, "
          f"batch={args.batch_size}")
    from .profiling import StepProfiler
    prof = StepProfiler(out_dir, "predictor", args.profile, device)
    for epoch in range(1, args.epochs + 1):
        model.train()
        running = torch.zeros((), dtype=torch.float64, device=device)
        seen = 0
        for it, batch in enumerate(train_loader, start=1):
            x, x_time = batch["x"].to(device), batch["x_time"].to(device)
            y = batch["y"].to(device)[:, 0, :]
            loss = loss_fn(model(x, x_time), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            if args.grad_clip and args.grad_clip > 0:
                torch.nn.utils.clip_grad_norm_(model.parameters(), args.grad_clip)
            opt.step()
            running += loss.detach().double() * x.size(0)
            seen += x.size(0)
            prof.step()
            if (it % args.log_every) == 0:
                print(f"{now()} [predictor][epoch {epoch:02d}] step {it:05d}/{len(train_loader):05d} "
                      f"loss={running.item() / max(seen, 1):.6f}")
        train_loss = running.item() / max(seen, 1)
        val_metrics = evaluate_predictor(model, val_loader, device, mean, std)
        print(f"{now()} [predictor][epoch {epoch:02d}] done. train_loss={train_loss:.6f} "
              f"val_mae={val_metrics['mae']:.4f} val_rmse={val_metrics['rmse']:.4f}")
        ckpt = {"epoch": epoch, "arch": args.arch, "model_state": model.state_dict(),
                "standardizer_mean": [float(v) for v in stdzr.mean],
                "standardizer_std": [float(v) for v in stdzr.std],
                "sensor_ids": sensor_ids, "args": vars(args)}
        torch.save(ckpt, last_path)
        if val_metrics["rmse"] < best_rmse:
            best_rmse = val_metrics["rmse"]
            torch.save(ckpt, best_path)
            print(f"{now()} [predictor] new best: rmse={best_rmse:.4f} -> {best_path.name}")

    prof.close()
    best_ckpt = torch.load(best_path, map_location=device, weights_only=True)
    model.load_state_dict(best_ckpt["model_state"])
    test_metrics = evaluate_predictor(model, test_loader, device, mean, std)
    print(f"{now()} [predictor] TEST: mae={test_metrics['mae']:.4f} rmse={test_metrics['rmse']:.4f}")
    print(f"{now()} [predictor] saved: {best_path.name}, {last_path.name}, meta.json")


if __name__ == "__main__":
    main()
