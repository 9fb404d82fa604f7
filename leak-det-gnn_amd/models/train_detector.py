"""Train + evaluate the leak detector on abrupt single-pipe leak scenarios (+ no-leak)
(reference models/train_detector.py): same CLI flags (:133-155), scenario splits
(:41-109), frozen-predictor loading (:112-128), loop order (:296-317), evaluation and
checkpoint schema (:346-353).

  python -m models.train_detector --leak_root DATA --inp_path L-TOWN-A.inp \\
         --predictor_ckpt OUT/predictor_best.ckpt --out_dir OUT [...]

The detector is this package's LeakDetector (HIP GRU / GCN / heads kernels); batches
come from datasets.DeviceBatchLoader (--loader torch restores the DataLoader path);
on the GPU the loss is models.loss.CrossEntropyLoss (two launches) and clip_grad_norm_ +
AdamW run as models.optim.ClipAdamW (two launches, the same arithmetic as torch's
clip then AdamW step); on the CPU they are torch's.  Checkpoints load with
torch.load(weights_only=True).

Data parallel (not in the reference, which is single-device): launched under torchrun
(one process per GPU; RANK / LOCAL_RANK / WORLD_SIZE from the environment),
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m models.train_detector ... --batch_size 512
every rank takes its contiguous slice of each GLOBAL batch of --batch_size samples (the
samples are seeded by seed + index, datasets.py:236,490, so the global batch is the
single-process batch at any world size), scales its mean loss by its share of the batch,
and one gradient all-reduce (models/ddp.py: RCCL over xGMI, gloo on CPU) averages the
gradients before clipping, so every rank takes the single-process step.  Rank 0
evaluates, logs and writes the checkpoints.

On the GPU every full-size batch's step is one captured HIP graph (--capture, default
auto: models/graph_step.CapturedTrainStep, the batch copied into its static inputs; at
world > 1 the heads' gradient all-reduce overlaps the trunk backward); a short tail
batch runs eagerly.  --perf_log writes windows/s per log interval as JSONL.
"""
from __future__ import annotations

import argparse
import builtins
import json
import os
import random
from collections import defaultdict
from dataclasses import asdict
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn as nn

from .datasets import AbruptLeakDetectorDataset, SensorStandardizer
from .ddp import GradAllReduce, dist_env, init_distributed, reseed_rank
from .detector import LeakDetector
from .loss import CrossEntropyLoss
from .optim import ClipAdamW
from .predictor import NormalPredictorGRU, NormalPredictorTCN
from .train_predictor import make_loader, pick_device, set_seed
from .utils import build_residual_sequence_from_segment, now
from .window_evaluator import DetectorEvaluator


class PerfLog:
    """JSONL perf log of the training loop: one line per --log_every interval with
    the global windows trained, wall seconds and windows/s since the previous line.  Written
    at the loss-logging points, which already synchronise (the loss is read back)."""

    def __init__(self, path, world: int):
        import time
        self.path, self.world, self._time = path, world, time.perf_counter
        self.t0, self.n = self._time(), 0
        if path is not None:
            Path(path).write_text("", encoding="utf-8")

    def add(self, n_local: int) -> None:
        self.n += n_local * self.world

    def flush(self, epoch: int, step: int, loss: float, mode: str) -> None:
        t = self._time()
        if self.path is not None:
            dt = max(t - self.t0, 1e-9)
            rec = {"epoch": epoch, "step": step, "windows": self.n, "seconds": round(dt, 6),
                   "windows_per_s": round(self.n / dt, 2), "loss": loss, "mode": mode, "world": self.world}
            with open(self.path, "a", encoding="utf-8") as f:
                f.write(json.dumps(rec) + "\n")
        self.t0, self.n = t, 0


def scenario_to_pipe_id(sid: str) -> str:
    """train_detector.py:41-45: '001927_p534_abrupt_r1' -> 'p534'."""
    parts = sid.split("_")
    if len(parts) < 2:
        raise ValueError(f"Bad scenario_id format: {sid}")
    return parts[1]


def split_leak_scenids(leak_scene_ids: List[str], seed: int, ratio=(0.8, 0.1, 0.1)) -> Tuple[List[str], ...]:
    """train_detector.py:47-96: every pipe keeps one scene in train; val / test are
    filled round-robin across pipes from the rest; random.Random(seed) throughout."""
    rng = random.Random(seed)
    pipe2scenes = defaultdict(list)
    for sid in leak_scene_ids:
        pipe2scenes[scenario_to_pipe_id(sid)].append(sid)
    train_ids: List[str] = []
    pipe2rest = {}
    for pid, scenes in pipe2scenes.items():
        scenes = list(scenes)
        rng.shuffle(scenes)
        train_ids.append(scenes[0])
        pipe2rest[pid] = scenes[1:]
    rest_total = sum(len(v) for v in pipe2rest.values())
    r_train, r_val, r_test = ratio
    denom = float(r_train + r_val + r_test)
    val_target = int(round(rest_total * (r_val / denom)))
    test_target = int(round(rest_total * (r_test / denom)))
    pipe_keys = list(pipe2rest.keys())
    rng.shuffle(pipe_keys)

    def pop_one_round_robin(target_n: int) -> List[str]:
        out: List[str] = []
        while len(out) < target_n:
            progressed = False
            for pid in pipe_keys:
                if len(out) >= target_n:
                    break
                lst = pipe2rest[pid]
                if lst:
                    out.append(lst.pop())
                    progressed = True
            if not progressed:
                break
        return out

    val_ids = pop_one_round_robin(val_target)
    test_ids = pop_one_round_robin(test_target)
    for pid in pipe_keys:
        train_ids.extend(pipe2rest[pid])
    rng.shuffle(train_ids)
    rng.shuffle(val_ids)
    rng.shuffle(test_ids)
    return train_ids, val_ids, test_ids


def split_normal_scenids(ids: List[str], seed: int, ratios=(0.8, 0.1, 0.1)) -> Tuple[List[str], ...]:
    """train_detector.py:98-109."""
    assert abs(sum(ratios) - 1.0) < 1e-6
    rng = random.Random(seed)
    ids = list(ids)
    rng.shuffle(ids)
    n = len(ids)
    n_train, n_val = int(n * ratios[0]), int(n * ratios[1])
    return ids[:n_train], ids[n_train:n_train + n_val], ids[n_train + n_val:]


def _load_ckpt(path: str | Path, device: torch.device) -> Dict:
    """Checkpoints written by this package load with weights_only=True.  One written by
    another trainer with numpy arrays inside needs LEAKGNN_TRUST_CKPT=1 (explicit opt-in
    to a full unpickle of a file the user vouches for)."""
    try:
        return torch.load(path, map_location=device, weights_only=True)
    except Exception:
        if os.environ.get("LEAKGNN_TRUST_CKPT") == "1":
            return torch.load(path, map_location=device, weights_only=False)
        raise


def load_predictor(ckpt_path: str | Path, device: torch.device) -> Tuple[nn.Module, Dict]:
    """Frozen predictor (train_detector.py:112-128)."""
    ckpt = _load_ckpt(ckpt_path, device)
    S = len(ckpt["sensor_ids"])
    model = NormalPredictorGRU(num_sensors=S, time_dim=9) if ckpt.get("arch", "tcn") == "gru" else \
        NormalPredictorTCN(num_sensors=S, time_dim=9)
    model.load_state_dict(ckpt["model_state"])
    model.to(device)
    model.eval()
    for p in model.parameters():
        p.requires_grad_(False)
    return model, ckpt


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--leak_root", type=str, required=True, help="Path to leak dataset root")
    ap.add_argument("--inp_path", type=str, required=True, help="Path to EPANET .inp file")
    ap.add_argument("--predictor_ckpt", type=str, required=True, help="Path to trained predictor checkpoint")
    ap.add_argument("--out_dir", type=str, required=True, help="Output directory for detector checkpoints/logs")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--steps_per_epoch", type=int, default=120000)
    ap.add_argument("--val_steps", type=int, default=10000)
    ap.add_argument("--test_steps", type=int, default=10000)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--weight_decay", type=float, default=1e-4)
    ap.add_argument("--grad_clip", type=float, default=1.0)
    ap.add_argument("--l_pred", type=int, default=36)
    ap.add_argument("--l_det", type=int, default=36)
    ap.add_argument("--topk", type=int, default=5)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--device", type=str, default="auto")
    ap.add_argument("--num_workers", type=int, default=0)
    ap.add_argument("--log_every", type=int, default=50)
    ap.add_argument("--loader", type=str, default="device", choices=["device", "torch"])
    ap.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16"],
                    help="node-MLP tier: fp32 (fp32 parity) or bf16 (GCN transforms and EdgeHead MLP as one bf16 "
                         "MFMA product, BASELINE configs[2])")
    ap.add_argument("--dist_backend", type=str, default="auto", choices=["auto", "nccl", "gloo"],
                    help="data parallel under torchrun: nccl (= RCCL on ROCm) for GPUs, gloo for CPU / tests")
    ap.add_argument("--capture", type=str, default="auto", choices=["auto", "on", "off"],
                    help="replay each full-size training batch's step as one captured HIP graph "
                         "(models/graph_step.py; auto = on for the GPU path); the tail batch runs eagerly")
    ap.add_argument("--profile", type=int, default=0,
                    help="torch.profiler over this many training steps (after one warm-up step): "
                         "<out_dir>/detector_trace.json + detector_ops.txt on rank 0 (models/profiling.py)")
    ap.add_argument("--perf_log", type=str, default="detector_perf.jsonl",
                    help="JSONL perf log (windows/s per log interval), relative to --out_dir; '' disables")
    args = ap.parse_args(argv)

    rank, local_rank, world = dist_env()
    if world > 1:
        backend = None if args.dist_backend == "auto" else args.dist_backend
        if backend is None:
            backend = "nccl" if (args.device != "cpu" and torch.cuda.is_available()) else "gloo"
        init_distributed(backend)
    lead = rank == 0
    out_dir = Path(args.out_dir)
    if lead:
        out_dir.mkdir(parents=True, exist_ok=True)
    set_seed(args.seed)
    device = pick_device(args.device)
    if world > 1 and device.type == "cuda":
        device = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(device)
    # one log (rank 0's); every rank runs the same steps
    print = builtins.print if lead else (lambda *a, **k: None)  # noqa: A001
    print(f"{now()} [detector] device={device} seed={args.seed} world={world}")
    print(f"{now()} [detector] leak_root={args.leak_root}")
    print(f"{now()} [detector] inp_path={args.inp_path}")
    print(f"{now()} [detector] predictor_ckpt={args.predictor_ckpt}")

    predictor, predictor_ckpt = load_predictor(args.predictor_ckpt, device)
    sensor_ids: List[str] = list(predictor_ckpt["sensor_ids"])
    std_mean, std_std = predictor_ckpt.get("standardizer_mean"), predictor_ckpt.get("standardizer_std")
    if std_mean is None or std_std is None:
        raise ValueError("Error: predictor ckpt missing standardizer stats.")
    stdzr = SensorStandardizer(mean=np.asarray(std_mean.cpu() if torch.is_tensor(std_mean) else std_mean,
                                               dtype=np.float32),
                               std=np.asarray(std_std.cpu() if torch.is_tensor(std_std) else std_std,
                                              dtype=np.float32))

    base_ds = AbruptLeakDetectorDataset(leak_root=args.leak_root, steps_per_epoch=1, seed=args.seed,
                                        standardizer=stdzr)
    if sensor_ids != base_ds.get_sensor_node_ids():
        raise ValueError("Sensor IDs do not match between the normal and abrupt datasets.")
    pipe_ids_in_order = base_ds.get_pipe_ids_in_order()
    leak_train, leak_val, leak_test = split_leak_scenids(base_ds.leak_scene_ids, args.seed, ratio=(0.8, 0.1, 0.1))
    nl_train, nl_val, nl_test = split_normal_scenids(base_ds.noleak_scene_ids, args.seed + 11,
                                                     ratios=(0.8, 0.1, 0.1))
    train_pipes, all_pipes = {scenario_to_pipe_id(s) for s in leak_train}, set(pipe_ids_in_order)
    missing = all_pipes - train_pipes
    if missing:
        raise RuntimeError(f"Train split missing {len(missing)} pipes, e.g. {sorted(list(missing))[:10]}")
    print(f"{now()} [detector] train dataset covers leak pipes: {len(train_pipes)}/{len(all_pipes)}")
    print(f"{now()} [detector] leak scenes: total={len(base_ds.leak_scene_ids)} train={len(leak_train)} "
          f"val={len(leak_val)} test={len(leak_test)}")
    print(f"{now()} [detector] noleak scenes: total={len(base_ds.noleak_scene_ids)} train={len(nl_train)} "
          f"val={len(nl_val)} test={len(nl_test)}")
    print(f"{now()} [detector] classes: num_pipes={base_ds.num_pipes} num_classes={base_ds.num_pipes + 1}")

    def mk(steps, seed, cache, leak_ids, nl_ids, shard=(0, 1)):
        ds = AbruptLeakDetectorDataset(leak_root=args.leak_root, l_pred_steps=args.l_pred, l_det_steps=args.l_det,
                                       steps_per_epoch=steps, seed=seed, sensor_ids=sensor_ids, standardizer=stdzr,
                                       cache_size=cache)
        ds.leak_scene_ids, ds.noleak_scene_ids = leak_ids, nl_ids
        return ds, make_loader(ds, args.batch_size, device, args.loader, args.num_workers, shard=shard)

    train_ds, train_loader = mk(args.steps_per_epoch, args.seed, 4096, leak_train, nl_train, shard=(rank, world))
    _, val_loader = mk(args.val_steps, args.seed + 1, 2048, leak_val, nl_val)
    _, test_loader = mk(args.test_steps, args.seed + 2, 2048, leak_test, nl_test)

    detector = LeakDetector(inp_path=args.inp_path, sensor_node_ids=sensor_ids, pipe_ids_in_order=pipe_ids_in_order,
                            sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1, use_time=True,
                            mlp_dtype=args.dtype).to(device)
    clip = args.grad_clip if args.grad_clip and args.grad_clip > 0 else None
    fused_step = device.type == "cuda"  # clip_grad_norm_ + AdamW.step as one fused op pair
    if fused_step:
        opt = ClipAdamW(detector.parameters(), lr=args.lr, weight_decay=args.weight_decay, max_norm=clip)
    else:
        opt = torch.optim.AdamW(detector.parameters(), lr=args.lr, weight_decay=args.weight_decay)
    loss_fn = CrossEntropyLoss()  # torch's own path on the CPU
    allreduce = GradAllReduce(detector.parameters())  # no-op at world 1
    # identical weights on every rank (built above from args.seed); from here on each rank
    # draws its own dropout seeds
    reseed_rank(args.seed, rank, world)
    evaluator = DetectorEvaluator(predictor=predictor, detector=detector, device=device, l_pred=args.l_pred,
                                  l_det=args.l_det,
                                  metric_groups=("basic", "binary", "bucket", "atd", "success", "accuracy_i"),
                                  topk=args.topk, inp_path=args.inp_path, pipe_ids_in_order=pipe_ids_in_order)

    best_acc = -1.0
    best_path, last_path = out_dir / "detector_best.ckpt", out_dir / "detector_last.ckpt"
    meta = {
        "inp_path": str(args.inp_path), "predictor_ckpt": str(args.predictor_ckpt), "sensor_ids": sensor_ids,
        "pipe_ids_in_order": pipe_ids_in_order, "num_classes": int(base_ds.num_pipes + 1),
        "sampling_config": asdict(train_ds.cfg),
        "split": {"leak_train": leak_train, "leak_val": leak_val, "leak_test": leak_test,
                  "noleak_train": nl_train, "noleak_val": nl_val, "noleak_test": nl_test},
        "args": vars(args),
    }
    if lead:
        (out_dir / "detector_meta.json").write_text(json.dumps(meta, indent=2, ensure_ascii=False), encoding="utf-8")

    def report(tag: str, m: Dict[str, float]) -> None:
        line = (f"{now()} [detector] {tag} leak_ar={m['ar_mean']:.4f} "
                f"leak_hit@{args.topk}={m[f'leak_acc_top{args.topk}']:.4f} det_f1={m.get('det_f1', 0.0):.4f} "
                f"det_p={m.get('det_precision', 0.0):.4f} det_r={m.get('det_recall', 0.0):.4f} "
                f"ATD={m['atd_mean_m']:.4f}")
        line += "".join(f" success_at_{int(r)}={m[f'success_at_{int(r)}']:.4f}" for r in evaluator.success_radii_m)
        line += "".join(f" accuracy_{int(i)}={m[f'accuracy_{int(i)}']:.4f}" for i in evaluator.accuracy_is)
        print(line)

    print(f"{now()} [detector] start training: epochs={args.epochs}, steps/epoch={args.steps_per_epoch}, "
          f"batch={args.batch_size}")
    def global_sum(v: torch.Tensor) -> torch.Tensor:
        if world > 1:
            v = v.clone()
            torch.distributed.all_reduce(v)
        return v

    use_graph = args.capture == "on" or (args.capture == "auto" and fused_step)
    if use_graph and not fused_step:
        raise ValueError("--capture on needs the GPU path (--device cuda)")
    per_rank_full = args.batch_size // world if args.batch_size % world == 0 else -1
    cstep = None  # graph_step.CapturedTrainStep, built at the first full-size batch
    perf = PerfLog(out_dir / args.perf_log if (lead and args.perf_log) else None, world)

    from .profiling import StepProfiler
    prof = StepProfiler(out_dir, "detector", args.profile if lead else 0, device)
    for epoch in range(1, args.epochs + 1):
        detector.train()
        running = torch.zeros((), dtype=torch.float64, device=device)
        seen = torch.zeros((), dtype=torch.float64, device=device)
        for it, batch in enumerate(train_loader, start=1):
            noisy_seg = batch["noisy_seg"].to(device)
            time_seg = batch["time_seg"].to(device)
            label = torch.as_tensor(batch["label"], device=device, dtype=torch.long)
            n_local = noisy_seg.size(0)
            if n_local == 0:  # a ragged last global batch left this rank no windows
                # (mean CE over no rows is NaN): contribute zero gradients to the all-reduce, take
                # the same optimizer step as the other ranks, and fall through to the shared
                # bookkeeping below (its logging all-reduces are collectives every rank makes)
                opt.zero_grad(set_to_none=True)
                for p in detector.parameters():
                    p.grad = torch.zeros_like(p)
                allreduce()
                if clip is not None and not fused_step:
                    torch.nn.utils.clip_grad_norm_(detector.parameters(), clip)
                opt.step()
                loss = torch.zeros((), device=device)
            else:
                with torch.no_grad():
                    residual = build_residual_sequence_from_segment(predictor, noisy_seg, time_seg, l_pred=args.l_pred,
                                                                    l_det=args.l_det, device=device)
                tfeat = time_seg[:, args.l_pred:, :]
                n_glob = min(args.batch_size, len(train_ds) - (it - 1) * args.batch_size)
                # decided on the GLOBAL batch, so every rank takes the same branch (same collectives)
                if use_graph and n_glob == args.batch_size and n_local == per_rank_full:
                    # full-size batch: the whole step (fwd, CE, bwd, all-reduce, clip + AdamW) as graph
                    # replays on static inputs; the same arithmetic as the eager branch below
                    if cstep is None:
                        from .graph_step import CapturedTrainStep
                        cstep = CapturedTrainStep(detector, loss_fn, opt, (residual.clone(), tfeat.contiguous().clone()),
                                                  label.clone(), clip=None, warmup=2, preserve_state=True)
                    else:
                        cstep.inputs[0].copy_(residual)
                        cstep.inputs[1].copy_(tfeat)
                        cstep.label.copy_(label)
                    loss = cstep()
                else:
                    logits = detector(residual, tfeat)
                    loss = loss_fn(logits, label)
                    opt.zero_grad(set_to_none=True)
                    if world > 1:  # mean over the GLOBAL batch after the all-reduce's average over ranks
                        (loss * (n_local * world / n_glob)).backward()
                        allreduce()
                    else:
                        loss.backward()
                    if clip is not None and not fused_step:
                        torch.nn.utils.clip_grad_norm_(detector.parameters(), clip)
                    opt.step()
            running += loss.detach().double() * n_local
            seen += n_local
            perf.add(n_local)
            prof.step()
            if (it % args.log_every) == 0:
                r_, s_ = global_sum(running), global_sum(seen)
                print(f"{now()} [detector][epoch {epoch:02d}] step {it:05d}/{len(train_loader):05d} "
                      f"loss={r_.item() / max(s_.item(), 1):.6f}")
                perf.flush(epoch, it, r_.item() / max(s_.item(), 1), "graph" if cstep is not None else "eager")
        r_, s_ = global_sum(running), global_sum(seen)
        if lead:
            val_metrics = evaluator.evaluate(val_loader)
            report(f"[epoch {epoch:02d}] done. train_loss={r_.item() / max(s_.item(), 1):.6f}", val_metrics)
            ckpt = {"epoch": epoch, "detector_state": detector.state_dict(), "sensor_ids": sensor_ids,
                    "pipe_ids_in_order": pipe_ids_in_order, "num_classes": int(len(pipe_ids_in_order) + 1),
                    "predictor_ckpt": str(args.predictor_ckpt), "args": vars(args)}
            torch.save(ckpt, last_path)
            if val_metrics["acc_top1"] > best_acc:
                best_acc = val_metrics["acc_top1"]
                torch.save(ckpt, best_path)
                print(f"{now()} [detector] new best: acc_top1={best_acc:.4f} -> {best_path.name}")
        if world > 1:
            torch.distributed.barrier()

    prof.close()
    if lead:
        best_ckpt = torch.load(best_path, map_location=device, weights_only=True)
        detector.load_state_dict(best_ckpt["detector_state"])
        report("TEST:", evaluator.evaluate(test_loader))
        print(f"{now()} [detector] saved: {best_path.name}, {last_path.name}, meta.json")
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
