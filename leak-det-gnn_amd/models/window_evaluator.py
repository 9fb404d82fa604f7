"""Window-level evaluator for the leak detector (reference models/window_evaluator.py).

Same metric groups and definitions as the reference DetectorEvaluator
(window_evaluator.py:227-483): basic (top-1/top-k, no-leak / leak-only accuracy, average
rank of the true pipe), binary (detection precision / recall / F1, false-alarm rates),
bucket (per early / late / pre / noleak bucket), atd (average topological distance),
success (Success@r), accuracy_i (true pipe among the i nearest pipes of the prediction).

MI355X path: the reference loops over samples with .item() per sample (a device sync
each); here every count is a device reduction over the batch and one small tensor
comes back per batch.  Pipe distances are a precomputed P x P table (the reference's own
midpoint formula on Dijkstra node distances, float64, plus its float32 rank table from
np.argsort), gathered per sample on the device.
"""
from __future__ import annotations

import heapq
import math
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from .utils import build_residual_sequence_from_segment, now, parse_epanet_inp


def _dijkstra(adj: List[List[Tuple[int, float]]], start: int) -> np.ndarray:
    """Single-source shortest paths, float64 relaxations, returned as float32
    (window_evaluator.py:58-73)."""
    n = len(adj)
    dist = np.full(n, np.inf, dtype=np.float64)
    dist[start] = 0.0
    pq: List[Tuple[float, int]] = [(0.0, start)]
    while pq:
        d, u = heapq.heappop(pq)
        if d > dist[u]:
            continue
        for v, w in adj[u]:
            nd = d + float(w)
            if nd < dist[v]:
                dist[v] = nd
                heapq.heappush(pq, (float(nd), v))
    return dist.astype(np.float32, copy=False)


def _parse_links_with_length(inp_path: str | Path, eps: float) -> Dict[str, Tuple[str, str, float, str]]:
    """link_id -> (node1, node2, length, kind); pumps and valves get length eps
    (window_evaluator.py:76-110)."""
    sections = parse_epanet_inp(inp_path)
    out: Dict[str, Tuple[str, str, float, str]] = {}
    for line in sections.get("PIPES", []):
        toks = line.split()
        if len(toks) < 4:
            continue
        try:
            length = float(toks[3])
        except Exception:
            length = 1.0
        out[toks[0]] = (toks[1], toks[2], length, "PIPES")
    for kind in ("PUMPS", "VALVES"):
        for line in sections.get(kind, []):
            toks = line.split()
            if len(toks) < 3:
                continue
            out[toks[0]] = (toks[1], toks[2], float(eps), kind)
    return out


@dataclass
class PipeDistanceOracle:
    """Pipe-to-pipe distances (window_evaluator.py:113-224)."""
    inp_path: str
    pipe_ids_in_order: List[str]
    node_names: List[str]
    node_to_idx: Dict[str, int]
    pipe_ends: np.ndarray
    pipe_len: np.ndarray
    node_adj: List[List[Tuple[int, float]]]
    node_dist_cache: Dict[int, np.ndarray]
    pipe_dist: Optional[np.ndarray]
    pipe_rank: Optional[np.ndarray]

    @staticmethod
    def build(inp_path: str | Path, pipe_ids_in_order: Sequence[str], eps: float = 0.1) -> "PipeDistanceOracle":
        inp_path = str(inp_path)
        pipe_ids = list(pipe_ids_in_order)
        links = _parse_links_with_length(inp_path, eps)
        if not links:
            raise ValueError("No links parsed from inp; cannot compute distance metrics.")
        node_names = sorted({n for (a, b, _, _) in links.values() for n in (a, b)})
        node_to_idx = {n: i for i, n in enumerate(node_names)}
        adj: List[List[Tuple[int, float]]] = [[] for _ in node_names]
        for (n1, n2, length, _) in links.values():
            u, v = node_to_idx[n1], node_to_idx[n2]
            w = float(length) if (length is not None and not math.isnan(length)) else 1.0
            adj[u].append((v, w))
            adj[v].append((u, w))
        P = len(pipe_ids)
        ends = np.zeros((P, 2), dtype=np.int32)
        plen = np.zeros((P,), dtype=np.float32)
        for i, pid in enumerate(pipe_ids):
            if pid not in links:
                raise ValueError(f"pipe_id '{pid}' not found in inp [PIPES]/[PUMPS]/[VALVES].")
            n1, n2, length, _ = links[pid]
            ends[i] = (node_to_idx[n1], node_to_idx[n2])
            plen[i] = float(length) if (length is not None and not math.isnan(length)) else 1.0
        return PipeDistanceOracle(inp_path, pipe_ids, node_names, node_to_idx, ends, plen, adj, {}, None, None)

    def _node_dists(self, start: int) -> np.ndarray:
        if start not in self.node_dist_cache:
            self.node_dist_cache[start] = _dijkstra(self.node_adj, start)
        return self.node_dist_cache[start]

    def pipe_distance(self, p: int, q: int) -> float:
        """window_evaluator.py:180-190 (midpoint approximation, python floats)."""
        if p == q:
            return 0.0
        up, vp = int(self.pipe_ends[p, 0]), int(self.pipe_ends[p, 1])
        uq, vq = int(self.pipe_ends[q, 0]), int(self.pipe_ends[q, 1])
        d_up, d_vp = self._node_dists(up), self._node_dists(vp)
        dmin = min(float(d_up[uq]), float(d_up[vq]), float(d_vp[uq]), float(d_vp[vq]))
        return dmin + 0.5 * float(self.pipe_len[p]) + 0.5 * float(self.pipe_len[q])

    def pair_distance_table(self) -> np.ndarray:
        """T[y, p] = pipe_distance(y, p) for all pairs (float64), the ATD / Success@r table."""
        P = len(self.pipe_ids_in_order)
        ends, L = self.pipe_ends, self.pipe_len.astype(np.float64)
        u, v = ends[:, 0], ends[:, 1]
        out = np.zeros((P, P), dtype=np.float64)
        for y in range(P):
            d_u = self._node_dists(int(ends[y, 0])).astype(np.float64)
            d_v = self._node_dists(int(ends[y, 1])).astype(np.float64)
            dmin = np.minimum.reduce([d_u[u], d_u[v], d_v[u], d_v[v]])
            out[y] = dmin + 0.5 * L[y] + 0.5 * L
            out[y, y] = 0.0
        return out

    def ensure_pipe_matrix(self) -> None:
        """window_evaluator.py:192-224: float32 distance matrix and its row argsort."""
        if self.pipe_dist is not None and self.pipe_rank is not None:
            return
        P = len(self.pipe_ids_in_order)
        ends, L = self.pipe_ends, self.pipe_len
        for s in np.unique(ends.reshape(-1)).tolist():
            self._node_dists(int(s))
        dist_mat = np.zeros((P, P), dtype=np.float32)
        u_list, v_list = ends[:, 0].astype(np.int32), ends[:, 1].astype(np.int32)
        for p in range(P):
            d_up = self.node_dist_cache[int(ends[p, 0])]
            d_vp = self.node_dist_cache[int(ends[p, 1])]
            dmin = np.minimum.reduce([d_up[u_list], d_up[v_list], d_vp[u_list], d_vp[v_list]]).astype(np.float32)
            dist_mat[p, :] = dmin + 0.5 * L[p] + 0.5 * L
            dist_mat[p, p] = 0.0
        self.pipe_dist = dist_mat
        self.pipe_rank = np.argsort(dist_mat, axis=1).astype(np.int32)


_BUCKETS = ("early", "late", "pre", "noleak")


class DetectorEvaluator:
    """Evaluator for (predictor + detector) on a loader of detector batches
    (window_evaluator.py:227-483); the batches may come from a DataLoader or from
    datasets.DeviceBatchLoader (tensors already on the device)."""

    def __init__(self, predictor: nn.Module, detector: nn.Module, device: torch.device, *, l_pred: int,
                 l_det: int, topk: int = 5, metric_groups: Sequence[str] = ("basic", "binary", "bucket"),
                 inp_path: Optional[str | Path] = None, pipe_ids_in_order: Optional[Sequence[str]] = None,
                 success_radii_m: Sequence[float] = (50.0, 100.0, 300.0),
                 accuracy_is: Sequence[int] = (1, 5, 10, 20)) -> None:
        self.predictor = predictor
        self.detector = detector
        self.device = torch.device(device)
        self.l_pred, self.l_det, self.topk = int(l_pred), int(l_det), int(topk)
        self.metric_groups = set(metric_groups) | {"basic"}
        self.inp_path = inp_path
        self.pipe_ids_in_order = pipe_ids_in_order
        self.success_radii_m = [float(x) for x in success_radii_m]
        self.accuracy_is = [int(i) for i in accuracy_is]
        self.residual_builder = build_residual_sequence_from_segment
        print(f"{now()} [metric_evaluator] building evaluator for metrics: {self.metric_groups}.")
        self.oracle: Optional[PipeDistanceOracle] = None
        self._dist = self._inv_rank = None
        if {"atd", "success", "accuracy_i"} & self.metric_groups:
            if self.inp_path is None or self.pipe_ids_in_order is None:
                raise ValueError("Distance metrics requested but inp_path/pipe_ids_in_order not provided.")
            self.oracle = PipeDistanceOracle.build(self.inp_path, self.pipe_ids_in_order)
            self._dist = torch.from_numpy(self.oracle.pair_distance_table()).to(self.device)
            if "accuracy_i" in self.metric_groups:
                self.oracle.ensure_pipe_matrix()
                rank = torch.from_numpy(self.oracle.pipe_rank.astype(np.int64))
                inv = torch.empty_like(rank)
                inv.scatter_(1, rank, torch.arange(rank.shape[1]).expand_as(rank))
                self._inv_rank = inv.to(self.device)  # inv[p, y] = position of y in pipe_rank[p]

    @torch.no_grad()
    def evaluate(self, loader: Iterable[Dict[str, Any]]) -> Dict[str, float]:
        self.predictor.eval()
        self.detector.eval()
        dev = self.device
        acc: Dict[str, torch.Tensor] = {}

        def add(name: str, v: torch.Tensor) -> None:
            v = v.to(torch.float64)
            acc[name] = acc[name] + v if name in acc else v

        ar_ranks: List[torch.Tensor] = []
        atd_vals: List[torch.Tensor] = []
        for batch in loader:
            noisy_seg = batch["noisy_seg"].to(dev)
            time_seg = batch["time_seg"].to(dev)
            label = torch.as_tensor(batch["label"], device=dev, dtype=torch.long)
            n = label.numel()
            bucket_list = batch.get("bucket", None) or ["unknown"] * n
            bcode = torch.tensor([_BUCKETS.index(str(b)) if str(b) in _BUCKETS else -1 for b in bucket_list],
                                 device=dev)
            num_classes = batch.get("num_classes", None)
            if isinstance(num_classes, (list, tuple)):
                num_classes = int(num_classes[0])
            elif torch.is_tensor(num_classes):
                num_classes = int(num_classes[0].item())
            residual = self.residual_builder(self.predictor, noisy_seg, time_seg, l_pred=self.l_pred,
                                             l_det=self.l_det, device=dev)
            logits = self.detector(residual, time_seg[:, self.l_pred:, :])
            if num_classes is None:
                num_classes = int(logits.size(-1))
            nlc = num_classes - 1
            pred1 = logits.argmax(dim=-1)
            k = min(self.topk, logits.size(-1))
            hitk = (logits.topk(k=k, dim=-1).indices == label.unsqueeze(1)).any(dim=1)
            hit1 = pred1 == label
            is_nl = label == nlc
            is_leak = ~is_nl
            add("total", torch.tensor(n, device=dev))
            add("correct1", hit1.sum())
            add("correctk", hitk.sum())
            add("nl_total", is_nl.sum())
            add("nl_correct", (hit1 & is_nl).sum())
            add("leak_total", is_leak.sum())
            add("leak_correct1", (hit1 & is_leak).sum())
            add("leak_correctk", (hitk & is_leak).sum())
            # AR: rank of the true pipe among the pipe logits (stable descending argsort)
            pipe_logits = logits[:, :nlc]
            order = torch.argsort(pipe_logits, dim=1, descending=True)
            inv = torch.empty_like(order)
            inv.scatter_(1, order, torch.arange(nlc, device=dev).unsqueeze(0).expand(order.size(0), -1))
            ranks = inv.gather(1, label.clamp_max(nlc - 1).unsqueeze(1)).squeeze(1) + 1
            ar_ranks.append(ranks[is_leak])
            pred_leak = pred1 != nlc
            add("tp", (pred_leak & is_leak).sum())
            add("fp", (pred_leak & is_nl).sum())
            add("fn", (~pred_leak & is_leak).sum())
            add("tn", (~pred_leak & is_nl).sum())
            if "bucket" in self.metric_groups:
                for bi, b in enumerate(_BUCKETS):
                    m = bcode == bi
                    add(f"b_total_{b}", m.sum())
                    add(f"b_correct1_{b}", (hit1 & m).sum())
                    add(f"b_correctk_{b}", (hitk & m).sum())
                    add(f"b_pred_nl_{b}", ((pred1 == nlc) & m).sum())
                fa = is_nl & pred_leak
                add("pre_false_alarm", (fa & (bcode == 2)).sum())
                add("noleak_false_alarm", (fa & (bcode == 3)).sum())
                add("pre_total", (bcode == 2).sum())
                add("noleak_only_total", (bcode == 3).sum())
            if self._dist is not None:
                y = label[is_leak]
                p = pred1[is_leak]
                missed = p == nlc
                d = torch.where(missed, torch.full_like(y, 0, dtype=torch.float64),
                                self._dist[y, p.clamp_max(nlc - 1)])
                d = torch.where(missed, torch.full_like(d, float("inf")), d)
                atd_vals.append(d)
                for r in self.success_radii_m:
                    add(f"success_{r}", (d <= r).sum())
                if self._inv_rank is not None:
                    pos = self._inv_rank[p.clamp_max(nlc - 1), y]
                    for ii in self.accuracy_is:
                        add(f"acc_i_{ii}", ((~missed) & (pos < ii) & (ii > 0)).sum())

        c = {name: float(v.item()) for name, v in acc.items()}
        g = lambda name: c.get(name, 0.0)  # noqa: E731

        def safe_div(a: float, b: float) -> float:
            return float(a / b) if b > 0 else 0.0

        ar = torch.cat(ar_ranks).cpu().numpy() if ar_ranks else np.zeros(0)
        out: Dict[str, float] = {}
        leak_pred_as_noleak = g("fn")
        out.update({
            "acc_top1": safe_div(g("correct1"), g("total")),
            f"acc_top{self.topk}": safe_div(g("correctk"), g("total")),
            "noleak_acc": safe_div(g("nl_correct"), g("nl_total")),
            "leak_acc_top1": safe_div(g("leak_correct1"), g("leak_total")),
            f"leak_acc_top{self.topk}": safe_div(g("leak_correctk"), g("leak_total")),
            "ar_mean": float(np.mean(ar)) if ar.size else float("inf"),
            "ar_median": float(np.median(ar)) if ar.size else float("inf"),
            "ar_n": float(ar.size),
            "n_total": g("total"), "n_leak": g("leak_total"), "n_noleak": g("nl_total"),
        })
        if "binary" in self.metric_groups:
            tp, fp, fn, tn = g("tp"), g("fp"), g("fn"), g("tn")
            prec, rec = safe_div(tp, tp + fp), safe_div(tp, tp + fn)
            out.update({
                "det_precision": prec, "det_recall": rec,
                "det_f1": safe_div(2 * prec * rec, prec + rec) if (prec + rec) > 0 else 0.0,
                "det_tp": tp, "det_fp": fp, "det_fn": fn, "det_tn": tn,
                "leak_pred_as_noleak_rate": safe_div(leak_pred_as_noleak, g("leak_total")),
            })
            if g("pre_total") > 0:
                out["pre_false_alarm_rate"] = safe_div(g("pre_false_alarm"), g("pre_total"))
            if g("noleak_only_total") > 0:
                out["noleak_false_alarm_rate"] = safe_div(g("noleak_false_alarm"), g("noleak_only_total"))
        if "bucket" in self.metric_groups:
            for b in _BUCKETS:
                tot = g(f"b_total_{b}")
                out[f"{b}_n"] = tot
                out[f"{b}_acc_top1"] = safe_div(g(f"b_correct1_{b}"), tot)
                out[f"{b}_acc_top{self.topk}"] = safe_div(g(f"b_correctk_{b}"), tot)
                out[f"{b}_pred_as_noleak_rate"] = safe_div(g(f"b_pred_nl_{b}"), tot)
        if "atd" in self.metric_groups:
            vals = torch.cat(atd_vals).cpu().numpy() if atd_vals else np.zeros(0)
            finite = vals[np.isfinite(vals)]
            out["atd_mean_m"] = float(np.mean(finite)) if finite.size else float("inf")
            out["atd_median_m"] = float(np.median(finite)) if finite.size else float("inf")
            out["atd_n"] = float(vals.size)
            out["atd_missed_rate"] = safe_div(float((~np.isfinite(vals)).sum()), vals.size)
        if "success" in self.metric_groups:
            detected = g("leak_total") - leak_pred_as_noleak
            for r in self.success_radii_m:
                out[f"success_at_{int(r)}"] = safe_div(g(f"success_{r}"), detected)
                out[f"success_at_{int(r)}_e2e"] = safe_div(g(f"success_{r}"), g("leak_total"))
        if "accuracy_i" in self.metric_groups:
            for ii in self.accuracy_is:
                out[f"accuracy_{int(ii)}"] = safe_div(g(f"acc_i_{ii}"), g("leak_total"))
        return out
