"""Host-side graph construction and residual building for the detector.

Mirrors the public API of reference models/utils.py:
  now()                               (utils.py:15-16)
  parse_epanet_inp(inp_path)          (utils.py:18-51)
  WDNGraph                            (utils.py:72-82)
  build_wdn_graph_from_inp(...)       (utils.py:84-166)
  build_residual_sequence_from_segment(...)   (utils.py:169-216)

The graph builder runs once per model on the CPU and fixes the bit-exact integer
contract of the hot path: node order = Python-sorted node names, edge columns
[u->v, v->u] per link in PIPES, PUMPS, VALVES order (later duplicates of a link
id overwrite earlier ones in place, as a dict update does), pipe_ends from
[PIPES] only.  Everything after it (CSR, gcn_norm, incidence) is derived on the
device by libleakgnn.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import tcn_plan

_SECTION = re.compile(r"^\s*\[(.+?)\]\s*$")


def now() -> str:
    return datetime.now().strftime("%Y-%m-%d %H:%M:%S")


def parse_epanet_inp(inp_path: str | Path) -> Dict[str, List[str]]:
    """Section name (upper case) -> non-empty, comment-stripped lines, in file order."""
    sections: Dict[str, List[str]] = {}
    cur: Optional[List[str]] = None
    text = Path(inp_path).read_text(encoding="utf-8", errors="ignore")
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        m = _SECTION.match(line)
        if m:
            cur = sections.setdefault(m.group(1).strip().upper(), [])
            continue
        if cur is None:
            continue
        line = line.partition(";")[0].strip()
        if line:
            cur.append(line)
    return sections


def _first_tokens(lines: Sequence[str]) -> List[str]:
    return [ln.split()[0] for ln in lines if ln.split()]


def _link_table(lines: Sequence[str]) -> Dict[str, Tuple[str, str]]:
    table: Dict[str, Tuple[str, str]] = {}
    for ln in lines:
        tok = ln.split()
        if len(tok) >= 3:
            table[tok[0]] = (tok[1], tok[2])
    return table


@dataclass(frozen=True)
class WDNGraph:
    node_names: List[str]
    node_to_idx: Dict[str, int]
    pipe_ids: List[str]
    pipe_to_idx: Dict[str, int]
    pipe_ends: np.ndarray   # (P, 2) int64
    edge_index: Any         # torch.LongTensor (2, E)


def build_wdn_graph_from_inp(
    inp_path: str | Path,
    sensor_node_ids: Sequence[str],
    pipe_ids_in_order: Sequence[str],
    *,
    include_all_nodes: bool = True,
    include_links: Sequence[str] = ("PIPES", "PUMPS", "VALVES"),
    add_self_loops: bool = True,
    make_undirected: bool = True,
) -> WDNGraph:
    sec = parse_epanet_inp(inp_path)

    links: Dict[str, Tuple[str, str]] = {}
    for name in include_links:
        links.update(_link_table(sec.get(name.upper(), [])))
    if not links:
        raise ValueError(f"No link endpoints found from sections {tuple(include_links)} in inp file.")

    names = set(sensor_node_ids)
    if include_all_nodes:
        for s in ("JUNCTIONS", "RESERVOIRS", "TANKS"):
            names.update(_first_tokens(sec.get(s, [])))
    for a, b in links.values():
        names.add(a)
        names.add(b)
    node_names = sorted(names)
    node_to_idx = {n: i for i, n in enumerate(node_names)}

    pipes = _link_table(sec.get("PIPES", []))
    if not pipes:
        raise ValueError("No [PIPES] section found or empty; cannot map pipe_ids to endpoints.")
    pipe_ids = list(pipe_ids_in_order)
    pipe_to_idx = {p: i for i, p in enumerate(pipe_ids)}
    pipe_ends = np.zeros((len(pipe_ids), 2), dtype=np.int64)
    for i, pid in enumerate(pipe_ids):
        if pid not in pipes:
            raise ValueError(f"Pipe id {pid} not found in inp [PIPES].")
        a, b = pipes[pid]
        pipe_ends[i] = (node_to_idx[a], node_to_idx[b])

    ends = np.array([(node_to_idx[a], node_to_idx[b]) for a, b in links.values()], dtype=np.int64).reshape(-1, 2)
    if make_undirected:
        src = np.stack([ends[:, 0], ends[:, 1]], axis=1).reshape(-1)
        dst = np.stack([ends[:, 1], ends[:, 0]], axis=1).reshape(-1)
    else:
        src, dst = ends[:, 0].copy(), ends[:, 1].copy()
    if add_self_loops:
        loops = np.arange(len(node_names), dtype=np.int64)
        src = np.concatenate([src, loops])
        dst = np.concatenate([dst, loops])
    edge_index = torch.from_numpy(np.stack([src, dst]).astype(np.int64))

    return WDNGraph(node_names=node_names, node_to_idx=node_to_idx, pipe_ids=pipe_ids, pipe_to_idx=pipe_to_idx,
                    pipe_ends=pipe_ends, edge_index=edge_index)


# LEAKGNN_RESIDUAL=stock keeps the per-window module calls (for A/B timing).
RESIDUAL_FAST_PATH = os.environ.get("LEAKGNN_RESIDUAL", "fast") != "stock"


def build_residual_sequence_from_segment(predictor: Any, noisy_seg: Any, time_seg: Any, l_pred: int, l_det: int,
                                         device: Optional[Any] = None) -> Any:
    """residual[b, k] = noisy[b, l_pred+k] - predictor(noisy[b, k:k+l_pred], time[b, k:k+l_pred]).

    One predictor call over all l_det shifted windows stacked shift-major
    (row = k*B + b), as the reference does (utils.py:194-212)."""
    squeeze = noisy_seg.dim() == 2
    if squeeze:
        noisy_seg, time_seg = noisy_seg.unsqueeze(0), time_seg.unsqueeze(0)
    B, T, S = noisy_seg.shape
    assert T == l_pred + l_det, (T, l_pred, l_det)
    if device is not None:
        noisy_seg, time_seg = noisy_seg.to(device), time_seg.to(device)
    if noisy_seg.is_cuda and RESIDUAL_FAST_PATH and tcn_plan.fast_path_eligible(predictor):
        # frozen default TCN on the GPU: one shared-window pass per segment (HIP,
        # lg_tcn_conv_fwd); same values as the per-window passes below within fp32 rounding
        res = tcn_plan.tcn_residual(predictor, noisy_seg.float(), time_seg.float(), l_pred, l_det)
        return res.squeeze(0) if squeeze else res
    # (l_det, B, l_pred, C) windows via unfold: window k covers [k, k + l_pred)
    xw = noisy_seg.unfold(1, l_pred, 1)[:, :l_det].permute(1, 0, 3, 2).reshape(l_det * B, l_pred, S)
    tw = time_seg.unfold(1, l_pred, 1)[:, :l_det].permute(1, 0, 3, 2).reshape(l_det * B, l_pred, -1)
    target = noisy_seg[:, l_pred:, :].transpose(0, 1).reshape(l_det * B, S)
    y_hat = predictor(xw.contiguous(), tw.contiguous())
    if y_hat.dim() == 3:
        y_hat = y_hat[:, -1, :]
    res = (target - y_hat).view(l_det, B, S).transpose(0, 1).contiguous()
    return res.squeeze(0) if squeeze else res
