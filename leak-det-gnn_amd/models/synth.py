"""Synthetic pipe-network graphs (configs C4 / C5 of BASELINE.json) and an EPANET
.inp writer, so LeakDetector(inp_path, ...) is constructed unchanged.

Topology: nodes on a jittered sqrt(N) x sqrt(N) grid; a random spanning tree of
the 4-neighbour grid (Kruskal on random weights) plus loop chords drawn from the
remaining grid edges, degree capped at 5; all seeded.  Node ids n{i}, pipe ids
p{i}; the last node is the reservoir.  Generated because the reference's data
generators need `wntr` (absent) — SURVEY §8(d) C4/C5.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


def _find(parent: np.ndarray, i: int) -> int:
    root = i
    while parent[root] != root:
        root = parent[root]
    while parent[i] != root:
        parent[i], i = root, parent[i]
    return root


def synthetic_pipe_ends(num_nodes: int, num_pipes: int, seed: int = 0, max_degree: int = 5) -> np.ndarray:
    N, P = int(num_nodes), int(num_pipes)
    if P < N - 1:
        raise ValueError("need at least N-1 pipes for a connected network")
    rng = np.random.default_rng(seed)
    W = int(np.ceil(np.sqrt(N)))
    ids = np.arange(N)
    x, y = ids % W, ids // W
    right = ids[(x + 1 < W) & (ids + 1 < N)]
    down = ids[ids + W < N]
    cand = np.concatenate([np.stack([right, right + 1], 1), np.stack([down, down + W], 1)])
    cand = cand[rng.permutation(len(cand))]
    parent = np.arange(N)
    deg = np.zeros(N, dtype=np.int64)
    tree, rest = [], []
    for a, b in cand:
        ra, rb = _find(parent, a), _find(parent, b)
        if ra != rb:
            parent[ra] = rb
            tree.append((a, b))
            deg[a] += 1
            deg[b] += 1
        else:
            rest.append((a, b))
    if len(tree) != N - 1:
        raise RuntimeError("grid spanning tree failed")
    chords = []
    need = P - (N - 1)
    for a, b in rest:
        if len(chords) >= need:
            break
        if deg[a] < max_degree and deg[b] < max_degree:
            chords.append((a, b))
            deg[a] += 1
            deg[b] += 1
    if len(chords) < need:
        raise ValueError(f"cannot place {P} pipes on {N} grid nodes with degree <= {max_degree}")
    ends = np.array(tree + chords, dtype=np.int64)
    flip = rng.random(len(ends)) < 0.5
    ends[flip] = ends[flip][:, ::-1]
    return ends[rng.permutation(len(ends))]


def synthetic_pipe_graph(num_nodes: int, num_pipes: int, seed: int = 0) -> Tuple[torch.Tensor, np.ndarray]:
    """(edge_index (2, 2P) with columns [u->v, v->u] per pipe, pipe_ends (P, 2)) in generator numbering."""
    ends = synthetic_pipe_ends(num_nodes, num_pipes, seed)
    src = np.stack([ends[:, 0], ends[:, 1]], 1).reshape(-1)
    dst = np.stack([ends[:, 1], ends[:, 0]], 1).reshape(-1)
    return torch.from_numpy(np.stack([src, dst])), ends


def write_synthetic_inp(path: str | Path, num_nodes: int, num_pipes: int, seed: int = 0) -> Tuple[list, list]:
    """Write an EPANET .inp with the synthetic topology; returns (node_ids, pipe_ids)."""
    ends = synthetic_pipe_ends(num_nodes, num_pipes, seed)
    N = int(num_nodes)
    rng = np.random.default_rng(seed + 1)
    W = int(np.ceil(np.sqrt(N)))
    node_ids = [f"n{i}" for i in range(N)]
    pipe_ids = [f"p{i}" for i in range(len(ends))]
    lines = ["[TITLE]", f"synthetic pipe network N={N} P={len(ends)} seed={seed}", "", "[JUNCTIONS]"]
    lines += [f" {node_ids[i]} 50.0 0.1" for i in range(N - 1)]
    lines += ["", "[RESERVOIRS]", f" {node_ids[N - 1]} 100", "", "[PIPES]"]
    lines += [f" {pipe_ids[k]} {node_ids[a]} {node_ids[b]} 50.0 150 120 0 Open" for k, (a, b) in enumerate(ends)]
    lines += ["", "[COORDINATES]"]
    jit = rng.uniform(-0.3, 0.3, size=(N, 2))
    lines += [f"{node_ids[i]} {100.0 * (i % W + jit[i, 0]):.3f} {100.0 * (i // W + jit[i, 1]):.3f}" for i in range(N)]
    lines += ["", "[END]"]
    Path(path).write_text("\n".join(lines) + "\n", encoding="utf-8")
    return node_ids, pipe_ids


def pick_sensors(node_ids: Sequence[str], count: int = 29, seed: int = 0) -> list:
    rng = np.random.default_rng(seed + 2)
    return [node_ids[i] for i in sorted(rng.choice(len(node_ids) - 1, size=count, replace=False))]


def pick_pipes(pipe_ids: Sequence[str], ratio: float, seed: int = 198) -> list:
    """The leak set's pipe list for `--pipe_sample_ratio ratio` (reference
    data_gen/leak_generation.py:90-99 with default_rng(seed), seed 198 as in cmd.sh:10),
    sorted as the datasets order them (datasets.py:353): the detector's pipe_ids_in_order.
    ratio 0.5 on L-TOWN-A's 764 pipes gives P = 382."""
    ratio = min(max(float(ratio), 0.0), 1.0)
    if ratio <= 0 or not pipe_ids:
        return []
    n = max(1, int(round(len(pipe_ids) * ratio)))
    idx = np.random.default_rng(int(seed)).choice(len(pipe_ids), size=n, replace=False)
    return sorted(pipe_ids[i] for i in idx)


# ------------------------------------------------------------------ sensor data sets
def _sensor_frame(sensor_ids: Sequence[str], T: int, rng: np.random.Generator, start: str,
                  drop: Optional[np.ndarray] = None):
    """(clean, noisy) DataFrames in the reference layout (index 'datetime' at 5 min, one
    column per sensor): 40 + 5 sin(t/20 + phase) + N(0, 1) per sensor (SURVEY §8 d, C1),
    multiplicative noise N(1, 2.5e-4); `drop` (T, S) is subtracted from the clean signal."""
    import pandas as pd
    S = len(sensor_ids)
    t = np.arange(T, dtype=np.float64)[:, None]
    phase = rng.uniform(0, 2 * np.pi, size=(1, S))
    clean = 40.0 + 5.0 * np.sin(t / 20.0 + phase) + rng.normal(0.0, 1.0, size=(T, S))
    if drop is not None:
        clean = clean - drop
    noisy = clean * rng.normal(1.0, 2.5e-4, size=(T, S))
    idx = pd.date_range(start, periods=T, freq="5min", name="datetime")
    return (pd.DataFrame(clean, index=idx, columns=list(sensor_ids)),
            pd.DataFrame(noisy, index=idx, columns=list(sensor_ids)))


def write_synthetic_normal_set(root: str | Path, sensor_ids: Sequence[str], n_windows: int = 12, T: int = 577,
                               seed: int = 0) -> List[str]:
    """No-leak set in the reference format (datasets.py:72-111, 200-257): manifest.jsonl rows
    {"window_id", "status": "ok"}, <id>/sensors.csv (noisy) and <id>/sensors_gt.csv."""
    root = Path(root)
    root.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(seed)
    ids = [f"w{i:05d}" for i in range(n_windows)]
    for i, wid in enumerate(ids):
        (root / wid).mkdir(exist_ok=True)
        gt, noisy = _sensor_frame(sensor_ids, T, rng, start=f"2024-01-{1 + i % 28:02d} 00:00")
        noisy.to_csv(root / wid / "sensors.csv")
        gt.to_csv(root / wid / "sensors_gt.csv")
    with open(root / "manifest.jsonl", "w", encoding="utf-8") as f:
        for wid in ids:
            f.write(json.dumps({"window_id": wid, "status": "ok"}) + "\n")
    return ids


def write_synthetic_leak_set(root: str | Path, sensor_ids: Sequence[str], pipe_ids: Sequence[str],
                             scenes_per_pipe: int = 2, n_noleak: int = 6, T: int = 400, seed: int = 0) -> dict:
    """Abrupt-leak set in the reference format (datasets.py:282-435, leak_generation.py):
    manifest rows {"scenario_id": "NNNNNN_<pipe>_abrupt_rK", "status", "kind": "leak",
    "leak_type": "abrupt", "pipe_id"} plus no-leak rows {"scenario_id", "kind": "no_leak"} (leak_generation.py:373);
    each leak scene has leak_flow_m3h.csv (column = pipe id, 0 before the onset) and a
    pressure drop after the onset.  One row is marked status "failed" (filtered out)."""
    import pandas as pd
    root = Path(root)
    root.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(seed)
    rows = []
    k = 0
    for pid in pipe_ids:
        for r in range(scenes_per_pipe):
            sid = f"{k:06d}_{pid}_abrupt_r{r + 1}"
            k += 1
            tau = int(rng.integers(100, T - 60))
            drop = np.zeros((T, len(sensor_ids)))
            drop[tau:] = rng.uniform(0.05, 0.5, size=(1, len(sensor_ids)))
            (root / sid).mkdir(exist_ok=True)
            gt, noisy = _sensor_frame(sensor_ids, T, rng, start=f"2024-02-{1 + k % 28:02d} 00:00", drop=drop)
            noisy.to_csv(root / sid / "sensors.csv")
            gt.to_csv(root / sid / "sensors_gt.csv")
            q = np.zeros(T)
            q[tau:] = rng.uniform(1.0, 5.0)
            pd.DataFrame({pid: q}, index=gt.index).to_csv(root / sid / "leak_flow_m3h.csv")
            rows.append({"scenario_id": sid, "status": "ok", "kind": "leak", "leak_type": "abrupt", "pipe_id": pid})
    for j in range(n_noleak):
        sid = f"{k:06d}_noleak"
        k += 1
        (root / sid).mkdir(exist_ok=True)
        gt, noisy = _sensor_frame(sensor_ids, T, rng, start=f"2024-03-{1 + j % 28:02d} 00:00")
        noisy.to_csv(root / sid / "sensors.csv")
        gt.to_csv(root / sid / "sensors_gt.csv")
        rows.append({"scenario_id": sid, "status": "ok", "kind": "no_leak"})
    rows.append({"scenario_id": "999999_failed", "status": "failed", "kind": "no_leak"})
    with open(root / "manifest.jsonl", "w", encoding="utf-8") as f:
        for row in rows:
            f.write(json.dumps(row) + "\n")
    return {"rows": rows}
