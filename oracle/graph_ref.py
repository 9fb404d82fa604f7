"""ORACLE (test infrastructure only) — integer graph work of the hot path.

Restates, in plain Python / numpy:
  parse_inp          reference models/utils.py:18-51   (parse_epanet_inp)
  build_graph        reference models/utils.py:84-166  (build_wdn_graph_from_inp)
  batchify           reference models/detector.py:105-114 (_batchify_edge_index)
  gcn_csr            PyG gcn_norm (add_remaining_self_loops, deg^-1/2) as a CSR keyed
                     by target, entries in ascending edge order, self loop last
  incidence_csr      pipe-endpoint incidence keyed by node, items 2p+role ascending
"""
from __future__ import annotations

import numpy as np


def parse_inp(path):
    """utils.py:18-51: section -> lines; ';' comments stripped; blank lines dropped."""
    out, cur = {}, None
    with open(path, "r", encoding="utf-8", errors="ignore") as f:
        for raw in f:
            s = raw.strip()
            if not s:
                continue
            if s.startswith("[") and s.endswith("]") and len(s) > 2:
                cur = s[1:-1].strip().upper()
                out.setdefault(cur, [])
                continue
            if cur is None:
                continue
            if ";" in s:
                s = s[: s.index(";")].strip()
            if s:
                out[cur].append(s)
    return out


def _links(lines):
    """utils.py:63-69: id -> (node1, node2); later ids overwrite earlier ones."""
    d = {}
    for s in lines:
        t = s.split()
        if len(t) >= 3:
            d[t[0]] = (t[1], t[2])
    return d


def build_graph(path, sensor_ids, pipe_ids, include_links=("PIPES", "PUMPS", "VALVES"),
                add_self_loops=False, make_undirected=True):
    """utils.py:84-166 -> (node_names, edge_index int64 (2,E), pipe_ends int64 (P,2))."""
    sec = parse_inp(path)
    links = {}
    for name in include_links:
        links.update(_links(sec.get(name.upper(), [])))
    nodes = set(sensor_ids)
    for name in ("JUNCTIONS", "RESERVOIRS", "TANKS"):
        for s in sec.get(name, []):
            t = s.split()
            if t:
                nodes.add(t[0])
    for a, b in links.values():
        nodes.add(a)
        nodes.add(b)
    names = sorted(nodes)
    idx = {n: i for i, n in enumerate(names)}
    pipes = _links(sec.get("PIPES", []))
    ends = np.array([[idx[pipes[p][0]], idx[pipes[p][1]]] for p in pipe_ids], dtype=np.int64).reshape(-1, 2)
    src, dst = [], []
    for a, b in links.values():
        src.append(idx[a]); dst.append(idx[b])
        if make_undirected:
            src.append(idx[b]); dst.append(idx[a])
    if add_self_loops:
        for i in range(len(names)):
            src.append(i); dst.append(i)
    return names, np.array([src, dst], dtype=np.int64), ends


def batchify(edge_index, num_nodes, batch_size):
    """detector.py:105-114: repeat(1, B) + arange(B).repeat_interleave(E) * N."""
    E = edge_index.shape[1]
    off = np.repeat(np.arange(batch_size, dtype=np.int64), E) * num_nodes
    return np.tile(edge_index, (1, batch_size)) + off[None, :]


def gcn_csr(edge_index, num_nodes, add_self_loops=True, normalize=True, fill=1.0, transpose=False):
    """PyG gcn_norm as a CSR.  Keyed by target (transpose=False) or source (True).

    add_remaining_self_loops: existing loops dropped, (i, i) appended for every node
    with weight `fill`; deg[d] = sum of weights into d (fp32); dis = deg^-1/2 with
    inf -> 0; w = (dis[src] * weight) * dis[dst]  (fp32, left to right).
    Returns rowptr int32 (N+1), col int32, w float32; rows keep ascending edge order,
    the appended loop last."""
    src = edge_index[0].astype(np.int64)
    dst = edge_index[1].astype(np.int64)
    N = int(num_nodes)
    wt = np.ones(src.shape[0], dtype=np.float32)
    if add_self_loops:
        keep = src != dst
        src, dst, wt = src[keep], dst[keep], wt[keep]
        loops = np.arange(N, dtype=np.int64)
        src = np.concatenate([src, loops])
        dst = np.concatenate([dst, loops])
        wt = np.concatenate([wt, np.full(N, fill, dtype=np.float32)])
    if normalize:
        deg = np.zeros(N, dtype=np.float32)
        np.add.at(deg, dst, wt)
        with np.errstate(divide="ignore"):
            dis = (np.float32(1.0) / np.sqrt(deg)).astype(np.float32)
        dis[np.isinf(dis)] = 0.0
        w = ((dis[src] * wt).astype(np.float32) * dis[dst]).astype(np.float32)
    else:
        w = wt
    key, other = (src, dst) if transpose else (dst, src)
    order = np.argsort(key, kind="stable")  # ascending edge order inside a row; loops were appended last
    counts = np.bincount(key, minlength=N)
    rowptr = np.zeros(N + 1, dtype=np.int32)
    rowptr[1:] = np.cumsum(counts)
    return rowptr, other[order].astype(np.int32), w[order].astype(np.float32)


def incidence_csr(pipe_ends, num_nodes):
    """Items 2p + role (role 0 = u, 1 = v) grouped by node, ascending."""
    flat = pipe_ends.reshape(-1)
    order = np.argsort(flat, kind="stable")
    counts = np.bincount(flat, minlength=num_nodes)
    rowptr = np.zeros(num_nodes + 1, dtype=np.int32)
    rowptr[1:] = np.cumsum(counts)
    return rowptr, order.astype(np.int32)
