"""ORACLE (test infrastructure only) — the counter-based dropout hash of libleakgnn,
restated in numpy so train-mode masks can be replayed exactly on the host.

Restates leak-det-gnn_amd/csrc/common.h (lg_mix32 / lg_dropout_key / lg_keep).  The
product defines its own counter-based stream because dropout RNG cannot match
torch's bitwise (SURVEY §7 "Dropout RNG cannot match bitwise"); the tests pin it here:
  mix32(x)  = lowbias32: x ^= x>>16; x *= 0x7feb352d; x ^= x>>15; x *= 0x846ca68b; x ^= x>>16
  key       = mix32(lo32(seed) ^ mix32(hi32(seed) ^ salt * 0x9E3779B9))
  h(idx)    = mix32(lo32(idx) * 0x9E3779B9 ^ key ^ hi32(idx) * 0x85EBCA6B)     (uint32 wrap-around)
  keep      <=> (h >> 8) / 2^24 >= p ;  kept values scaled by 1 / (1 - p)
keep_mask is the NoLeakHead's rule; the node init (salt 0), the GCN layers and the EdgeHead
draw row streams (row_stream_mask / edge_stream_mask below).
"""
from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFF)


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & _M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M
    x ^= x >> np.uint64(16)
    return x


def dropout_key(seed: int, salt: int) -> int:
    lo, hi = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    inner = _mix32(np.array([hi ^ ((salt * 0x9E3779B9) & 0xFFFFFFFF)], dtype=np.uint64))[0]
    return int(_mix32(np.array([lo ^ int(inner)], dtype=np.uint64))[0])


def keep_mask(seed: int, salt: int, idx: np.ndarray, p: float) -> np.ndarray:
    key = np.uint64(dropout_key(seed, salt))
    idx = idx.astype(np.uint64)
    lo = idx & _M
    hi = idx >> np.uint64(32)
    x = ((lo * np.uint64(0x9E3779B9)) & _M) ^ key ^ ((hi * np.uint64(0x85EBCA6B)) & _M)
    h = _mix32(x)
    u = (h >> np.uint64(8)).astype(np.float64) / 16777216.0
    return u.astype(np.float32) >= np.float32(p)


# ---- row-stream dropout of the fused GCN forward (common.h lg_row_stream_seed) ----
#   seed(row, q) = mix32(mix32(lo32(row) * 0x9E3779B9 ^ key) ^ hi32(row) * 0x85EBCA6B ^ q * 0x632BE5AB),
#                  0 replaced by 0x6D2B79F5
#   lane group q of a row owns channels 16 mt + 4 q + reg (t = 4 mt + reg); its stream
#   steps xorshift32 (s ^= s<<13; s ^= s>>17; s ^= s<<5) once per channel PAIR (t >> 1);
#   channel t keeps iff its 16-bit half (low for even t, high for odd t) >= rint(p * 2^16).
def _xorshift32(s: np.ndarray) -> np.ndarray:
    s = s ^ ((s << np.uint64(13)) & _M)
    s = s ^ (s >> np.uint64(17))
    return s ^ ((s << np.uint64(5)) & _M)


def row_stream_seed(key: int, rows: np.ndarray, q: int) -> np.ndarray:
    rows = rows.astype(np.uint64)
    lo, hi = rows & _M, rows >> np.uint64(32)
    a = _mix32(((lo * np.uint64(0x9E3779B9)) & _M) ^ np.uint64(key))
    s = _mix32(a ^ ((hi * np.uint64(0x85EBCA6B)) & _M) ^ np.uint64((q * 0x632BE5AB) & 0xFFFFFFFF))
    return np.where(s == 0, np.uint64(0x6D2B79F5), s)


def keep_threshold16(p: float) -> int:
    """rint(float32(p) * 2^16) (round half to even, as rintf)."""
    return int(np.rint(np.float32(p) * np.float32(65536.0)))


def row_stream_mask(seed: int, salt: int, rows: np.ndarray, D: int, p: float) -> np.ndarray:
    """Keep mask [len(rows), D] of the fused GCN forward for the given global rows."""
    key = dropout_key(seed, salt)
    thr = np.uint64(keep_threshold16(p))
    rows = np.asarray(rows, dtype=np.uint64).reshape(-1)
    out = np.zeros((rows.size, D), dtype=bool)
    for q in range(4):
        s = row_stream_seed(key, rows, q)
        for t in range(D // 16 * 4):
            if t % 2 == 0:
                s = _xorshift32(s)
            u16 = (s & np.uint64(0xFFFF)) if t % 2 == 0 else (s >> np.uint64(16))
            out[:, 16 * (t // 4) + 4 * q + (t % 4)] = u16 >= thr
    return out


# ---- row-stream dropout of the fused EdgeHead forward (edge.hip k_edge_fwd) ----
#   hidden block nh (units [32 nh, 32 nh + 32)) x lane group q of a row draws the stream
#   row_stream_seed(key, row, 4 nh + q) and owns units 32 nh + 16 i + 4 q + reg in
#   t = 4 i + reg order (i, reg < 2, 4); same xorshift / 16-bit-half rule as row_stream_mask.
def edge_stream_mask(seed: int, salt: int, rows: np.ndarray, p: float, hidden: int = 128) -> np.ndarray:
    """Keep mask [len(rows), hidden] of the EdgeHead hidden layer for the given pipe rows
    (row = b * P + p)."""
    key = dropout_key(seed, salt)
    thr = np.uint64(keep_threshold16(p))
    rows = np.asarray(rows, dtype=np.uint64).reshape(-1)
    out = np.zeros((rows.size, hidden), dtype=bool)
    for nh in range(hidden // 32):
        for q in range(4):
            s = row_stream_seed(key, rows, 4 * nh + q)
            for t in range(8):
                if t % 2 == 0:
                    s = _xorshift32(s)
                u16 = (s & np.uint64(0xFFFF)) if t % 2 == 0 else (s >> np.uint64(16))
                out[:, 32 * nh + 16 * (t // 4) + 4 * q + (t % 4)] = u16 >= thr
    return out
