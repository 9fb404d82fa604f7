"""ORACLE (test infrastructure only) — the counter-based dropout hash of libleakgnn,
restated in numpy so train-mode masks can be replayed exactly on the host.

Restates leak-det-gnn_amd/csrc/common.h (lg_mix32 / lg_dropout_key / lg_keep).  The
product defines its own counter-based stream because dropout RNG cannot match
torch's bitwise (SURVEY §7 "Dropout RNG cannot match bitwise"); the tests pin it here:
  mix32(x)  = lowbias32: x ^= x>>16; x *= 0x7feb352d; x ^= x>>15; x *= 0x846ca68b; x ^= x>>16
  key       = mix32(lo32(seed) ^ mix32(hi32(seed) ^ salt * 0x9E3779B9))
  h(idx)    = mix32(lo32(idx) * 0x9E3779B9 ^ key ^ hi32(idx) * 0x85EBCA6B)     (uint32 wrap-around)
  keep      <=> (h >> 8) / 2^24 >= p ;  kept values scaled by 1 / (1 - p)
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
