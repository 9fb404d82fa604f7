"""ORACLE (test infrastructure only) — the counter-based dropout hash of libleakgnn,
restated in numpy so train-mode masks can be replayed exactly on the host.

Restates common.h lg_hash / lg_dropout (product code; dropout RNG cannot match
torch's bitwise — SURVEY §7 "Dropout RNG cannot match bitwise" — so the product
defines its own counter-based stream and the tests pin it here):
  z = seed ^ (salt << 32) ^ (idx * 0x9E3779B97F4A7C15);  z += 0x9E3779B97F4A7C15
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9;  z = (z ^ (z >> 27)) * 0x94D049BB133111EB;  z ^= z >> 31
  u = (z >> 40) / 2^24;   keep <=> u >= p;   kept values scaled by 1 / (1 - p)
"""
from __future__ import annotations

import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def keep_mask(seed: int, salt: int, idx: np.ndarray, p: float) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) ^ (np.uint64(salt) << np.uint64(32)) ^ (idx.astype(np.uint64) * _G)
        z = z + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) / 16777216.0
    return u.astype(np.float32) >= np.float32(p)
