"""ORACLE (test infrastructure only) — frozen-predictor residual builder on torch CPU.

Restates, per window exactly as the reference evaluates it:
  NormalPredictorTCN.forward   (reference models/predictor.py:55-81)
      h = input_proj(cat[x, x_time]^T)                      1x1 Conv1d
      4 x TCNBlock (predictor.py:31-52), dilation 2^i:
          h = h + Drop(ReLU(LN(CausalConv(Drop(ReLU(LN(CausalConv(h))))))))
          CausalConv (predictor.py:17-28): Conv1d, padding (k-1) d on both sides, the
          right (k-1) d outputs cropped -> zero LEFT padding of each window
      y = head(h[:, :, -1])
  build_residual_sequence_from_segment (reference models/utils.py:169-216)
      residual[b, k] = noisy[b, l_pred + k] - y(window noisy[b, k:k+l_pred], time[b, k:k+l_pred])
Dropout is the identity (the predictor is frozen in eval mode, utils.py:189).

Pinned by tests/golden/predictor.npz and tests/golden/residual.npz, both produced by
the reference's own utils.build_residual_sequence_from_segment (oracle/make_golden.py).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this module.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def tcn_forward(sd: Dict[str, torch.Tensor], x: torch.Tensor, x_time: torch.Tensor, num_blocks: int = 4,
                eps: float = 1e-5) -> torch.Tensor:
    """One NormalPredictorTCN forward on (W, L, S) windows -> (W, S)."""
    h = F.conv1d(torch.cat([x, x_time], dim=-1).transpose(1, 2), sd["input_proj.weight"], sd["input_proj.bias"])
    for i in range(num_blocks):
        d = 2 ** i
        blk_in = h
        for j in (1, 2):
            w, b = sd[f"tcn.{i}.conv{j}.conv.weight"], sd[f"tcn.{i}.conv{j}.conv.bias"]
            pad = (w.shape[-1] - 1) * d
            y = F.conv1d(h, w, b, dilation=d, padding=pad)[..., :-pad]
            y = F.layer_norm(y.transpose(1, 2), (y.shape[1],), sd[f"tcn.{i}.norm{j}.weight"],
                             sd[f"tcn.{i}.norm{j}.bias"], eps)
            h = F.relu(y).transpose(1, 2)
        h = blk_in + h
    return h[:, :, -1] @ sd["head.weight"].t() + sd["head.bias"]


def residual_ref(sd: Dict[str, torch.Tensor], noisy_seg: torch.Tensor, time_seg: torch.Tensor, l_pred: int,
                 l_det: int) -> torch.Tensor:
    """(B, l_pred + l_det, S) segments -> (B, l_det, S) residuals, one window at a time."""
    B, T, S = noisy_seg.shape
    assert T == l_pred + l_det
    out = torch.empty(B, l_det, S, dtype=noisy_seg.dtype)
    with torch.no_grad():
        for k in range(l_det):
            y = tcn_forward(sd, noisy_seg[:, k:k + l_pred], time_seg[:, k:k + l_pred])
            out[:, k] = noisy_seg[:, l_pred + k] - y
    return out
