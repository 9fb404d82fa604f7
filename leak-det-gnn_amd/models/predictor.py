"""Frozen normal-state predictors that feed the detector (caller side of the hot path).

Same constructors, forward signatures and state-dict keys as reference
models/predictor.py (CausalConv1d :17-28, TCNBlock :31-52, NormalPredictorTCN
:55-81, NormalPredictorGRU :84-111).  They contain no message passing and run on
stock PyTorch-ROCm (MIOpen conv / GRU); SURVEY §8(f) ranks a fused TCN kernel as
the next row after the GNN path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class CausalConv1d(nn.Module):
    """Conv1d padded on both sides by (k-1)*dilation, right pad cropped: y[t] sees x[<= t]."""

    def __init__(self, in_ch: int, out_ch: int, kernel_size: int, dilation: int = 1) -> None:
        super().__init__()
        self.pad = (kernel_size - 1) * dilation
        self.conv = nn.Conv1d(in_ch, out_ch, kernel_size, dilation=dilation, padding=self.pad)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.conv(x)
        return y[..., :-self.pad] if self.pad > 0 else y


class TCNBlock(nn.Module):
    """x + [conv -> LayerNorm(C) -> ReLU -> Dropout] x 2, on (B, C, L)."""

    def __init__(self, channels: int, kernel_size: int, dilation: int, dropout: float) -> None:
        super().__init__()
        self.conv1 = CausalConv1d(channels, channels, kernel_size, dilation=dilation)
        self.conv2 = CausalConv1d(channels, channels, kernel_size, dilation=dilation)
        self.dropout = nn.Dropout(dropout)
        self.norm1 = nn.LayerNorm(channels)
        self.norm2 = nn.LayerNorm(channels)

    def _stage(self, conv: CausalConv1d, norm: nn.LayerNorm, h: torch.Tensor) -> torch.Tensor:
        h = norm(conv(h).transpose(1, 2))
        return self.dropout(F.relu(h)).transpose(1, 2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x + self._stage(self.conv2, self.norm2, self._stage(self.conv1, self.norm1, x))


class NormalPredictorTCN(nn.Module):
    def __init__(self, num_sensors: int, time_dim: int = 9, hidden_channels: int = 128, kernel_size: int = 3,
                 num_blocks: int = 4, dropout: float = 0.1) -> None:
        super().__init__()
        self.num_sensors = int(num_sensors)
        self.time_dim = int(time_dim)
        self.input_proj = nn.Conv1d(self.num_sensors + self.time_dim, hidden_channels, kernel_size=1)
        self.tcn = nn.Sequential(*[TCNBlock(hidden_channels, kernel_size, 2 ** i, dropout) for i in range(num_blocks)])
        self.head = nn.Linear(hidden_channels, self.num_sensors)

    def forward(self, x: torch.Tensor, x_time: torch.Tensor) -> torch.Tensor:
        h = self.input_proj(torch.cat([x, x_time], dim=-1).transpose(1, 2))  # (B, hidden, L)
        return self.head(self.tcn(h)[:, :, -1])                               # (B, S)


class NormalPredictorGRU(nn.Module):
    def __init__(self, num_sensors: int, time_dim: int = 9, hidden_size: int = 128, num_layers: int = 2,
                 dropout: float = 0.1) -> None:
        super().__init__()
        self.num_sensors = int(num_sensors)
        self.time_dim = int(time_dim)
        self.gru = nn.GRU(input_size=self.num_sensors + self.time_dim, hidden_size=hidden_size,
                          num_layers=num_layers, batch_first=True, dropout=dropout if num_layers > 1 else 0.0)
        self.head = nn.Linear(hidden_size, self.num_sensors)

    def forward(self, x: torch.Tensor, x_time: torch.Tensor) -> torch.Tensor:
        out, _ = self.gru(torch.cat([x, x_time], dim=-1))
        return self.head(out[:, -1, :])
