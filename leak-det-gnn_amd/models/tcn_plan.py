"""Row plan of the shared-window residual builder (SURVEY §8 f rank 1).

build_residual_sequence_from_segment (reference utils.py:169-216) runs the frozen
NormalPredictorTCN (predictor.py:55-81) on L_det sliding windows of length L_pred taken
from one (L_pred + L_det)-step segment and keeps only the last output of each.  The TCN
is causal with zero left padding per window, so windows cannot simply be merged — but an
activation of conv layer l at window-internal position t depends only on the window's
inputs in [t - R_l, t] (R_l = cumulative dilation reach, 2 d per conv), so for t >= R_l it
equals the activation of ONE segment-wide pass at segment position k + t (k = window
start).  The plan therefore computes, per conv layer:
  * shared rows: every segment position p of a single pass over the whole segment;
  * special rows: for each window k, only the positions t < R_l that the window's final
    output actually reaches (backward reachability from t = L_pred - 1),
and wires each row's three taps (t, t - d, t - 2d) to a shared row, a special row of the
previous layer, or zero.  For the default TCN (4 blocks, d = 1, 2, 4, 8, kernel 3) and
L_pred = L_det = 36 this is 72 shared + 24 special rows per window per 8 conv layers
instead of 36 * 36 * 8 window positions — the same arithmetic per row, ~8x fewer rows.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np


@dataclass
class ConvPlan:
    dilation: int
    rows: int                 # rows per segment: seg_len shared + n_win * len(special_t)
    special_t: List[int]      # window-internal positions computed per window (t < reach)
    taps: np.ndarray          # (rows, 3) int32: input row (in the previous buffer) of tap j = t - j*d, or -1
    res: np.ndarray           # (rows,) int32: residual row in the block-input buffer (conv2 only), or -1


@dataclass
class TcnPlan:
    seg_len: int
    l_pred: int
    n_win: int
    convs: List[ConvPlan]     # 2 per block, in order
    out_rows: np.ndarray      # (n_win,) row of each window's last position in the final buffer


def _row_of(layer_special: Sequence[int], seg_len: int, k: int, t: int, reach: int) -> int:
    """Row index, in a buffer with `layer_special` positions per window, of window k's
    internal position t (reach = R of that buffer's layer)."""
    if t < 0:
        return -1
    if t >= reach:
        return k + t  # shared row = segment position
    return seg_len + k * len(layer_special) + layer_special.index(t)


def make_plan(l_pred: int, l_det: int, dilations: Sequence[int] = (1, 2, 4, 8), kernel: int = 3) -> TcnPlan:
    if kernel != 3:
        raise NotImplementedError("the shared-window plan is written for kernel_size 3")
    seg_len, n_win = l_pred + l_det, l_det
    layers = [d for d in dilations for _ in range(2)]  # conv1, conv2 of each block
    # reach after each conv (R of its output); the input projection has reach 0
    reach_out = []
    r = 0
    for d in layers:
        r += 2 * d
        reach_out.append(r)
    # backward reachability of window-internal positions from the last one (fixed point):
    # a conv layer reads its taps from the layer below; a block's conv2 also reads the
    # block input (output of the layer two below) at the same positions (residual)
    need = [set() for _ in layers]
    need[-1] = {l_pred - 1}
    changed = True
    while changed:
        changed = False
        for li in range(len(layers) - 1, 0, -1):
            d = layers[li]
            taps = {t - j * d for t in need[li] for j in range(3) if t - j * d >= 0}
            if not taps <= need[li - 1]:
                need[li - 1] |= taps
                changed = True
            if li % 2 == 1 and li >= 2 and not need[li] <= need[li - 2]:
                need[li - 2] |= need[li]
                changed = True
    special = [sorted(t for t in need[li] if t < reach_out[li]) for li in range(len(layers))]
    convs: List[ConvPlan] = []
    for li, d in enumerate(layers):
        rows = seg_len + n_win * len(special[li])
        taps = np.full((rows, 3), -1, dtype=np.int32)
        res = np.full((rows,), -1, dtype=np.int32)
        prev_special = special[li - 1] if li > 0 else []
        prev_reach = reach_out[li - 1] if li > 0 else 0
        blk_special = special[li - 2] if li >= 2 else []
        blk_reach = reach_out[li - 2] if li >= 2 else 0
        for p in range(seg_len):  # shared rows: one pass over the whole segment
            for j in range(3):
                taps[p, j] = p - j * d if p - j * d >= 0 else -1
            if li % 2 == 1:
                res[p] = p
        for k in range(n_win):
            for i, t in enumerate(special[li]):
                row = seg_len + k * len(special[li]) + i
                for j in range(3):
                    taps[row, j] = _row_of(prev_special, seg_len, k, t - j * d, prev_reach)
                if li % 2 == 1:
                    res[row] = _row_of(blk_special, seg_len, k, t, blk_reach)
        convs.append(ConvPlan(d, rows, special[li], taps, res))
    last = len(layers) - 1
    out_rows = np.array([_row_of(special[last], seg_len, k, l_pred - 1, reach_out[last]) for k in range(n_win)],
                        dtype=np.int32)
    return TcnPlan(seg_len, l_pred, n_win, convs, out_rows)


def emulate(plan: TcnPlan, predictor, noisy_seg, time_seg):
    """Pure-torch execution of the plan (test oracle for the HIP path; any device)."""
    import torch
    import torch.nn.functional as F
    B = noisy_seg.shape[0]
    x = torch.cat([noisy_seg, time_seg], -1)                       # (B, seg, S+9)
    W0 = predictor.input_proj.weight[:, :, 0]
    h = x @ W0.t() + predictor.input_proj.bias                     # (B, seg, C) shared rows only
    C = h.shape[-1]
    zero = torch.zeros(B, 1, C, dtype=h.dtype, device=h.device)
    bufs = [h]
    for li, cp in enumerate(plan.convs):
        blk = predictor.tcn[li // 2]
        conv = (blk.conv1 if li % 2 == 0 else blk.conv2).conv
        norm = blk.norm1 if li % 2 == 0 else blk.norm2
        prev = torch.cat([bufs[-1], zero], 1)                      # row -1 -> zero row (last)
        taps = torch.as_tensor(cp.taps, dtype=torch.long, device=h.device)
        g = prev[:, taps]                                          # (B, rows, 3, C): taps t, t-d, t-2d
        # conv weight (C_out, C_in, 3): kernel index 2 is tap t, 1 is t-d, 0 is t-2d
        Wt = conv.weight.flip(-1).permute(0, 2, 1).reshape(C, 3 * C)
        y = g.reshape(B, cp.rows, 3 * C) @ Wt.t() + conv.bias
        y = F.relu(F.layer_norm(y, (C,), norm.weight, norm.bias, norm.eps))
        if li % 2 == 1:
            blk_in = torch.cat([bufs[-2], zero], 1)
            y = blk_in[:, torch.as_tensor(cp.res, dtype=torch.long, device=h.device)] + y
        bufs.append(y)
    final = bufs[-1][:, torch.as_tensor(plan.out_rows, dtype=torch.long, device=h.device)]  # (B, n_win, C)
    y_hat = final @ predictor.head.weight.t() + predictor.head.bias
    return noisy_seg[:, plan.l_pred:, :] - y_hat


# --------------------------------------------------------------------------------------
# Device executor (HIP): lg_tcn_conv_fwd per conv layer.
# --------------------------------------------------------------------------------------
_PLAN_CACHE: Dict[Tuple[int, int], TcnPlan] = {}


def plan_for(l_pred: int, l_det: int) -> TcnPlan:
    key = (int(l_pred), int(l_det))
    if key not in _PLAN_CACHE:
        _PLAN_CACHE[key] = make_plan(*key)
    return _PLAN_CACHE[key]


def fast_path_eligible(predictor) -> bool:
    """True for a NormalPredictorTCN of the default shape in eval mode (the frozen
    predictor of train_detector / the evaluators): kernel 3, dilations 1, 2, 4, ...,
    128 channels.  Anything else goes through the stock module."""
    tcn = getattr(predictor, "tcn", None)
    proj = getattr(predictor, "input_proj", None)
    if tcn is None or proj is None or getattr(predictor, "head", None) is None or predictor.training:
        return False
    if proj.out_channels != 128 or proj.kernel_size != (1,):
        return False
    for i, blk in enumerate(tcn):
        for conv in (blk.conv1.conv, blk.conv2.conv):
            if (conv.kernel_size != (3,) or conv.dilation != (2 ** i,) or conv.in_channels != 128
                    or conv.out_channels != 128 or conv.padding != (2 * 2 ** i,) or conv.bias is None):
                return False
    return len(tcn) == 4


class _DevicePlan:
    def __init__(self, plan: TcnPlan, device) -> None:
        import torch
        self.tables = []
        for cp in plan.convs:
            t = np.concatenate([cp.taps, cp.res[:, None]], axis=1).astype(np.int32)
            self.tables.append(torch.from_numpy(np.ascontiguousarray(t)).to(device))
        self.out_rows = torch.from_numpy(plan.out_rows.astype(np.int64)).to(device)


def _packed_weights(predictor, device):
    """Packed conv weights, cached on the module and rebuilt if any parameter changed."""
    import torch
    from . import _native as nat
    params = [p for blk in predictor.tcn for p in (blk.conv1.conv.weight, blk.conv2.conv.weight)]
    stamp = tuple((p.data_ptr(), p._version) for p in params)
    cache = getattr(predictor, "_lg_tcn_packed", None)
    if cache is not None and cache[0] == stamp:
        return cache[1]
    lib = nat.load_library()
    n = lib.lg_tcn_packed_weight_floats(128)
    packed = []
    for p in params:
        w = p.detach().contiguous()
        nat.require_device(w)
        out = torch.empty(n, dtype=torch.float32, device=device)
        nat.check(lib.lg_tcn_pack_weight(nat.ptr(w), nat.ptr(out), 128, nat.stream_of(w)), "lg_tcn_pack_weight")
        packed.append(out)
    object.__setattr__(predictor, "_lg_tcn_packed", (stamp, packed))
    return packed


def tcn_residual(predictor, noisy_seg, time_seg, l_pred: int, l_det: int):
    """residual (B, l_det, S) = noisy_seg[:, l_pred:] - predictor(window k) for every
    window k, computed on the GPU with one shared-window pass per segment
    (lg_tcn_conv_fwd for the 8 convs; input projection and head as plain GEMMs).
    Matches the reference's per-window evaluation within fp32 rounding."""
    import torch
    from . import _native as nat
    if not fast_path_eligible(predictor):
        raise ValueError("tcn_residual needs a default-shape NormalPredictorTCN in eval mode")
    B, T, S = noisy_seg.shape
    if T != l_pred + l_det:
        raise ValueError(f"segment length {T} != l_pred + l_det = {l_pred + l_det}")
    device = noisy_seg.device
    nat.require_device(noisy_seg.contiguous())
    lib = nat.load_library()
    plan = plan_for(l_pred, l_det)
    dplans = getattr(predictor, "_lg_tcn_plans", None)
    if dplans is None:
        dplans = {}
        object.__setattr__(predictor, "_lg_tcn_plans", dplans)
    key = (l_pred, l_det, str(device))
    if key not in dplans:
        dplans[key] = _DevicePlan(plan, device)
    dp = dplans[key]
    packed = _packed_weights(predictor, device)

    C = 128
    with torch.no_grad():
        x = torch.cat([noisy_seg, time_seg], dim=-1).reshape(B * T, -1)
        proj = predictor.input_proj
        h = torch.addmm(proj.bias, x, proj.weight[:, :, 0].t()).contiguous()  # (B*T, C) rows = segment positions
        bufs = [(h, T)]
        stream = nat.stream_of(h)
        for li, cp in enumerate(plan.convs):
            blk = predictor.tcn[li // 2]
            conv = blk.conv1.conv if li % 2 == 0 else blk.conv2.conv
            norm = blk.norm1 if li % 2 == 0 else blk.norm2
            prev, rows_prev = bufs[-1]
            blk_in, rows_blk = bufs[-2] if li % 2 == 1 else (None, 0)
            out = torch.empty(B * cp.rows, C, dtype=torch.float32, device=device)
            nat.check(lib.lg_tcn_conv_fwd(nat.ptr(prev), nat.ptr(blk_in), nat.ptr(dp.tables[li]), nat.ptr(packed[li]),
                                          nat.ptr(conv.bias), nat.ptr(norm.weight), nat.ptr(norm.bias),
                                          float(norm.eps), nat.ptr(out), B, rows_prev, rows_blk, cp.rows, C, stream),
                      "lg_tcn_conv_fwd")
            bufs.append((out, cp.rows))
        last, rows_last = bufs[-1]
        final = last.view(B, rows_last, C).index_select(1, dp.out_rows)                 # (B, l_det, C)
        y_hat = torch.addmm(predictor.head.bias, final.reshape(B * l_det, C), predictor.head.weight.t())
        return noisy_seg[:, l_pred:, :] - y_hat.view(B, l_det, S)
