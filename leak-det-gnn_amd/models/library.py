"""torch.library registration of the libleakgnn operators (namespace ``leakgnn``).

SURVEY §8(b): the hot path sits behind registered PyTorch operators whose bodies call
the C ABI (include/leakgnn.h) on torch's current HIP stream, with autograd formulas in
Python, so torch.compile / torch.export / any dispatcher-level caller sees them as
ordinary ops (fake / meta implementations give output shapes without running kernels).

  leakgnn::gcn_conv            PyG GCNConv.forward (detector.py:163,199): Ahat (x W^T) + b
  leakgnn::mean_pool           PyG global_mean_pool over B equal windows (detector.py:215)
  leakgnn::sensor_proj         sensor_to_node on the sensor rows (detector.py:184-189)
  leakgnn::gru_encoder         SharedSensorGRUEncoder's GRU (detector.py:60-73)
  leakgnn::gnn_trunk           node init + L x [GCNConv, ReLU, Dropout] (detector.py:178-201)
  leakgnn::detector_heads      pipe gather + EdgeHead + mean pool + NoLeakHead
                               (detector.py:76-102, 206-218)
and one ``*_backward`` op per differentiable op (registered autograd formulas call them).

Every op takes plain tensors (the graph CSR and its node tables are inputs, not Python
objects) and fp32 CUDA tensors; there is no CPU kernel, so a CPU call raises.  Dropout
seeds are a 1-element int64 tensor: a CPU tensor's value, or - under HIP-graph capture -
a device tensor whose ADDRESS the kernels read at launch (LG_SALT_SEED_PTR), so replays
draw fresh masks.
"""
from __future__ import annotations

import contextlib
import ctypes

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _native as nat
from ._native import check, load_library, ptr, stream_of
from .ops import (EDGE_HEAD_SALT, GCN_BWD_NM_EXTRA_FLAGS, GCN_FWD_DENSE_EXTRA_FLAGS, GCN_FWD_NM_EXTRA_FLAGS,
                  NM_MAX_BYTES, NOLEAK_HEAD_SALT, _check_d, _timed)

NS = "leakgnn"


def _seed_args(seed: Tensor) -> Tuple[int, int]:
    """(seed value or device address, salt bits) of a dropout seed tensor."""
    if seed.is_cuda:
        return seed.data_ptr(), nat.LG_SALT_SEED_PTR
    return int(seed.item()), 0


def _req(*ts: Optional[Tensor]) -> None:
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("leakgnn ops run only on a ROCm GPU (tensor on %s); there is no CPU path" % t.device)
        if t.is_floating_point() and t.dtype != torch.float32:
            raise TypeError(f"leakgnn ops compute in fp32, got {t.dtype} (cast the inputs with .float())")


def _c(t: Optional[Tensor]) -> Optional[Tensor]:
    return None if t is None else t.contiguous()


# ============================================================================ gcn_conv
# GCNConv's single-graph kernels at D = 64: True (default) = the node-table row tiles
# lg_gcn_{fwd,bwd}_rows (split-bf16 MFMA, fp32-level accuracy; at C5 17.7 / 40.4 us against
# 26.7 / 50.5 us, profiles/r03/r03ac), False = window-major lg_gcn_fwd / lg_gcn_bwd (exact
# fp32 MFMA, and the D = 32 path)
_ROWS = True


def _use_rows(Ntot: int, D: int) -> bool:
    """The row-tile kernels take the graph only when its node-major activation fits one launch's
    32-bit buffer offsets (N * D * 4 <= ops.NM_MAX_BYTES, ~8.4M nodes at D = 64); larger graphs
    go to lg_gcn_fwd / lg_gcn_bwd (window-major, up to kLgMaxRows rows)."""
    return D == 64 and _ROWS and Ntot * D * 4 <= NM_MAX_BYTES

@torch.library.custom_op(f"{NS}::gcn_conv", mutates_args=(), device_types="cuda")
def gcn_conv(x: Tensor, weight: Tensor, bias: Optional[Tensor], rowptr: Tensor, col: Tensor, w: Tensor,
             rowptr_t: Tensor, col_t: Tensor, w_t: Tensor, nodetab: Tensor, pairs: Tensor, nodetab_t: Tensor,
             pairs_t: Tensor) -> Tensor:
    """y = Ahat (x W^T) + b on one graph: lg_gcn_fwd_rows (D = 64: 16-node tiles off the node
    table nodetab / pairs of GCNGraph) or lg_gcn_fwd (D = 32, or `_ROWS = False`: exact fp32
    MFMA over the gcn_norm'ed CSR rowptr / col / w of lg_graph_build)."""
    lib = load_library()
    x, weight, bias = _c(x), _c(weight), _c(bias)
    _req(x, weight, bias)
    Ntot, D = x.shape
    _check_d(D)
    if weight.shape != (D, D):
        raise NotImplementedError("GCNConv kernels need in_channels == out_channels")
    y = torch.empty_like(x)
    flags = nat.LG_F_BIAS if bias is not None else 0
    with _timed("gcn_fwd", x.device):
        if _use_rows(Ntot, D):
            check(lib.lg_gcn_fwd_rows(ptr(nodetab), ptr(pairs), ptr(x), ptr(weight), ptr(bias), ptr(y), Ntot, D, flags,
                                      stream_of(x)), "lg_gcn_fwd_rows")
        else:
            check(lib.lg_gcn_fwd(ptr(rowptr), ptr(col), ptr(w), ptr(x), ptr(weight), ptr(bias), ptr(y), 1, Ntot, D,
                                 col.numel(), flags, 0.0, 0, 0, stream_of(x)), "lg_gcn_fwd")
    return y


@gcn_conv.register_fake
def _(x, weight, bias, rowptr, col, w, rowptr_t, col_t, w_t, nodetab, pairs, nodetab_t, pairs_t):
    return torch.empty_like(x)


@torch.library.custom_op(f"{NS}::gcn_conv_backward", mutates_args=(), device_types="cuda")
def gcn_conv_backward(dy: Tensor, x: Tensor, weight: Tensor, rowptr_t: Tensor, col_t: Tensor,
                      w_t: Tensor, nodetab_t: Tensor, pairs_t: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """(dx, dW, db) of gcn_conv (lg_gcn_bwd over the transposed CSR; lg_gcn_bwd_rows over the
    transposed node table when the row-tile kernels are selected)."""
    lib = load_library()
    dy, x, weight = _c(dy), _c(x), _c(weight)
    _req(dy, x, weight)
    Ntot, D = x.shape
    dx = torch.empty_like(x)
    dW = torch.empty_like(weight)
    db = torch.empty(D, device=x.device, dtype=x.dtype)
    with _timed("gcn_bwd", x.device):
        if _use_rows(Ntot, D):
            ws = torch.empty(int(lib.lg_gcn_bwd_nm_workspace_bytes(D)), device=x.device, dtype=torch.uint8)
            check(lib.lg_gcn_bwd_rows(ptr(nodetab_t), ptr(pairs_t), ptr(dy), ptr(x), ptr(weight), ptr(dx), ptr(dW),
                                      ptr(db), Ntot, D, ptr(ws), ws.numel(), stream_of(x)), "lg_gcn_bwd_rows")
        else:
            ws = torch.empty(int(lib.lg_gcn_bwd_workspace_bytes(D)), device=x.device, dtype=torch.uint8)
            check(lib.lg_gcn_bwd(ptr(rowptr_t), ptr(col_t), ptr(w_t), ptr(dy), None, ptr(x), ptr(weight), ptr(dx),
                                 ptr(dW), ptr(db), None, None, 1, Ntot, D, col_t.numel(), 0, 1.0, 1.0, ptr(ws), ws.numel(),
                                 stream_of(x)), "lg_gcn_bwd")
    return dx, dW, db


@gcn_conv_backward.register_fake
def _(dy, x, weight, rowptr_t, col_t, w_t, nodetab_t, pairs_t):
    return torch.empty_like(x), torch.empty_like(weight), x.new_empty(x.shape[1])


def _gcn_conv_setup(ctx, inputs, output):
    x, weight, bias, _, _, _, rowptr_t, col_t, w_t, _, _, nodetab_t, pairs_t = inputs
    ctx.has_bias = bias is not None
    ctx.save_for_backward(x, weight, rowptr_t, col_t, w_t, nodetab_t, pairs_t)


def _gcn_conv_bwd(ctx, dy):
    x, weight, rowptr_t, col_t, w_t, nodetab_t, pairs_t = ctx.saved_tensors
    dx, dW, db = torch.ops.leakgnn.gcn_conv_backward(dy, x, weight, rowptr_t, col_t, w_t, nodetab_t, pairs_t)
    return (dx, dW, (db if ctx.has_bias else None)) + (None,) * 10


gcn_conv.register_autograd(_gcn_conv_bwd, setup_context=_gcn_conv_setup)


# ============================================================================ spmm_cols
# GCNConv's general path (models/gcn.py): widths other than the fused kernels' 32 / 64, or
# in_channels != out_channels.  The propagate runs on lg_spmm_cols (any column count, bias
# fused), the transform on a library GEMM.
@torch.library.custom_op(f"{NS}::spmm_cols", mutates_args=(), device_types="cuda")
def spmm_cols(x: Tensor, bias: Optional[Tensor], rowptr: Tensor, col: Tensor, w: Tensor, rowptr_t: Tensor,
              col_t: Tensor, w_t: Tensor) -> Tensor:
    """y = Ahat x (+ bias) for x [N][C], any C (lg_spmm_cols over the gcn_norm'ed CSR)."""
    lib = load_library()
    x, bias = _c(x), _c(bias)
    _req(x, bias)
    N, C = x.shape
    y = torch.empty_like(x)
    with _timed("spmm_cols", x.device):
        check(lib.lg_spmm_cols(ptr(rowptr), ptr(col), ptr(w), ptr(x), C, ptr(bias), ptr(y), C, N, C, stream_of(x)),
              "lg_spmm_cols")
    return y


@spmm_cols.register_fake
def _(x, bias, rowptr, col, w, rowptr_t, col_t, w_t):
    return torch.empty_like(x)


def _spmm_cols_setup(ctx, inputs, output):
    _, bias, _, _, _, rowptr_t, col_t, w_t = inputs
    ctx.has_bias = bias is not None
    ctx.save_for_backward(rowptr_t, col_t, w_t)


def _spmm_cols_bwd(ctx, dy):
    rowptr_t, col_t, w_t = ctx.saved_tensors
    # dx = Ahat^T dy: the same propagate over the transposed CSR (its rows are the columns of Ahat)
    dx = torch.ops.leakgnn.spmm_cols(dy, None, rowptr_t, col_t, w_t, rowptr_t, col_t, w_t)
    return dx, (dy.sum(0) if ctx.has_bias else None), None, None, None, None, None, None


spmm_cols.register_autograd(_spmm_cols_bwd, setup_context=_spmm_cols_setup)


# ============================================================================ mean_pool
@torch.library.custom_op(f"{NS}::mean_pool", mutates_args=(), device_types="cuda")
def mean_pool(x: Tensor, B: int, N: int) -> Tensor:
    """global_mean_pool for batch = arange(B).repeat_interleave(N) (lg_mean_pool_fwd)."""
    lib = load_library()
    x = _c(x)
    _req(x)
    D = x.shape[-1]
    _check_d(D)
    out = torch.empty(B, D, device=x.device, dtype=torch.float32)
    check(lib.lg_mean_pool_fwd(ptr(x), ptr(out), B, N, D, stream_of(x)), "lg_mean_pool_fwd")
    return out


@mean_pool.register_fake
def _(x, B, N):
    return x.new_empty(B, x.shape[-1])


def _mean_pool_setup(ctx, inputs, output):
    ctx.BN = (inputs[1], inputs[2])


def _mean_pool_bwd(ctx, dout):
    B, N = ctx.BN
    return (dout / float(N)).unsqueeze(1).expand(B, N, dout.shape[-1]).reshape(B * N, -1), None, None


mean_pool.register_autograd(_mean_pool_bwd, setup_context=_mean_pool_setup)


# ============================================================================ sensor_proj
@torch.library.custom_op(f"{NS}::sensor_proj", mutates_args=(), device_types="cuda")
def sensor_proj(h_s: Tensor, weight: Tensor, bias: Tensor) -> Tensor:
    """sensor_to_node on the rows that carry a sensor (detector.py:160, 184-189): their
    Linear input is [h_s, 1], so proj = h_s W[:, :Ds]^T + (W[:, Ds] + b), one GEMM."""
    _req(h_s, weight, bias)
    B, S, Ds = h_s.shape
    D = weight.shape[0]
    with torch.autocast("cuda", enabled=False):
        return torch.addmm(weight[:, Ds] + bias, h_s.reshape(B * S, Ds), weight[:, :Ds].t()).view(B, S, D)


@sensor_proj.register_fake
def _(h_s, weight, bias):
    return h_s.new_empty(h_s.shape[0], h_s.shape[1], weight.shape[0])


@torch.library.custom_op(f"{NS}::sensor_proj_backward", mutates_args=(), device_types="cuda")
def sensor_proj_backward(dproj: Tensor, h_s: Tensor, weight: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """dh_s = dproj W[:, :Ds] (GEMM); dW (incl. the mask column) and db in one split-K
    MFMA kernel (lg_linear_dw) instead of a skinny-K (K = B*S) GEMM."""
    lib = load_library()
    dproj, h_s, weight = _c(dproj), _c(h_s), _c(weight)
    _req(dproj, h_s, weight)
    B, S, Ds = h_s.shape
    D = weight.shape[0]
    K = B * S
    d2, h2 = dproj.view(K, D), h_s.view(K, Ds)
    with torch.autocast("cuda", enabled=False):
        dh = (d2 @ weight[:, :Ds]).view(B, S, Ds)
    dW = torch.empty(D, Ds + 1, device=d2.device, dtype=torch.float32)
    db = torch.empty(D, device=d2.device, dtype=torch.float32)
    ws = torch.empty(int(lib.lg_linear_dw_workspace_bytes(K, D, Ds)), device=d2.device, dtype=torch.uint8)
    with _timed("linear_dw", d2.device):
        check(lib.lg_linear_dw(ptr(d2), ptr(h2), K, D, Ds, ptr(dW), ptr(db), ptr(ws), ws.numel(), stream_of(d2)), "lg_linear_dw")
    return dh, dW, db


@sensor_proj_backward.register_fake
def _(dproj, h_s, weight):
    return torch.empty_like(h_s), weight.new_empty(weight.shape), weight.new_empty(weight.shape[0])


def _sensor_proj_setup(ctx, inputs, output):
    h_s, weight, _ = inputs
    ctx.save_for_backward(h_s, weight)


def _sensor_proj_bwd(ctx, dproj):
    h_s, weight = ctx.saved_tensors
    dh, dW, db = torch.ops.leakgnn.sensor_proj_backward(dproj, h_s, weight)
    return (dh if ctx.needs_input_grad[0] else None), dW, db


sensor_proj.register_autograd(_sensor_proj_bwd, setup_context=_sensor_proj_setup)


# ============================================================================ gru_encoder
@torch.library.custom_op(f"{NS}::gru_encoder", mutates_args=(), device_types="cuda")
def gru_encoder(residual: Tensor, tfeat: Optional[Tensor], w_ih: Tensor, w_hh: Tensor, b_ih: Tensor, b_hh: Tensor,
                save: bool) -> Tuple[Tensor, Tensor, Tensor]:
    """(h_L (B, S, H), h_seq, gates): nn.GRU over the B*S sensor sequences, x_t =
    [residual[b, t, s], tfeat[b, t, :]] read in place (lg_gru_fwd).  save: keep h_t and
    the gate values of every step for the backward (else both are empty)."""
    lib = load_library()
    residual, tfeat, w_ih, w_hh, b_ih, b_hh = (_c(t) for t in (residual, tfeat, w_ih, w_hh, b_ih, b_hh))
    _req(residual, tfeat, w_ih, w_hh, b_ih, b_hh)
    B, L, S = residual.shape
    G, I = w_ih.shape
    H = w_hh.shape[1]
    if tfeat is not None and tuple(tfeat.shape) != (B, L, 9):
        raise ValueError(f"tfeat must be (B, L, 9), got {tuple(tfeat.shape)}")
    dev = residual.device
    h_seq = torch.empty(L, B * S, H, device=dev) if save else torch.empty(0, device=dev)
    gates = torch.empty(L, B * S, 4, H, device=dev) if save else torch.empty(0, device=dev)
    h_last = torch.empty(B, S, H, device=dev)
    with _timed("gru_fwd", dev):
        check(lib.lg_gru_fwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh),
                             ptr(h_seq) if save else None, ptr(gates) if save else None, ptr(h_last), B, L, S, I, H,
                             stream_of(residual)), "lg_gru_fwd")
    return h_last, h_seq, gates


@gru_encoder.register_fake
def _(residual, tfeat, w_ih, w_hh, b_ih, b_hh, save):
    B, L, S = residual.shape
    H = w_hh.shape[1]
    if save:
        return (residual.new_empty(B, S, H), residual.new_empty(L, B * S, H), residual.new_empty(L, B * S, 4, H))
    return residual.new_empty(B, S, H), residual.new_empty(0), residual.new_empty(0)


@torch.library.custom_op(f"{NS}::gru_encoder_backward", mutates_args=(), device_types="cuda")
def gru_encoder_backward(dh: Tensor, residual: Tensor, tfeat: Optional[Tensor], w_ih: Tensor, w_hh: Tensor,
                         h_seq: Tensor, gates: Tensor, need_dx: bool
                         ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(dx (B*S, L, I) or empty, dW_ih, dW_hh, db_ih, db_hh) by BPTT over the saved gates
    (lg_gru_bwd)."""
    lib = load_library()
    dh, residual, tfeat, w_ih, w_hh = (_c(t) for t in (dh, residual, tfeat, w_ih, w_hh))
    _req(dh, residual, tfeat, w_ih, w_hh)
    if h_seq.numel() == 0 or gates.numel() == 0:
        raise RuntimeError("gru_encoder was run with save=False; no backward")
    B, L, S = residual.shape
    G, I = w_ih.shape
    H = w_hh.shape[1]
    dev = residual.device
    dx = torch.empty(B * S, L, I, device=dev) if need_dx else torch.empty(0, device=dev)
    dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
    db_ih, db_hh = torch.empty(3 * H, device=dev), torch.empty(3 * H, device=dev)
    ws = torch.empty(int(lib.lg_gru_bwd_workspace_bytes(B, S, I, H)), device=dev, dtype=torch.uint8)
    with _reduce_batch(lib, stream_of(residual)), _timed("gru_bwd", dev):
        check(lib.lg_gru_bwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(h_seq), ptr(gates), ptr(dh),
                             ptr(dx) if need_dx else None, ptr(dw_ih), ptr(dw_hh), ptr(db_ih), ptr(db_hh), B, L, S, I,
                             H, ptr(ws), ws.numel(), stream_of(residual)), "lg_gru_bwd")
    return dx, dw_ih, dw_hh, db_ih, db_hh


@gru_encoder_backward.register_fake
def _(dh, residual, tfeat, w_ih, w_hh, h_seq, gates, need_dx):
    B, L, S = residual.shape
    H = w_hh.shape[1]
    dx = residual.new_empty(B * S, L, w_ih.shape[1]) if need_dx else residual.new_empty(0)
    return dx, torch.empty_like(w_ih), torch.empty_like(w_hh), w_ih.new_empty(3 * H), w_ih.new_empty(3 * H)


def _gru_setup(ctx, inputs, output):
    residual, tfeat, w_ih, w_hh, _, _, _ = inputs
    _, h_seq, gates = output
    ctx.mark_non_differentiable(h_seq, gates)
    ctx.set_materialize_grads(False)  # no zero-filled (L, B*S, 4H) gradients for the saved tensors
    ctx.has_tfeat = tfeat is not None
    ctx.save_for_backward(residual, tfeat, w_ih, w_hh, h_seq, gates)


def _gru_bwd(ctx, dh, _dhseq, _dgates):
    if dh is None:
        return (None,) * 7
    residual, tfeat, w_ih, w_hh, h_seq, gates = ctx.saved_tensors
    B, L, S = residual.shape
    I = w_ih.shape[1]
    need_dx = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
    dx, dw_ih, dw_hh, db_ih, db_hh = torch.ops.leakgnn.gru_encoder_backward(
        dh.contiguous(), residual, tfeat if ctx.has_tfeat else None, w_ih, w_hh, h_seq, gates, need_dx)
    dres = dtf = None
    if ctx.needs_input_grad[0]:
        dres = dx[..., 0].reshape(B, S, L).transpose(1, 2)
    if ctx.has_tfeat and ctx.needs_input_grad[1]:
        dtf = dx[..., 1:].reshape(B, S, L, I - 1).sum(dim=1)
    return dres, dtf, dw_ih, dw_hh, db_ih, db_hh, None


gru_encoder.register_autograd(_gru_bwd, setup_context=_gru_setup)


REDUCE_BATCH = True  # tests switch it off to compare with one reduction launch per op


@contextlib.contextmanager
def _reduce_batch(lib, st):
    """All slab reductions of the enclosed backward launches as one launch at the end
    (lg_reduce_batch_begin / _flush, include/leakgnn.h).  The enclosed code keeps every
    workspace it passes alive until the flush (the caller's locals).  A batch per backward pass
    instead of per op was measured (+0.7 %) and dropped: autograd reads or copies an op's
    gradients (AccumulateGrad into an existing .grad, a clone when another reference is held)
    before an end-of-pass flush would have written them."""
    if not REDUCE_BATCH:
        yield
        return
    check(lib.lg_reduce_batch_begin(), "lg_reduce_batch_begin")
    try:
        yield
    finally:
        check(lib.lg_reduce_batch_flush(st), "lg_reduce_batch_flush")


def expand_x0(xs0: Tensor, x0bits: Tensor, sensor_slot: Tensor, node_bias: Tensor, N: int, p: float) -> Tensor:
    """x_0 (N, B, D) materialised from the compressed node init (lg_node_init_expand):
    diagnostics and tests only (LeakDetector.capture)."""
    lib = load_library()
    S, B, D = xs0.shape
    x0 = torch.empty(N, B, D, device=xs0.device, dtype=torch.float32)
    check(lib.lg_node_init_expand(ptr(sensor_slot), ptr(xs0), ptr(x0bits), ptr(node_bias), ptr(x0), B, N, D,
                                  nat.LG_F_DROPOUT if p > 0.0 else 0, p, stream_of(xs0)), "lg_node_init_expand")
    return x0


# ============================================================================ gnn_trunk
def _compress_x0(nodetab_s: Optional[Tensor], node_major: bool, L: int) -> bool:
    """Whether gnn_trunk keeps x_0 compressed (sensor rows + [x_0 > 0] bits).  Needs a layer
    after layer 0 (L >= 2): the last layer's backward reads its input mask through
    LG_F_MASK_IN, which the x0 backward has no form of (lg_gcn_bwd_nm_x0 returns
    LG_EUNSUPPORTED), so at L == 1 the dense node init runs.  A trunk-forward flag that selects
    another forward kernel (LG_F_NM3, LG_F_F32_MFMA: the A/B and exact-fp32 modes) has no x0
    variant either; it also gets the dense node init, so the flag applies to every layer."""
    other = GCN_FWD_NM_EXTRA_FLAGS & (nat.LG_F_NM3 | nat.LG_F_F32_MFMA)
    return nodetab_s is not None and node_major and L > 1 and not other


@torch.library.custom_op(f"{NS}::gnn_trunk", mutates_args=(), device_types="cuda")
def gnn_trunk(h_s: Tensor, proj_weight: Tensor, node_bias: Tensor, weights: List[Tensor], biases: List[Tensor],
              sensor_slot: Tensor, sensor_idx: Tensor, nonsensor_idx: Tensor, slot_live: Optional[Tensor],
              nodetab: Tensor, pairs: Tensor, rowptr: Tensor, col: Tensor, w: Tensor, nodetab_t: Tensor,
              pairs_t: Tensor, rowptr_t: Tensor, col_t: Tensor, w_t: Tensor, p: float, node_major: bool, seed: Tensor,
              nodetab_s: Optional[Tensor], pairs_s: Optional[Tensor], pos_slot_t: Optional[Tensor],
              *, bf16: bool = False) -> List[Tensor]:
    """[x_0, ..., x_L, ymask, x0bits]: sensor_to_node + node init (detector.py:160, 178-190),
    then L x dropout(relu(GCNConv)).

      x_0     = dropout(relu(slot >= 0 ? [h_s[b, slot], 1] W^T + b : b))   (lg_node_init_proj_fwd)
      x_{l+1} = dropout(relu(Ahat x_l W_l^T + b_l))                        (lg_gcn_fwd[_nm], fused)
    h_s: (B, S, Ds) sensor encodings; proj_weight: sensor_to_node.weight (D, Ds + 1);
    node_bias: its bias.  The projection is formed inside the node-init launch (no GEMM, no
    proj buffer).  node_major: features [N][B][D] (lg_gcn_fwd_nm), else [B][N][D].  p:
    dropout prob (0 = eval).  Every activation is returned: the backward reads its
    ReLU/dropout masks back as [x > 0] and needs x_l for dW.  ymask (node-major only, int16
    (N * ceil(B/16) * 64,), else empty): [x_L > 0] as bits (lg_gcn_fwd_nm_bits), which the
    last layer's backward reads instead of gathering x_L.
    bf16: the node-major transform as one bf16 MFMA product (LG_F_BF16, the configs[2] tier).
    nodetab_s, pairs_s, pos_slot_t (ops.SensorMarks; node-major, L >= 1): x_0 stays
    compressed (lg_node_init_bits_fwd): the returned x_0 is its sensor rows (S, B, D), x0bits
    [x_0 > 0] of every row (int16, ymask's layout), and layer 0 reads them through the marked
    table (lg_gcn_fwd_nm_x0: the dense forward up to the order of its sums).  Otherwise x0bits is empty."""
    lib = load_library()
    h_s, proj_weight, node_bias = _c(h_s), _c(proj_weight), _c(node_bias)
    weights, biases = [_c(t) for t in weights], [_c(t) for t in biases]
    _req(h_s, proj_weight, node_bias, *weights, *biases)
    B, S, Ds = h_s.shape
    D = proj_weight.shape[0]
    _check_d(D)
    if bf16 and not node_major:  # the window-major kernels have no bf16 form (ops.use_node_major)
        raise ValueError("gnn_trunk: the bf16 tier runs on the node-major layout only")
    if tuple(proj_weight.shape) != (D, Ds + 1):
        raise ValueError(f"proj_weight must be (D, Ds + 1) = ({D}, {Ds + 1}), got {tuple(proj_weight.shape)}")
    N = sensor_slot.shape[0]
    drop = p > 0.0
    seed_v, sbit = _seed_args(seed) if drop else (0, 0)
    dflag = nat.LG_F_DROPOUT if drop else 0
    st = stream_of(h_s)
    L = len(weights)
    nmask = N * ((B + 15) // 16) * 64
    x0c = _compress_x0(nodetab_s, node_major, L)
    if x0c:
        x0 = torch.empty((S, B, D), device=h_s.device, dtype=torch.float32)
        x0bits = torch.empty(nmask, device=h_s.device, dtype=torch.int16)
        with _timed("node_init", h_s.device):
            check(lib.lg_node_init_bits_fwd(ptr(sensor_slot), ptr(sensor_idx), ptr(h_s), ptr(proj_weight),
                                            ptr(node_bias), ptr(x0), ptr(x0bits), B, N, S, Ds, D, dflag, p, seed_v,
                                            0 | sbit, st), "lg_node_init_bits_fwd")
    else:
        x0 = torch.empty((N, B, D) if node_major else (B, N, D), device=h_s.device, dtype=torch.float32)
        x0bits = torch.empty(0, device=h_s.device, dtype=torch.int16)
        with _timed("node_init", h_s.device):
            check(lib.lg_node_init_proj_fwd(ptr(sensor_slot), ptr(sensor_idx), ptr(h_s), ptr(proj_weight),
                                            ptr(node_bias), ptr(x0), B, N, S, Ds, D,
                                            dflag | (nat.LG_F_NODE_MAJOR if node_major else 0), p, seed_v, 0 | sbit, st),
                  "lg_node_init_proj_fwd")
    xs = [x0]
    ymask = torch.empty(nmask if (node_major and L > 0) else 0, device=h_s.device, dtype=torch.int16)
    for l, (W, b) in enumerate(zip(weights, biases)):
        y = torch.empty((N, B, D), device=h_s.device, dtype=torch.float32) if node_major else torch.empty_like(x0)
        flags = nat.LG_F_BIAS | nat.LG_F_RELU | dflag | (nat.LG_F_BF16 if bf16 else 0)
        with _timed("gcn_fwd" if not (x0c and l == 0) else "gcn_fwd_l0", h_s.device):
            if x0c and l == 0:
                check(lib.lg_gcn_fwd_nm_x0(ptr(nodetab_s), ptr(pairs_s), ptr(x0), ptr(x0bits), ptr(node_bias),
                                           ptr(W), ptr(b), ptr(y), B, N, S, D, flags | GCN_FWD_NM_EXTRA_FLAGS, p,
                                           seed_v, (l + 1) | sbit, st), "lg_gcn_fwd_nm_x0")
            elif node_major:
                fx = GCN_FWD_DENSE_EXTRA_FLAGS if not bf16 else 0
                check(lib.lg_gcn_fwd_nm_bits(ptr(nodetab), ptr(pairs), ptr(xs[-1]), ptr(W), ptr(b), ptr(y), B, N,
                                             D, col.numel(), flags | GCN_FWD_NM_EXTRA_FLAGS | fx, p, seed_v,
                                             (l + 1) | sbit, st, ptr(ymask) if l == L - 1 else None),
                      "lg_gcn_fwd_nm_bits")
            else:
                check(lib.lg_gcn_fwd(ptr(rowptr), ptr(col), ptr(w), ptr(xs[-1]), ptr(W), ptr(b), ptr(y), B, N, D,
                                     col.numel(), flags, p, seed_v, (l + 1) | sbit, st), "lg_gcn_fwd")
        xs.append(y)
    return xs + [ymask, x0bits]


@gnn_trunk.register_fake
def _(h_s, proj_weight, node_bias, weights, biases, sensor_slot, sensor_idx, nonsensor_idx, slot_live, nodetab, pairs,
      rowptr, col, w, nodetab_t, pairs_t, rowptr_t, col_t, w_t, p, node_major, seed, nodetab_s, pairs_s, pos_slot_t, *,
      bf16=False):
    B, S = h_s.shape[0], h_s.shape[1]
    D = proj_weight.shape[0]
    N = sensor_slot.shape[0]
    shape = (N, B, D) if node_major else (B, N, D)
    L = len(weights)
    nmask = N * ((B + 15) // 16) * 64 if (node_major and L > 0) else 0
    x0c = _compress_x0(nodetab_s, node_major, L)
    x0 = h_s.new_empty((S, B, D)) if x0c else h_s.new_empty(shape)
    return ([x0] + [h_s.new_empty(shape) for _ in range(L)] + [h_s.new_empty((nmask,), dtype=torch.int16)]
            + [h_s.new_empty((nmask if x0c else 0,), dtype=torch.int16)])


@torch.library.custom_op(f"{NS}::gnn_trunk_backward", mutates_args=(), device_types="cuda")
def gnn_trunk_backward(grad_out: Tensor, xs: List[Tensor], ymask: Tensor, h_s: Tensor, proj_weight: Tensor,
                       weights: List[Tensor],
                       sensor_slot: Tensor, sensor_idx: Tensor, nonsensor_idx: Tensor, slot_live: Optional[Tensor],
                       nodetab_t: Tensor, pairs_t: Tensor, rowptr_t: Tensor, col_t: Tensor, w_t: Tensor, p: float,
                       node_major: bool, x0bits: Optional[Tensor], x0_bias: Optional[Tensor],
                       pos_slot_t: Optional[Tensor], *, bf16: bool = False
                       ) -> Tuple[Tensor, Tensor, Tensor, List[Tensor], List[Tensor]]:
    """(dh_s, dproj_weight, dnode_bias, [dW_l], [db_l]): one fused lg_gcn_bwd[_nm] per layer,
    last first (ReLU/dropout masks of a layer's output and input applied inside the kernel
    from the saved activations; the non-sensor rows' node-bias gradient summed inside layer
    0's launch), then ONE lg_sensor_proj_bwd for the projection (gather of the sensor rows,
    dh_s, dW and the full bias gradient).  x0bits, x0_bias (the node init's bias), pos_slot_t: x_0 is
    compressed (gnn_trunk's x0marks path; xs[0] its sensor rows) and layer 0's backward reads
    it through lg_gcn_bwd_nm_x0."""
    lib = load_library()
    L = len(weights)
    dev = grad_out.device
    st = stream_of(grad_out)
    if node_major:
        N, B, D = xs[-1].shape
    else:
        B, N, D = xs[0].shape
    S, Ds = h_s.shape[1], h_s.shape[2]
    scale = 1.0 / (1.0 - p) if p > 0.0 else 1.0
    dy = grad_out.contiguous()
    wsb = lib.lg_gcn_bwd_nm_workspace_bytes(D) if node_major else lib.lg_gcn_bwd_workspace_bytes(D)
    # one workspace per layer: the layers' slab reductions run together at the batch flush
    wss = [torch.empty(int(wsb), device=dev, dtype=torch.uint8) for _ in range(L)]
    dWs: List[Tensor] = [grad_out] * L
    dbs: List[Tensor] = [grad_out] * L
    dbias_ns = torch.empty(D, device=dev, dtype=torch.float32)
    with _reduce_batch(lib, st):
        dh_s, dWp, dbp = _trunk_backward_launches(lib, dy, xs, ymask, h_s, proj_weight, weights, sensor_slot, sensor_idx,
                                                  nonsensor_idx, slot_live, nodetab_t, pairs_t, rowptr_t, col_t, w_t,
                                                  node_major, bf16, scale, wss, dWs, dbs, dbias_ns, st,
                                                  (x0bits, x0_bias, pos_slot_t) if x0bits is not None else None, p)
    return dh_s, dWp, dbp, dWs, dbs


def _trunk_backward_launches(lib, dy, xs, ymask, h_s, proj_weight, weights, sensor_slot, sensor_idx, nonsensor_idx, slot_live,
                             nodetab_t, pairs_t, rowptr_t, col_t, w_t, node_major, bf16, scale, wss, dWs, dbs, dbias_ns,
                             st, x0c=None, p=0.0):
    dy = _trunk_layer_launches(lib, dy, xs, ymask, weights, sensor_slot, nodetab_t, pairs_t, rowptr_t, col_t, w_t,
                               node_major, bf16, scale, wss, dWs, dbs, dbias_ns, st, x0c, p)
    L = len(weights)
    dev = dy.device
    if node_major:
        N, B, D = xs[-1].shape
    else:
        B, N, D = xs[0].shape
    S, Ds = h_s.shape[1], h_s.shape[2]
    if L == 0:  # no layer-0 launch applied the node init's relu/dropout mask
        dy = dy * (xs[0] > 0) * scale
        dbias_ns = dy.index_select(0 if node_major else 1, nonsensor_idx).sum(dim=(0, 1))
    dh_s = torch.empty(B, S, Ds, device=dev, dtype=torch.float32)
    dWp = torch.empty(D, Ds + 1, device=dev, dtype=torch.float32)
    dbp = torch.empty(D, device=dev, dtype=torch.float32)
    wsp = torch.empty(int(lib.lg_sensor_proj_bwd_workspace_bytes(B, S, Ds, D)), device=dev, dtype=torch.uint8)
    wss.append(wsp)  # held by the caller until the reduce batch is flushed
    with _timed("linear_dw", dev):
        check(lib.lg_sensor_proj_bwd(ptr(dy), ptr(sensor_idx), ptr(slot_live) if slot_live is not None else None,
                                     ptr(h_s), ptr(proj_weight), ptr(dbias_ns), ptr(dh_s), ptr(dWp), ptr(dbp), B, N,
                                     S, Ds, D, nat.LG_F_NODE_MAJOR if node_major else 0, ptr(wsp), wsp.numel(), st),
              "lg_sensor_proj_bwd")
    return dh_s, dWp, dbp


def _trunk_layer_launches(lib, dy, xs, ymask, weights, sensor_slot, nodetab_t, pairs_t, rowptr_t, col_t, w_t, node_major,
                          bf16, scale, wss, dWs, dbs, dbias_ns, st, x0c=None, p=0.0) -> Tensor:
    """The GCN layers' backward, last first; returns the node init's pre-activation gradient
    (layer 0's dx: masked by the node init's ReLU / dropout; node-major with the compressed
    node init: the sensor nodes' rows only) and leaves the non-sensor rows' sum in dbias_ns."""
    L = len(weights)
    dev = dy.device
    if node_major:
        N, B, D = xs[-1].shape
    else:
        B, N, D = xs[0].shape
    for l in range(L - 1, -1, -1):
        ws = wss[l]
        flags = nat.LG_F_MASK_OUT | (nat.LG_F_MASK_IN if l == L - 1 else 0) | (nat.LG_F_BF16 if bf16 else 0)
        if node_major and not bf16:
            flags |= GCN_BWD_NM_EXTRA_FLAGS
        if l == 0:  # lg_sensor_proj_bwd reads only the sensor rows of layer 0's dx
            flags |= nat.LG_F_DX_SENSOR_ROWS
        dx = torch.empty_like(dy)
        dW = torch.empty(D, D, device=dev, dtype=torch.float32)
        db = torch.empty(D, device=dev, dtype=torch.float32)
        slot_p, dbias_p = (ptr(sensor_slot), ptr(dbias_ns)) if l == 0 else (None, None)
        with _timed("gcn_bwd" if l == L - 1 else f"gcn_bwd_l{l}", dev):
            if x0c is not None and l == 0:  # the compressed node init (xs[0]: its sensor rows, (S, B, D))
                x0bits, node_bias, pos_slot_t = x0c
                S = xs[0].shape[0]
                check(lib.lg_gcn_bwd_nm_x0(ptr(nodetab_t), ptr(pairs_t), ptr(pos_slot_t), ptr(dy), ptr(xs[0]),
                                           ptr(x0bits), ptr(node_bias), ptr(weights[0]), ptr(dx), ptr(dW), ptr(db),
                                           slot_p, dbias_p, B, N, S, D, flags | (nat.LG_F_DROPOUT if p > 0.0 else 0),
                                           p, scale, ptr(ws), ws.numel(), st), "lg_gcn_bwd_nm_x0")
            elif node_major:
                bits = ptr(ymask) if (l == L - 1 and ymask.numel() > 0) else None  # [x_L > 0] as bits
                check(lib.lg_gcn_bwd_nm_bits(ptr(nodetab_t), ptr(pairs_t), ptr(dy), ptr(xs[l + 1]), ptr(xs[l]),
                                             ptr(weights[l]), ptr(dx), ptr(dW), ptr(db), slot_p, dbias_p, B, N, D,
                                             flags, scale, scale, ptr(ws), ws.numel(), st, bits), "lg_gcn_bwd_nm_bits")
            else:
                check(lib.lg_gcn_bwd(ptr(rowptr_t), ptr(col_t), ptr(w_t), ptr(dy), ptr(xs[l + 1]), ptr(xs[l]),
                                     ptr(weights[l]), ptr(dx), ptr(dW), ptr(db), slot_p, dbias_p, B, N, D,
                                     col_t.numel(), flags, scale, scale, ptr(ws), ws.numel(), st), "lg_gcn_bwd")
        dWs[l], dbs[l] = dW, db
        dy = dx  # already masked by the previous op's relu/dropout
    return dy


@gnn_trunk_backward.register_fake
def _(grad_out, xs, ymask, h_s, proj_weight, weights, sensor_slot, sensor_idx, nonsensor_idx, slot_live, nodetab_t,
      pairs_t, rowptr_t, col_t, w_t, p, node_major, x0bits, x0_bias, pos_slot_t, *, bf16=False):
    D = proj_weight.shape[0]
    return (torch.empty_like(h_s), torch.empty_like(proj_weight), grad_out.new_empty(D),
            [torch.empty_like(t) for t in weights], [grad_out.new_empty(D) for _ in weights])


def _trunk_setup(ctx, inputs, keyword_only_inputs, output):
    (h_s, proj_weight, node_bias, weights, biases, sensor_slot, sensor_idx, nonsensor_idx, slot_live, _, _, _, _, _,
     nodetab_t, pairs_t, rowptr_t, col_t, w_t, p, node_major, _, _, _, pos_slot_in) = inputs
    bf16 = bool(keyword_only_inputs.get("bf16", False))
    ctx.L = len(weights)
    ctx.bf16 = bf16
    ctx.x0c = output[ctx.L + 2].numel() > 0  # x_0 compressed (x0bits non-empty)
    # x_0 .. x_{L-1} (returned for the backward's masks), ymask and x0bits
    ctx.mark_non_differentiable(*output[:ctx.L], output[ctx.L + 1], output[ctx.L + 2])
    ctx.set_materialize_grads(False)  # their gradients would be zero-filled (B, N, D) tensors
    ctx.p, ctx.node_major, ctx.has_live = p, node_major, slot_live is not None
    pos_slot_t = pos_slot_in if ctx.x0c else sensor_slot
    ctx.save_for_backward(*output, h_s, proj_weight, *weights, sensor_slot, sensor_idx, nonsensor_idx,
                          slot_live if slot_live is not None else sensor_slot, nodetab_t, pairs_t, rowptr_t, col_t, w_t,
                          node_bias, pos_slot_t)


def _trunk_bwd(ctx, grads):
    L = ctx.L
    saved = ctx.saved_tensors
    xs, ymask, x0bits, h_s, proj_weight = list(saved[:L + 1]), saved[L + 1], saved[L + 2], saved[L + 3], saved[L + 4]
    weights = list(saved[L + 5:2 * L + 5])
    (sensor_slot, sensor_idx, nonsensor_idx, live, nodetab_t, pairs_t, rowptr_t, col_t, w_t, node_bias,
     pos_slot_t) = saved[2 * L + 5:]
    g = grads[L]
    if g is None:
        return (None,) * 25
    dh_s, dWp, dbp, dWs, dbs = torch.ops.leakgnn.gnn_trunk_backward(
        g, xs, ymask, h_s, proj_weight, weights, sensor_slot, sensor_idx, nonsensor_idx, live if ctx.has_live else None,
        nodetab_t, pairs_t, rowptr_t, col_t, w_t, ctx.p, ctx.node_major, x0bits if ctx.x0c else None,
        node_bias if ctx.x0c else None, pos_slot_t if ctx.x0c else None, bf16=ctx.bf16)
    return (dh_s, dWp, dbp, dWs, dbs) + (None,) * 20


gnn_trunk.register_autograd(_trunk_bwd, setup_context=_trunk_setup)


# ============================================================================ encoder_trunk
# The sensor encoder, the node init and the GCN layers as ONE registered op (the node-major
# trunk with the compressed node init): the GRU's training forward forms the node init's
# sensor rows and [x0 > 0] words in its epilogue (lg_gru_node_init_fwd), and the backward runs
# the layers, then the GRU with the sensor projection's backward in its prologue / epilogue
# (lg_gru_node_init_bwd), all weight-gradient reductions in one launch.  Against gru_encoder +
# gnn_trunk: the node-init launch and the projection-backward launch leave the step, and the
# trunk's and the GRU's reductions share one launch.  Same arithmetic, bit for bit
# (tests/test_gpu_x0.py::test_encoder_trunk_equals_separate_ops).
def encoder_trunk_supported(B: int, N: int, H: int, D: int, L: int, node_major: bool, compress: bool) -> bool:
    """The fused op's case: node-major layout, the compressed node init (L >= 2, no alternate
    forward-kernel flag), node_hidden == sensor_hidden in {32, 64}."""
    return (node_major and compress and H == D and D in (32, 64)
            and _compress_x0(torch.empty(0), node_major, L))


@torch.library.custom_op(f"{NS}::encoder_trunk", mutates_args=(), device_types="cuda")
def encoder_trunk(residual: Tensor, tfeat: Optional[Tensor], w_ih: Tensor, w_hh: Tensor, b_ih: Tensor, b_hh: Tensor,
                  proj_weight: Tensor, node_bias: Tensor, weights: List[Tensor], biases: List[Tensor],
                  sensor_slot: Tensor, sensor_idx: Tensor, slot_live: Optional[Tensor], nodetab: Tensor, pairs: Tensor,
                  nodetab_t: Tensor, pairs_t: Tensor, nodetab_s: Tensor, pairs_s: Tensor, pos_slot_t: Tensor, p: float,
                  seed: Tensor, save: bool, *, bf16: bool = False) -> List[Tensor]:
    """[x_1, ..., x_L, ymask, xs0, x0bits, h_seq, gates]: SharedSensorGRUEncoder (detector.py:60-73),
    the node init (:179-190: h0, the mask column, sensor_to_node, ReLU, dropout) and L x
    dropout(relu(GCNConv)) (:198-201) on the node-major layout [N][B][D].  x_0 stays
    compressed: xs0 (S, B, D) its sensor rows, x0bits [x_0 > 0] of the other rows.  ymask: x_L's
    [x > 0] bits.  h_seq / gates: the GRU's saved steps (empty unless save).  residual and tfeat
    are data (no gradient)."""
    lib = load_library()
    residual, tfeat = _c(residual), _c(tfeat)
    w_ih, w_hh, b_ih, b_hh, proj_weight, node_bias = (_c(t) for t in (w_ih, w_hh, b_ih, b_hh, proj_weight, node_bias))
    weights, biases = [_c(t) for t in weights], [_c(t) for t in biases]
    _req(residual, tfeat, w_ih, w_hh, b_ih, b_hh, proj_weight, node_bias, *weights, *biases)
    B, Lw, S = residual.shape
    G, I = w_ih.shape
    H = w_hh.shape[1]
    D = proj_weight.shape[0]
    N = sensor_slot.shape[0]
    L = len(weights)
    if not encoder_trunk_supported(B, N, H, D, L, True, True):
        raise NotImplementedError("encoder_trunk: node-major trunk with the compressed node init, "
                                  "node_hidden == sensor_hidden in {32, 64}, at least two layers")
    if tuple(proj_weight.shape) != (D, H + 1):
        raise ValueError(f"proj_weight must be ({D}, {H + 1}), got {tuple(proj_weight.shape)}")
    dev = residual.device
    st = stream_of(residual)
    drop = p > 0.0
    seed_v, sbit = _seed_args(seed) if drop else (0, 0)
    dflag = nat.LG_F_DROPOUT if drop else 0
    nmask = N * ((B + 15) // 16) * 64
    h_seq = torch.empty(Lw, B * S, H, device=dev) if save else torch.empty(0, device=dev)
    gates = torch.empty(Lw, B * S, 4, H, device=dev) if save else torch.empty(0, device=dev)
    h_last = torch.empty(B, S, H, device=dev)
    xs0 = torch.empty((S, B, D), device=dev, dtype=torch.float32)
    x0bits = torch.empty(nmask, device=dev, dtype=torch.int16)
    with _timed("gru_fwd", dev):
        check(lib.lg_gru_node_init_fwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh),
                                       ptr(h_seq) if save else None, ptr(gates) if save else None, ptr(h_last),
                                       ptr(sensor_slot), ptr(sensor_idx), ptr(proj_weight), ptr(node_bias), ptr(xs0),
                                       ptr(x0bits), B, Lw, S, I, H, N, dflag, p, seed_v, 0 | sbit, st),
              "lg_gru_node_init_fwd")
    ymask = torch.empty(nmask, device=dev, dtype=torch.int16)
    xs = [xs0]
    for l, (W, b) in enumerate(zip(weights, biases)):
        y = torch.empty((N, B, D), device=dev, dtype=torch.float32)
        flags = nat.LG_F_BIAS | nat.LG_F_RELU | dflag | (nat.LG_F_BF16 if bf16 else 0)
        with _timed("gcn_fwd" if l > 0 else "gcn_fwd_l0", dev):
            if l == 0:
                check(lib.lg_gcn_fwd_nm_x0(ptr(nodetab_s), ptr(pairs_s), ptr(xs0), ptr(x0bits), ptr(node_bias), ptr(W),
                                           ptr(b), ptr(y), B, N, S, D, flags | GCN_FWD_NM_EXTRA_FLAGS, p, seed_v,
                                           (l + 1) | sbit, st), "lg_gcn_fwd_nm_x0")
            else:
                fx = GCN_FWD_DENSE_EXTRA_FLAGS if not bf16 else 0
                check(lib.lg_gcn_fwd_nm_bits(ptr(nodetab), ptr(pairs), ptr(xs[-1]), ptr(W), ptr(b), ptr(y), B, N, D,
                                             pairs.shape[0], flags | GCN_FWD_NM_EXTRA_FLAGS | fx, p, seed_v, (l + 1) | sbit,
                                             st, ptr(ymask) if l == L - 1 else None), "lg_gcn_fwd_nm_bits")
        xs.append(y)
    return xs[1:] + [ymask, xs0, x0bits, h_seq, gates]


@encoder_trunk.register_fake
def _(residual, tfeat, w_ih, w_hh, b_ih, b_hh, proj_weight, node_bias, weights, biases, sensor_slot, sensor_idx,
      slot_live, nodetab, pairs, nodetab_t, pairs_t, nodetab_s, pairs_s, pos_slot_t, p, seed, save, *, bf16=False):
    B, Lw, S = residual.shape
    H = w_hh.shape[1]
    D = proj_weight.shape[0]
    N = sensor_slot.shape[0]
    nmask = N * ((B + 15) // 16) * 64
    h_seq = residual.new_empty(Lw, B * S, H) if save else residual.new_empty(0)
    gates = residual.new_empty(Lw, B * S, 4, H) if save else residual.new_empty(0)
    return ([residual.new_empty(N, B, D) for _ in weights] + [residual.new_empty((nmask,), dtype=torch.int16),
            residual.new_empty(S, B, D), residual.new_empty((nmask,), dtype=torch.int16), h_seq, gates])


@torch.library.custom_op(f"{NS}::encoder_trunk_backward", mutates_args=(), device_types="cuda")
def encoder_trunk_backward(grad_out: Tensor, xs: List[Tensor], ymask: Tensor, x0bits: Tensor, residual: Tensor,
                           tfeat: Optional[Tensor], w_ih: Tensor, w_hh: Tensor, h_seq: Tensor, gates: Tensor,
                           proj_weight: Tensor, node_bias: Tensor, weights: List[Tensor], sensor_slot: Tensor,
                           sensor_idx: Tensor, slot_live: Optional[Tensor], nodetab_t: Tensor, pairs_t: Tensor,
                           pos_slot_t: Tensor, p: float, *, bf16: bool = False) -> List[Tensor]:
    """[dw_ih, dw_hh, db_ih, db_hh, dproj_weight, dnode_bias, dW_0 .. dW_{L-1}, db_0 .. db_{L-1}]: the
    layers' backward (last first; layer 0 on the compressed x_0, its dx for the sensor rows
    only), then lg_gru_node_init_bwd; one reduce batch for all of them."""
    lib = load_library()
    if h_seq.numel() == 0 or gates.numel() == 0:
        raise RuntimeError("encoder_trunk was run with save=False; no backward")
    L = len(weights)
    dev = grad_out.device
    st = stream_of(grad_out)
    N, B, D = xs[-1].shape
    S, Lw = residual.shape[2], residual.shape[1]
    I, H = w_ih.shape[1], w_hh.shape[1]
    scale = 1.0 / (1.0 - p) if p > 0.0 else 1.0
    wsb = lib.lg_gcn_bwd_nm_workspace_bytes(D)
    wss = [torch.empty(int(wsb), device=dev, dtype=torch.uint8) for _ in range(L)]
    dWs: List[Tensor] = [grad_out] * L
    dbs: List[Tensor] = [grad_out] * L
    dbias_ns = torch.empty(D, device=dev, dtype=torch.float32)
    dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
    db_ih, db_hh = torch.empty(3 * H, device=dev), torch.empty(3 * H, device=dev)
    dWp, dbp = torch.empty_like(proj_weight), torch.empty(D, device=dev)
    wsg = torch.empty(int(lib.lg_gru_node_init_bwd_workspace_bytes(B, S, I, H)), device=dev, dtype=torch.uint8)
    with _reduce_batch(lib, st):
        dx0 = _trunk_layer_launches(lib, grad_out.contiguous(), xs, ymask, weights, sensor_slot, nodetab_t, pairs_t,
                                    None, None, None, True, bf16, scale, wss, dWs, dbs, dbias_ns, st,
                                    (x0bits, node_bias, pos_slot_t), p)
        with _timed("gru_bwd", dev):
            check(lib.lg_gru_node_init_bwd(ptr(residual), ptr(tfeat), ptr(w_ih), ptr(w_hh), ptr(h_seq), ptr(gates),
                                           ptr(dx0), ptr(sensor_idx), ptr(slot_live) if slot_live is not None else None,
                                           ptr(proj_weight), ptr(dbias_ns), ptr(dw_ih), ptr(dw_hh), ptr(db_ih),
                                           ptr(db_hh), ptr(dWp), ptr(dbp), B, Lw, S, I, H, N, ptr(wsg), wsg.numel(),
                                           st), "lg_gru_node_init_bwd")
    return [dw_ih, dw_hh, db_ih, db_hh, dWp, dbp] + dWs + dbs


@encoder_trunk_backward.register_fake
def _(grad_out, xs, ymask, x0bits, residual, tfeat, w_ih, w_hh, h_seq, gates, proj_weight, node_bias, weights,
      sensor_slot, sensor_idx, slot_live, nodetab_t, pairs_t, pos_slot_t, p, *, bf16=False):
    H = w_hh.shape[1]
    D = proj_weight.shape[0]
    return ([torch.empty_like(w_ih), torch.empty_like(w_hh), w_ih.new_empty(3 * H), w_ih.new_empty(3 * H),
             torch.empty_like(proj_weight), proj_weight.new_empty(D)] + [torch.empty_like(t) for t in weights]
            + [proj_weight.new_empty(D) for _ in weights])


def _et_setup(ctx, inputs, keyword_only_inputs, output):
    (residual, tfeat, w_ih, w_hh, b_ih, b_hh, proj_weight, node_bias, weights, biases, sensor_slot, sensor_idx,
     slot_live, nodetab, pairs, nodetab_t, pairs_t, nodetab_s, pairs_s, pos_slot_t, p, seed, save) = inputs
    L = len(weights)
    ctx.L, ctx.p, ctx.bf16 = L, p, bool(keyword_only_inputs.get("bf16", False))
    ctx.has_tfeat, ctx.has_live = tfeat is not None, slot_live is not None
    # x_1 .. x_{L-1}, ymask, xs0, x0bits, h_seq, gates: saved, never differentiated
    ctx.mark_non_differentiable(*output[:L - 1], *output[L:])
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(*output[:L], output[L], output[L + 1], output[L + 2], output[L + 3], output[L + 4],
                          residual, tfeat if tfeat is not None else residual, w_ih, w_hh, proj_weight, node_bias,
                          *weights, sensor_slot, sensor_idx, slot_live if slot_live is not None else sensor_slot,
                          nodetab_t, pairs_t, pos_slot_t)


def _et_bwd(ctx, grads):
    L = ctx.L
    g = grads[L - 1]
    if g is None:
        return (None,) * 23
    sv = ctx.saved_tensors
    xl = list(sv[:L])
    ymask, xs0, x0bits, h_seq, gates = sv[L:L + 5]
    residual, tfeat, w_ih, w_hh, proj_weight, node_bias = sv[L + 5:L + 11]
    weights = list(sv[L + 11:2 * L + 11])
    sensor_slot, sensor_idx, live, nodetab_t, pairs_t, pos_slot_t = sv[2 * L + 11:]
    out = torch.ops.leakgnn.encoder_trunk_backward(
        g, [xs0] + xl, ymask, x0bits, residual, tfeat if ctx.has_tfeat else None, w_ih, w_hh, h_seq, gates,
        proj_weight, node_bias, weights, sensor_slot, sensor_idx, live if ctx.has_live else None, nodetab_t, pairs_t,
        pos_slot_t, ctx.p, bf16=ctx.bf16)
    dw_ih, dw_hh, db_ih, db_hh, dWp, dbp = out[:6]
    dWs, dbs = list(out[6:6 + L]), list(out[6 + L:])
    return (None, None, dw_ih, dw_hh, db_ih, db_hh, dWp, dbp, dWs, dbs) + (None,) * 13


encoder_trunk.register_autograd(_et_bwd, setup_context=_et_setup)


# ============================================================================ detector_heads
@torch.library.custom_op(f"{NS}::detector_heads", mutates_args=(), device_types="cuda")
def detector_heads(h: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, nw1: Tensor, nb1: Tensor, nw2: Tensor,
                   nb2: Tensor, ends: Tensor, inc_rowptr: Tensor, inc_item: Tensor, p_edge: float, p_noleak: float,
                   node_major: bool, keep_hidden: bool, seed: Tensor, sched: Optional[Tensor] = None,
                   sched_hdr: Optional[List[int]] = None, *, bf16: bool = False) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """(logits (B, P+1), EdgeHead hidden, pooled, NoLeakHead hidden).  Columns [0, P) by
    lg_edge_head_fwd (endpoint gather -> MFMA MLP -> dot, the (B, P, 3D) features never
    stored), column P by lg_pool_head_fwd (mean pool + NoLeakHead): the torch.cat of
    detector.py:218 is never a separate copy.  keep_hidden: keep the EdgeHead hidden layer
    for a recompute-free backward (else it is empty).  bf16: the EdgeHead MLP as one bf16
    MFMA product (LG_F_BF16, the configs[2] tier); the NoLeakHead stays fp32.  sched /
    sched_hdr: the pipe schedule of inc_rowptr / inc_item (ops.Incidence.schedule(D)), for the
    backward's streamed node sums; None / [] for the per-window scatter."""
    lib = load_library()
    h, w1, b1, w2, b2, nw1, nb1, nw2, nb2 = (_c(t) for t in (h, w1, b1, w2, b2, nw1, nb1, nw2, nb2))
    _req(h, w1, b1, w2, b2, nw1, nb1, nw2, nb2)
    N, B, D = h.shape if node_major else (h.shape[1], h.shape[0], h.shape[2])
    _check_d(D)
    lay = nat.LG_F_NODE_MAJOR if node_major else 0
    hidden, nhidden = w1.shape[0], nw1.shape[0]
    P = ends.shape[0]
    seed_v, sbit = _seed_args(seed) if (p_edge > 0.0 or p_noleak > 0.0) else (0, 0)
    fe = (nat.LG_F_DROPOUT if p_edge > 0.0 else 0) | (nat.LG_F_BF16 if bf16 else 0)
    fn = nat.LG_F_DROPOUT if p_noleak > 0.0 else 0
    st = stream_of(h)
    dev = h.device
    logits = torch.empty(B, P + 1, device=dev, dtype=torch.float32)
    pooled = torch.empty(B, D, device=dev, dtype=torch.float32)
    hid = torch.empty(B, nhidden, device=dev, dtype=torch.float32)
    ehid = torch.empty(B * P, hidden, device=dev, dtype=torch.float32) if keep_hidden else torch.empty(0, device=dev)
    with _timed("edge_fwd", dev):
        check(lib.lg_edge_head_fwd(ptr(ends), ptr(h), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(logits), P + 1,
                                   ptr(ehid) if keep_hidden else None, B, N, P, D, hidden, fe | lay, p_edge, seed_v,
                                   EDGE_HEAD_SALT | sbit, st), "lg_edge_head_fwd")
    with _timed("pool_head", dev):
        check(lib.lg_pool_head_fwd(ptr(h), ptr(nw1), ptr(nb1), ptr(nw2), ptr(nb2), ptr(pooled), ptr(hid), ptr(logits),
                                   P + 1, P, B, N, D, nhidden, fn | lay, p_noleak, seed_v, NOLEAK_HEAD_SALT | sbit,
                                   st), "lg_pool_head_fwd")
    return logits, ehid, pooled, hid


@detector_heads.register_fake
def _(h, w1, b1, w2, b2, nw1, nb1, nw2, nb2, ends, inc_rowptr, inc_item, p_edge, p_noleak, node_major, keep_hidden,
      seed, sched=None, sched_hdr=None, *, bf16=False):
    B = h.shape[1] if node_major else h.shape[0]
    D = h.shape[2]
    P = ends.shape[0]
    ehid = h.new_empty(B * P, w1.shape[0]) if keep_hidden else h.new_empty(0)
    return h.new_empty(B, P + 1), ehid, h.new_empty(B, D), h.new_empty(B, nw1.shape[0])


@torch.library.custom_op(f"{NS}::detector_heads_backward", mutates_args=(), device_types="cuda")
def detector_heads_backward(dlogits: Tensor, h: Tensor, w1: Tensor, w2: Tensor, ehid: Tensor, pooled: Tensor,
                            hid: Tensor, nw1: Tensor, nw2: Tensor, ends: Tensor, inc_rowptr: Tensor, inc_item: Tensor,
                            sched: Optional[Tensor], sched_hdr: List[int], p_edge: float, p_noleak: float,
                            node_major: bool, *, bf16: bool = False
                            ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(dh, dW1, db1, dW2, db2, dnW1, dnb1, dnW2, dnb2): lg_pool_head_bwd -> dpooled and the
    NoLeakHead grads; lg_edge_head_bwd_scatter -> the per-pipe endpoint grads and, fused, their
    deterministic incidence reduce plus dpooled / N into every node row."""
    lib = load_library()
    if ehid.numel() == 0:
        raise RuntimeError("detector_heads was run with keep_hidden=False; no backward")
    dl, h = _c(dlogits), _c(h)
    N, B, D = h.shape if node_major else (h.shape[1], h.shape[0], h.shape[2])
    lay = nat.LG_F_NODE_MAJOR if node_major else 0
    P, hidden, nhidden = ends.shape[0], w1.shape[0], nw1.shape[0]
    fe = (nat.LG_F_DROPOUT if p_edge > 0.0 else 0) | (nat.LG_F_BF16 if bf16 else 0)
    fn = nat.LG_F_DROPOUT if p_noleak > 0.0 else 0
    dev = h.device
    st = stream_of(h)
    dpipe = torch.empty(B, P, 2, D, device=dev)
    dw1, db1 = torch.empty_like(w1), torch.empty(hidden, device=dev)
    dw2, db2 = torch.empty_like(w2), torch.empty(1, device=dev)
    ndw1, ndb1 = torch.empty_like(nw1), torch.empty(nhidden, device=dev)
    ndw2, ndb2 = torch.empty_like(nw2), torch.empty(1, device=dev)
    ws = torch.empty(int(lib.lg_edge_head_bwd_workspace_bytes(B, P, D, hidden)), device=dev, dtype=torch.uint8)
    wsn = torch.empty(int(lib.lg_pool_head_bwd_workspace_bytes(B, D, nhidden)), device=dev, dtype=torch.uint8)
    dh = torch.empty_like(h)
    # one launch for the EdgeHead's and the NoLeakHead's weight-grad reductions
    with _reduce_batch(lib, st):
        _heads_backward_launches(lib, dl, h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr, inc_item, sched,
                                 sched_hdr, P, B, N, D, hidden, nhidden, fe | lay, fn, p_edge, p_noleak, dpipe, dh, dw1,
                                 db1, dw2, db2, ndw1, ndb1, ndw2, ndb2, ws, wsn, st)
    return dh, dw1, db1, dw2, db2, ndw1, ndb1, ndw2, ndb2


# True: the pipe scatter fused into the EdgeHead backward (lg_edge_head_bwd_scatter): with the
# pipe schedule (ABI 22, the default at B >= the CU count) the node sums are STREAMED tile by
# tile from the dfeat rows in LDS, so no per-pipe row reaches HBM; without one, per window
# after its last tile (ABI 19).  False: two launches (lg_edge_head_bwd + lg_pipe_scatter_bwd).
# Same node gradient bit for bit (one incidence order for all;
# tests/test_gpu_library.py::test_fused_pipe_scatter_matches_two_launches).  Measured at
# B = 256 (DESIGN §3 "Round 4"): streamed 125-132 us in the step (profiles/r04/r04z3), against
# 152.6 us for the per-window form and 114.6 + 35.3 us for the two launches (round 3); since
# round 5 the streamed launch also runs the NoLeakHead backward (_FUSED_HEADS below):
# 135-139 us in the step for both heads (profiles/r05/r05p), against 125-132 + 10-11 us.
_FUSED_SCATTER = True
# True: with the streamed scatter, the NoLeakHead backward runs in the EdgeHead backward's
# prologue (lg_heads_bwd_scatter: one launch for both heads); False: lg_pool_head_bwd first
_FUSED_HEADS = True


def _heads_backward_launches(lib, dl, h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr, inc_item, sched,
                             sched_hdr, P, B, N, D, hidden, nhidden, fe, fn, p_edge, p_noleak, dpipe, dh, dw1, db1, dw2,
                             db2, ndw1, ndb1, ndw2, ndb2, ws, wsn, st):
    """NoLeakHead backward first (its dpooled feeds the node rows), then the EdgeHead backward
    with the incidence scatter fused in (lg_edge_head_bwd_scatter): dh complete."""
    dev = h.device
    dpooled = torch.empty(B, D, device=dev)
    lay = fe & nat.LG_F_NODE_MAJOR
    if _FUSED_SCATTER and _FUSED_HEADS:
        # both heads in one launch where the streamed form applies (else the two calls inside)
        with _timed("edge_bwd", dev):
            hdr = (ctypes.c_int32 * 16)(*sched_hdr) if (sched is not None and sched_hdr) else None
            check(lib.lg_heads_bwd_scatter(ptr(pooled), ptr(hid), ptr(nw1), ptr(nw2), ptr(ndw1), ptr(ndb1), ptr(ndw2),
                                           ptr(ndb2), fn, p_noleak, ptr(wsn), wsn.numel(), ptr(ends), ptr(h), ptr(w1),
                                           ptr(w2), ptr(ehid), ptr(dl), P + 1, ptr(dpipe), ptr(dw1), ptr(db1), ptr(dw2),
                                           ptr(db2), ptr(inc_rowptr), ptr(inc_item), ptr(sched) if hdr else None, hdr,
                                           ptr(dpooled), ptr(dh), B, N, P, D, hidden, fe, p_edge, ptr(ws), ws.numel(),
                                           st), "lg_heads_bwd_scatter")
        return
    with _timed("pool_head_bwd", dev):
        check(lib.lg_pool_head_bwd(ptr(pooled), ptr(hid), ptr(nw1), ptr(nw2), ptr(dl), P + 1, P, ptr(dpooled),
                                   ptr(ndw1), ptr(ndb1), ptr(ndw2), ptr(ndb2), B, D, nhidden, fn, p_noleak, ptr(wsn), wsn.numel(),
                                   st), "lg_pool_head_bwd")
    if _FUSED_SCATTER:
        with _timed("edge_bwd", dev):
            hdr = (ctypes.c_int32 * 16)(*sched_hdr) if (sched is not None and sched_hdr) else None
            check(lib.lg_edge_head_bwd_scatter(ptr(ends), ptr(h), ptr(w1), ptr(w2), ptr(ehid), ptr(dl), P + 1,
                                               ptr(dpipe), ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), ptr(inc_rowptr),
                                               ptr(inc_item), ptr(sched) if hdr else None, hdr, ptr(dpooled), ptr(dh),
                                               B, N, P, D, hidden, fe, p_edge, ptr(ws), ws.numel(), st),
                  "lg_edge_head_bwd_scatter")
        return
    with _timed("edge_bwd", dev):
        check(lib.lg_edge_head_bwd(ptr(ends), ptr(h), ptr(w1), ptr(w2), ptr(ehid), ptr(dl), P + 1, ptr(dpipe),
                                   ptr(dw1), ptr(db1), ptr(dw2), ptr(db2), B, N, P, D, hidden, fe, p_edge,
                                   ptr(ws), ws.numel(), st), "lg_edge_head_bwd")
    with _timed("pipe_scatter", dev):
        check(lib.lg_pipe_scatter_bwd(ptr(inc_rowptr), ptr(inc_item), ptr(dpipe), ptr(dpooled), ptr(dh), B, N, P, D,
                                      lay, st), "lg_pipe_scatter_bwd")


@detector_heads_backward.register_fake
def _(dlogits, h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr, inc_item, sched, sched_hdr, p_edge, p_noleak,
      node_major, *, bf16=False):
    H, NH = w1.shape[0], nw1.shape[0]
    return (torch.empty_like(h), torch.empty_like(w1), w1.new_empty(H), torch.empty_like(w2), w2.new_empty(1),
            torch.empty_like(nw1), nw1.new_empty(NH), torch.empty_like(nw2), nw2.new_empty(1))


def _heads_setup(ctx, inputs, keyword_only_inputs, output):
    (h, w1, b1, w2, b2, nw1, nb1, nw2, nb2, ends, inc_rowptr, inc_item, p_edge, p_noleak, node_major, _, _) = inputs[:17]
    sched = inputs[17] if len(inputs) > 17 else None
    sched_hdr = inputs[18] if len(inputs) > 18 else None
    bf16 = bool(keyword_only_inputs.get("bf16", False))
    _, ehid, pooled, hid = output
    ctx.mark_non_differentiable(ehid, pooled, hid)
    ctx.set_materialize_grads(False)  # else autograd zero-fills a (B*P, 128) gradient for ehid
    ctx.cfg = (p_edge, p_noleak, node_major, bf16, list(sched_hdr or []) if sched is not None else [])
    ctx.nin = len(inputs)
    ctx.save_for_backward(h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr, inc_item, sched)


def _heads_bwd(ctx, dlogits, _dehid, _dpooled, _dhid):
    if dlogits is None:
        return (None,) * ctx.nin
    h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr, inc_item, sched = ctx.saved_tensors
    p_edge, p_noleak, node_major, bf16, hdr = ctx.cfg
    g = torch.ops.leakgnn.detector_heads_backward(dlogits, h, w1, w2, ehid, pooled, hid, nw1, nw2, ends, inc_rowptr,
                                                  inc_item, sched, hdr, p_edge, p_noleak, node_major, bf16=bf16)
    return tuple(g) + (None,) * (ctx.nin - 9)


detector_heads.register_autograd(_heads_bwd, setup_context=_heads_setup)


# ============================================================================ module-facing helpers
def seed_tensor(device: torch.device) -> Tensor:
    """The dropout seed of one call site as a tensor (see ops._new_seed): a CPU int64 value
    drawn from torch's CPU generator in eager mode; under HIP-graph capture a device word
    re-drawn on every replay (a SeedSlots slot, or torch's graph-safe CUDA generator)."""
    from . import ops
    if ops._SEED_SLOTS is not None:
        return ops._SEED_SLOTS.take_tensor()
    if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
        return torch.randint(0, 2 ** 62, (1,), dtype=torch.long, device=device)
    return torch.randint(0, 2 ** 62, (1,), dtype=torch.long)


def detector_ops_available() -> bool:
    return hasattr(torch.ops, NS) and hasattr(torch.ops.leakgnn, "gnn_trunk")
