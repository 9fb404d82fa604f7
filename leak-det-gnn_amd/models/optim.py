"""clip_grad_norm_ + AdamW as one launch (reference train_detector.py:313-317).

The reference ends every step with

    torch.nn.utils.clip_grad_norm_(model.parameters(), grad_clip)
    opt.step()                      # torch.optim.AdamW(lr, weight_decay)

which torch runs as ~11 launches for the detector's ~60k parameters (foreach norms, the
norm of norms, clamp, foreach mul, the fused AdamW).  ClipAdamW does both in ONE HIP
launch (lg_clip_adamw, csrc/optim.hip: every workgroup sums the squares of its own slice, a
grid barrier, then every workgroup sums the slice partials in a fixed order and updates its
slice; two launches past one slice per CU): the same AdamW arithmetic (decoupled weight
decay, bias corrections, amsgrad=False) on gradients scaled by
min(1, max_norm / (||g||_2 + 1e-6)), written back to .grad as clip_grad_norm_ does.  The
step counter is device-resident, so the step can be captured in a HIP graph
(models/graph_step.py) — pass max_norm here and clip=None there.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional

import torch

from ._native import check, load_library, stream_of


class ClipAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW(params, lr, betas, eps, weight_decay) preceded by
    clip_grad_norm_(params, max_norm) (max_norm None: no clipping), fp32 CUDA parameters.
    State per parameter: exp_avg, exp_avg_sq (torch's names); one device step counter per
    group.  After step(), `last_grad_norm` is the device tensor of the pre-clip total norm
    (what clip_grad_norm_ returns)."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, max_norm: Optional[float] = None):
        if not 0.0 <= lr:
            raise ValueError(f"invalid lr {lr}")
        # capturable: the step counter is device-resident (models/graph_step.py checks the flag)
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      max_norm=max_norm, capturable=True))
        self.last_grad_norm: Optional[torch.Tensor] = None
        self._ws: dict = {}  # group index -> per-slice partial-norm workspace (fp64 per 1024 elements)
        # ops.SeedSlots whose next draw step() makes in its own launch (lg_clip_adamw_seeds):
        # set by graph_step.CapturedTrainStep while it captures the step, so the step ends by
        # drawing the next replay's dropout seeds instead of starting with a launch of its own
        self.seed_slots = None

    def load_state_dict(self, state_dict) -> None:
        super().load_state_dict(state_dict)
        for group in self.param_groups:  # words 1-3 are the launch's counter / error word: 0 between launches
            st = group.get("step_t")
            if torch.is_tensor(st):
                if st.numel() < 4:  # a state dict from before ABI 25 ([step, ticket])
                    st = group["step_t"] = torch.cat([st.reshape(-1)[:1], st.new_zeros(3)])
                st[1:].zero_()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = load_library()
        live = [g for g in self.param_groups if any(p.grad is not None for p in g["params"])]
        if len(live) > 1 and any(g["max_norm"] is not None for g in live):
            # clip_grad_norm_(model.parameters()) takes ONE norm over every parameter; the fused
            # launch clips per group, which equals it only for a single group
            raise RuntimeError("ClipAdamW: max_norm with more than one param group is not supported "
                               "(clip_grad_norm_ takes one norm over all parameters); use one group")
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32
                        and p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("ClipAdamW takes contiguous fp32 CUDA parameters and gradients")
                st = self.state[p]
                if not st:
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
            if "step_t" not in group:
                # [step, the launch's arrival / ticket counter (uint32 bits, 0 between launches),
                #  error word (uint32, nonzero if a grid-barrier wait timed out), reserved]
                group["step_t"] = torch.zeros(4, dtype=torch.float32, device=params[0].device)
            if self.last_grad_norm is None:
                self.last_grad_norm = torch.zeros(1, dtype=torch.float32, device=params[0].device)
            if len(params) > 48:
                raise RuntimeError("ClipAdamW: at most 48 parameter tensors per group (one launch)")
            # host arrays, passed by value into the launch (capturable: no host->device copy)
            table = (ctypes.c_int64 * (4 * len(params)))(*[x for p in params for x in (
                p.data_ptr(), p.grad.data_ptr(), self.state[p]["exp_avg"].data_ptr(),
                self.state[p]["exp_avg_sq"].data_ptr())])
            sizes = (ctypes.c_int64 * len(params))(*[p.numel() for p in params])
            ws = self._ws.get(gi)
            nws = int(lib.lg_clip_adamw_workspace_bytes(ctypes.addressof(sizes), len(params)))
            if ws is None or ws.numel() < nws:
                ws = self._ws[gi] = torch.empty(nws, dtype=torch.uint8, device=params[0].device)
            b1, b2 = group["betas"]
            mn = group["max_norm"]
            args = (ctypes.addressof(table), ctypes.addressof(sizes), len(params), group["step_t"].data_ptr(),
                    float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]),
                    float(mn) if mn is not None else 0.0, self.last_grad_norm.data_ptr(), ws.data_ptr(), ws.numel())
            sl = self.seed_slots if gi == len(self.param_groups) - 1 else None  # the last group's launch draws them
            if sl is not None:
                check(lib.lg_clip_adamw_seeds(*args, sl.buf.data_ptr(), sl.n, sl.state.data_ptr(), stream_of(params[0])),
                      "lg_clip_adamw_seeds")
            else:
                check(lib.lg_clip_adamw(*args, stream_of(params[0])), "lg_clip_adamw")
        return loss
