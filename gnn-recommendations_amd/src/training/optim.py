"""Adam for the training path on the GPU: torch.optim.Adam's algorithm and
state (the reference's optimizer, trainer.py:59-63: Adam with L2 weight decay) with the
update as one native kernel per parameter (gnnrec_adam_step_f32). At G100M the embedding
tables are 128M parameters and the update is a pure HBM stream; torch's multi-tensor and
fused forms split it into 28-75 launches per step. The gradient clip coefficient can be
passed in (`grad_scale`) instead of scaling the gradient in place first.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..ops import _lib
from ..ops._lib import check, ptr


class NativeAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or weight_decay < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1):
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[torch.Tensor] = None):
        """One Adam step; `grad_scale` (0-d fp32 device tensor) multiplies every gradient
        first (clip_grad_norm_'s coefficient)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = _lib.lib()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                        and p.grad.is_contiguous() and not p.grad.is_sparse):
                    raise ValueError("NativeAdam needs contiguous fp32 ROCm parameters/grads")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                t = float(st["step"])
                step_size = group["lr"] / (1 - b1 ** t)
                bc2_sqrt = math.sqrt(1 - b2 ** t)
                scale = None
                if grad_scale is not None:
                    scale = grad_scale.to(device=p.device, dtype=torch.float32).reshape(())
                check(L.gnnrec_adam_step_f32(ptr(p), ptr(p.grad), ptr(st["exp_avg"]),
                                             ptr(st["exp_avg_sq"]), p.numel(), step_size, b1,
                                             b2, bc2_sqrt, group["eps"], group["weight_decay"],
                                             ptr(scale), _lib.stream_of(p.device)),
                      "gnnrec_adam_step_f32")
        return loss
