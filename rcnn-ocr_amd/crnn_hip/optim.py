"""Fused AdamW over the model's flat fp32 parameter/gradient buffers (one launch).

Update rule of torch.optim.AdamW (the reference's AdamW option, training/train.py:294-295):
  p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = b2 v + (1-b2) g^2 ;
  p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
"""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import call, ptr


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        params = list(model.parameters())
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.model = model
        self.step_count = 0
        self._m = None
        self._v = None

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        m = self.model
        flat, gflat = m._flat_param, m._flat_grad
        if flat is None:
            raise RuntimeError("FusedAdamW needs the model to have run once on the device (flat buffers)")
        L.require_device(flat)
        if self._m is None or self._m.numel() != flat.numel():
            self._m = torch.zeros_like(flat)
            self._v = torch.zeros_like(flat)
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        call("crnn_adamw", ptr(flat), ptr(gflat), ptr(self._m), ptr(self._v), flat.numel(), float(g["lr"]),
             float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), self.step_count, float(grad_scale),
             L.stream_ptr())
        m.mark_params_changed()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics. set_to_none: .grad becomes None and the next backward re-attaches the
        flat-buffer views and OVERWRITES them (no memset); otherwise the flat buffer is zeroed and
        the next backward accumulates into it."""
        if set_to_none:
            for p in self.model.parameters():
                p.grad = None
        elif self.model._flat_grad is not None:
            self.model._flat_grad.zero_()
