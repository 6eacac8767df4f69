"""Fused AdamW over the model's flat fp32 parameter/gradient buffers (one launch).

Update rule of torch.optim.AdamW (the reference's AdamW option, training/train.py:294-295):
  p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = b2 v + (1-b2) g^2 ;
  p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)

The moments live in two flat fp32 buffers in parameter order (one kernel, one pass). The
checkpoint format is torch.optim.AdamW's: state_dict()["state"][i] = {"step", "exp_avg",
"exp_avg_sq"} per parameter, so save_checkpoint / load_checkpoint (training/utils.py:24-58)
resume the moments and the step count, and an AdamW checkpoint of the reference loads here
(and the other way round).
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

    def _params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _alloc_moments(self, flat):
        """zeroed moments, or the ones a load_state_dict left in self.state, in flat order"""
        self._m = torch.zeros_like(flat)
        self._v = torch.zeros_like(flat)
        off = 0
        for p in self._params():
            n = p.numel()
            st = self.state.get(p)
            if st and "exp_avg" in st:
                self._m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                self._v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
            off += n
        if off != flat.numel():
            raise RuntimeError("FusedAdamW: the model's flat buffer does not hold exactly the optimizer's parameters")
        self._bind_state()

    def _bind_state(self):
        """self.state[p] = views of the flat moments (what torch's state_dict() serialises)"""
        off = 0
        for p in self._params():
            n = p.numel()
            self.state[p] = {"step": torch.tensor(float(self.step_count)),
                             "exp_avg": self._m[off:off + n].view_as(p),
                             "exp_avg_sq": self._v[off:off + n].view_as(p)}
            off += n

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        m = self.model
        flat, gflat = m._flat_param, m._flat_grad
        if flat is None:
            raise RuntimeError("FusedAdamW needs the model to have run once on the device (flat buffers)")
        L.require_device(flat)
        if self._m is None or self._m.numel() != flat.numel() or self._m.device != flat.device:
            self._alloc_moments(flat)
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        call("crnn_adamw", ptr(flat), ptr(gflat), ptr(self._m), ptr(self._v), flat.numel(), float(g["lr"]),
             float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), self.step_count, float(grad_scale),
             L.stream_ptr())
        m.mark_params_changed()
        return loss

    def state_dict(self):
        if self._m is not None:
            self._bind_state()      # refresh "step"; the moment views already alias the flat buffers
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        steps = {int(float(st["step"])) for st in self.state.values() if "step" in st}
        if len(steps) > 1:
            raise ValueError(f"FusedAdamW keeps one step count for all parameters, checkpoint has {sorted(steps)}")
        self.step_count = steps.pop() if steps else 0
        flat = self.model._flat_param
        if flat is not None:
            self._alloc_moments(flat)   # copy into the flat buffers now (views replace the loaded tensors)
        else:
            self._m = self._v = None    # copied at the first step(), once the flat buffers exist

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics. set_to_none: .grad becomes None and the next backward re-attaches the
        flat-buffer views and OVERWRITES them (no memset); otherwise the flat buffer is zeroed and
        the next backward accumulates into it."""
        if set_to_none:
            for p in self.model.parameters():
                p.grad = None
        elif self.model._flat_grad is not None:
            self.model._flat_grad.zero_()
