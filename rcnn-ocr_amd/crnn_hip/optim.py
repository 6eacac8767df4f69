"""Fused optimizers over the model's flat fp32 parameter/gradient buffers (one launch each).

The reference picks its optimizer by name (training/train.py:292-301, `cfg.optimizer`, default
"Adam"):
  FusedAdam   torch.optim.Adam   : g += wd*p (coupled L2) ; m = lerp(m, g, 1-b1) ;
                                   v = b2 v + (1-b2) g^2 ; p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
  FusedAdamW  torch.optim.AdamW  : p *= 1 - lr*wd (decoupled), then the same moment update
  FusedSGD    torch.optim.SGD    : d = g + wd*p ; buf = d (first step) | momentum*buf + d ; p -= lr*buf

The moments live in flat fp32 buffers in parameter order (one kernel, one pass). The checkpoint
format is torch's: state_dict()["state"][i] = {"step", "exp_avg", "exp_avg_sq"} (Adam / AdamW) or
{"momentum_buffer"} (SGD) per parameter, so save_checkpoint / load_checkpoint
(training/utils.py:24-58) resume them, and a reference checkpoint of the same optimizer loads here
(and the other way round).

Every update is guarded on the device by the persistent BiLSTM's sticky status word (crnn_hip.h
crnn_adam_step `skip`): a sweep that timed out leaves NaN gradients, and the kernel then leaves
weights and moments untouched; the host raises at the engine's next status poll.
"""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import call, ptr


def _skip_word(model):
    eng = getattr(model, "_engine", None)
    return eng.status_word() if eng is not None else None


class _FlatOptimizer(torch.optim.Optimizer):
    """shared plumbing: the model's flat buffers, state views for torch's state_dict format."""

    _state_keys = ()

    def __init__(self, model, defaults):
        params = list(model.parameters())
        super().__init__(params, defaults)
        self.model = model
        self.step_count = 0
        self._bufs = None       # flat state buffers, one per _state_keys entry

    def _params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _alloc_state(self, flat):
        """zeroed state, or the one a load_state_dict left in self.state, in flat order"""
        self._bufs = [torch.zeros_like(flat) for _ in self._state_keys]
        off = 0
        for p in self._params():
            n = p.numel()
            st = self.state.get(p)
            for k, b in zip(self._state_keys, self._bufs):
                if st and k in st and st[k] is not None:
                    b[off:off + n].copy_(st[k].reshape(-1))
            off += n
        if off != flat.numel():
            raise RuntimeError(f"{type(self).__name__}: the model's flat buffer does not hold exactly the optimizer's "
                               "parameters")
        self._bind_state()

    def _bind_state(self):
        """self.state[p] = views of the flat state (what torch's state_dict() serialises)"""
        off = 0
        for p in self._params():
            n = p.numel()
            st = self._state_extra()
            for k, b in zip(self._state_keys, self._bufs):
                st[k] = b[off:off + n].view_as(p)
            self.state[p] = st
            off += n

    def _state_extra(self):
        return {}

    def _flat(self):
        m = self.model
        flat, gflat = m._flat_param, m._flat_grad
        if flat is None:
            raise RuntimeError(f"{type(self).__name__} needs the model to have run once on the device (flat buffers)")
        L.require_device(flat)
        if self._bufs is None or self._bufs[0].numel() != flat.numel() or self._bufs[0].device != flat.device:
            self._alloc_state(flat)
        return flat, gflat

    def state_dict(self):
        if self._bufs is not None:
            self._bind_state()      # refresh "step"; the state views already alias the flat buffers
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._after_load()
        flat = self.model._flat_param
        if flat is not None:
            self._alloc_state(flat)   # copy into the flat buffers now (views replace the loaded tensors)
        else:
            self._bufs = None         # copied at the first step(), once the flat buffers exist

    def _after_load(self):
        pass

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics. set_to_none: .grad becomes None and the next backward re-attaches the
        flat-buffer views and OVERWRITES them (no memset); otherwise the flat buffer is zeroed and
        the next backward accumulates into it."""
        if set_to_none:
            for p in self.model.parameters():
                p.grad = None
        elif self.model._flat_grad is not None:
            self.model._flat_grad.zero_()


class FusedAdam(_FlatOptimizer):
    """torch.optim.Adam (coupled L2 weight decay): the reference's default optimizer
    (training/train.py:219,292-293, configs/config.json "optimizer": "Adam")."""

    coupled = True
    _state_keys = ("exp_avg", "exp_avg_sq")

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(model, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    def _state_extra(self):
        return {"step": torch.tensor(float(self.step_count))}

    def _after_load(self):
        steps = {int(float(st["step"])) for st in self.state.values() if "step" in st}
        if len(steps) > 1:
            raise ValueError(f"{type(self).__name__} keeps one step count for all parameters, checkpoint has "
                             f"{sorted(steps)}")
        self.step_count = steps.pop() if steps else 0

    @property
    def _m(self):
        return None if self._bufs is None else self._bufs[0]

    @property
    def _v(self):
        return None if self._bufs is None else self._bufs[1]

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        flat, gflat = self._flat()
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        call("crnn_adam_step", ptr(flat), ptr(gflat), ptr(self._bufs[0]), ptr(self._bufs[1]), flat.numel(),
             float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), self.step_count,
             float(grad_scale), 1 if self.coupled else 0, ptr(_skip_word(self.model)), L.stream_ptr())
        self.model.mark_params_changed()
        return loss


class FusedAdamW(FusedAdam):
    """torch.optim.AdamW (decoupled weight decay; training/train.py:294-295)."""

    coupled = False

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)


class FusedSGD(_FlatOptimizer):
    """torch.optim.SGD with momentum (training/train.py:296-299; dampening 0, no Nesterov)."""

    _state_keys = ("momentum_buffer",)

    def __init__(self, model, lr=1e-3, momentum=0.0, weight_decay=0.0):
        super().__init__(model, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, dampening=0,
                                     nesterov=False, maximize=False))
        self._have_buf = False

    def _after_load(self):
        self._have_buf = any(st.get("momentum_buffer") is not None for st in self.state.values())
        self.step_count = 1 if self._have_buf else 0

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        flat, gflat = self._flat()
        g = self.param_groups[0]
        mom = float(g["momentum"])
        call("crnn_sgd_step", ptr(flat), ptr(gflat), ptr(self._bufs[0]), flat.numel(), float(g["lr"]), mom,
             float(g["weight_decay"]), float(grad_scale), 0 if self._have_buf else 1, ptr(_skip_word(self.model)),
             L.stream_ptr())
        self._have_buf = mom != 0.0
        self.step_count += 1
        self.model.mark_params_changed()
        return loss


def make_optimizer(name: str, model, lr: float, weight_decay: float = 0.0, momentum: float = 0.9):
    """training/train.py:292-301: "Adam" | "AdamW" | "SGD" -> the fused equivalent."""
    if name == "Adam":
        return FusedAdam(model, lr=lr, weight_decay=weight_decay)
    if name == "AdamW":
        return FusedAdamW(model, lr=lr, weight_decay=weight_decay)
    if name == "SGD":
        return FusedSGD(model, lr=lr, momentum=momentum, weight_decay=weight_decay)
    raise ValueError(f"Unknown optimizer: {name}")
