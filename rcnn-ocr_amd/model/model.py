"""RCNN with the reference's API (sherstpasha/RCNN-OCR model/model.py:166-227),
running SE-ResNet31 -> BiLSTM -> CTC head on the MI355X HIP engine.

    RCNN(num_classes, hidden_size=256, sos_id=1, eos_id=2, pad_id=0, blank_id=3,
         enc_dropout_p=0.1, dropblock_p=0.0, dropblock_block_size=5,
         decoder="ctc", num_rnn_layers=2, compute_dtype=torch.bfloat16)
    .encode(x [B,3,H,W]) -> [B, T=W/8, hidden]        (model/model.py:215-221)
    .forward(x, text=None, is_train=True, batch_max_length=25) -> CTC logits [B, T, C]

State-dict keys are the reference's (cnn.*, enc_rnn.*) plus ctc_head.{weight,bias} for
decoder="ctc" (the reference's training head is an attention decoder; this path is
CTC), or plus the reference's attn.* for decoder="attn" — exactly the reference's key set, so its
checkpoints load strictly.
Every forward/backward runs in libcrnn_hip.so; there is no CPU path — on a CPU
tensor the module raises.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from crnn_hip import _lib as L
from crnn_hip.engine import CRNNEngine, round8
from model.seresnet31 import DropBlock2d, SEResNet31


class BidirectionalLSTM(nn.Module):
    """parameter container with the reference's names (model/model.py:151-163)."""

    def __init__(self, input_size, hidden_size, output_size):
        super().__init__()
        if output_size != hidden_size:
            raise NotImplementedError("the HIP BiLSTM stack keeps output_size == hidden_size")
        self.rnn = nn.LSTM(input_size, hidden_size, bidirectional=True, batch_first=True)
        self.linear = nn.Linear(hidden_size * 2, output_size)

    def forward(self, x):
        raise NotImplementedError("BiLSTM layers run inside the HIP engine; call RCNN.encode/forward")


def _noop():
    return None


class _EncodeFn(torch.autograd.Function):
    """images -> logits via the engine; backward writes parameter gradients
    straight into the flat grad buffer (the params' .grad views)."""

    @staticmethod
    def forward(ctx, anchor, images, model, need_grad):
        eng = model._engine_for(images)
        logits = eng.forward(images, train=model.training, save_for_backward=need_grad,
                             update_running=model.training, **model._drop_kwargs())
        ctx.model = model
        ctx.gen = eng.fwd_gen
        return logits.clone()

    @staticmethod
    def backward(ctx, grad_logits):
        model = ctx.model
        eng = model._engine
        eng.check_generation(ctx.gen)
        B, T, C = grad_logits.shape
        dl = eng.ws.get("autograd.dlogits", (B, T, eng.Cpad), torch.float32)
        if getattr(eng, "_dl_pad_ptr", None) != dl.data_ptr():   # pad columns: zeroed once per buffer
            dl[:, :, C:].zero_()
            eng._dl_pad_ptr = dl.data_ptr()
        dl[:, :, :C].copy_(grad_logits)
        grads, accumulate, attach = model._grad_views()
        eng.backward(dl, grads, accumulate=accumulate, stage_done=model.stage_done)
        attach()
        return None, None, None, None


class _AttnTrainFn(torch.autograd.Function):
    """images, text -> teacher-forced attention logits [B, steps, V]; backward: the decoder's BPTT
    (crnn_hip/attn.py) hands d enc to the engine's encoder backward (model/model.py:223-227)."""

    @staticmethod
    def forward(ctx, anchor, images, text, model, steps):
        eng = model._engine_for(images)
        kw = model._drop_kwargs()
        p = kw["dropout_p"]
        eng.forward(images, train=model.training, save_for_backward=True, update_running=model.training, **kw)
        key = "enc.drop" if p > 0.0 else f"r{model.num_rnn_layers - 1}.out"
        enc = eng.ws.bufs[key].float()
        dec = model._attn_decoder(enc.device)
        ap = model.attn_dropout_p if model.training else 0.0
        model._attn_seed = (model._attn_seed + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
        ctx.model = model
        ctx.gen = eng.fwd_gen     # the decoder's saved state is replaced together with the engine's
        return dec.run_train(enc, steps, text, drop_p=ap, seed=model._attn_seed)

    @staticmethod
    def backward(ctx, grad_logits):
        model = ctx.model
        model._engine.check_generation(ctx.gen)
        grads, accumulate, attach = model._grad_views()
        attn_grads = {k[len("attn."):]: v for k, v in grads.items() if k.startswith("attn.")}
        denc = model._attn_dec.backward(grad_logits.contiguous(), attn_grads, accumulate)
        if model.stage_done is not None:   # the decoder's gradients are final before the encoder's
            model.stage_done(["attn."])
        model._engine.backward(None, grads, accumulate=accumulate, denc=denc, stage_done=model.stage_done)
        attach()
        return None, None, None, None, None


class _AttentionCellParams(nn.Module):
    """parameter holder with model/model.py:24-31's names (AttentionCell)."""

    def __init__(self, input_size, hidden_size, num_embeddings):
        super().__init__()
        self.i2h = nn.Linear(input_size, hidden_size, bias=False)
        self.h2h = nn.Linear(hidden_size, hidden_size)
        self.score = nn.Linear(hidden_size, 1, bias=False)
        self.rnn = nn.LSTMCell(input_size + num_embeddings, hidden_size)


class _AttentionParams(nn.Module):
    """parameter holder with model/model.py:48-79's names (Attention: attention_cell, generator)."""

    def __init__(self, input_size, hidden_size, num_classes):
        super().__init__()
        self.attention_cell = _AttentionCellParams(input_size, hidden_size, num_classes)
        self.generator = nn.Linear(hidden_size, num_classes)


class RCNN(nn.Module):
    def __init__(self, num_classes, hidden_size=256, sos_id: int = 1, eos_id: int = 2, pad_id: int = 0,
                 blank_id: Optional[int] = 3, enc_dropout_p: float = 0.1, dropblock_p: float = 0.0,
                 dropblock_block_size: int = 5, decoder: str = "ctc", num_rnn_layers: int = 2,
                 compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        if decoder not in ("ctc", "attn"):
            raise ValueError(f"decoder must be 'ctc' or 'attn', got {decoder!r}")
        self.num_classes = num_classes
        self.hidden_size = hidden_size
        self.sos_id, self.eos_id, self.pad_id, self.blank_id = sos_id, eos_id, pad_id, blank_id
        self.decoder = decoder
        self.num_rnn_layers = num_rnn_layers
        self.compute_dtype = compute_dtype
        self.cnn = SEResNet31(in_channels=3, out_channels=512, dropblock_p=dropblock_p,
                              dropblock_block_size=dropblock_block_size)
        self.pool = nn.AdaptiveAvgPool2d((1, None))
        enc_dim = self.cnn.out_channels
        layers = [BidirectionalLSTM(enc_dim, hidden_size, hidden_size)]
        layers += [BidirectionalLSTM(hidden_size, hidden_size, hidden_size) for _ in range(1, num_rnn_layers)]
        self.enc_rnn = nn.Sequential(*layers)
        self.enc_dropout = nn.Dropout(enc_dropout_p)
        self.ctc_head = nn.Linear(hidden_size, num_classes) if decoder == "ctc" else None
        # the reference's attention head (model/model.py:23-79, :203-213): parameter holder with the
        # reference's state_dict names; compute on the HIP path (crnn_hip/attn.py), forward + backward
        self.attn = _AttentionParams(hidden_size, hidden_size, num_classes) if decoder == "attn" else None
        self._attn_dec = None
        self._attn_version = None
        self.attn_dropout_p = 0.1    # Attention(dropout_p=0.1) in the reference RCNN (model/model.py:203-213)
        self._attn_seed = 0x5EED
        self._engine: Optional[CRNNEngine] = None
        self._flat_param: Optional[torch.Tensor] = None
        self._flat_grad: Optional[torch.Tensor] = None
        self._gv_cache = None   # (flat grad buffer, [(name, param, grad view)], {name: view})
        # data parallel: called by every backward with the parameter-name prefixes whose gradients
        # have become final (crnn_hip.dist.OverlappedAllReduce.ready), so the gradient all-reduce
        # overlaps the rest of the backward; None = single process
        self.stage_done = None
        # the SE blocks' DropBlock2d (all blocks share p and block_size), kept out of the module tree
        self._dropblock = [next((m for m in self.cnn.modules() if isinstance(m, DropBlock2d)), None)]

    def _drop_kwargs(self) -> Dict[str, float]:
        """the engine's training-mode regularisers: enc_dropout (model/model.py:201,220) and the SE
        blocks' DropBlock2d (model/seresnet31.py:49-53,62); none in eval."""
        if not self.training:
            return dict(dropout_p=0.0)
        db = self._dropblock[0]
        return dict(dropout_p=self.enc_dropout.p, dropblock_p=db.p if db is not None else 0.0,
                    dropblock_block_size=db.block_size if db is not None else 5)

    # ------------------------------------------------------------------ engine plumbing
    def _param_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v for k, v in self.named_parameters()}

    def _buffer_dict(self) -> Dict[str, torch.Tensor]:
        return {k: v for k, v in self.named_buffers()}

    def flatten_parameters_(self):
        """Make every parameter (and its .grad) a view into one fp32 buffer: one fused
        AdamW launch and one RCCL all-reduce cover the whole model."""
        params = list(self.parameters())
        dev = params[0].device
        n = sum(p.numel() for p in params)
        if self._flat_param is not None and self._flat_param.device == dev:
            return
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        gflat = torch.zeros(n, dtype=torch.float32, device=dev)
        off = 0
        for p in params:
            k = p.numel()
            flat[off:off + k].copy_(p.data.reshape(-1))
            p.data = flat[off:off + k].view_as(p)
            p.grad = gflat[off:off + k].view_as(p)
            off += k
        self._flat_param, self._flat_grad = flat, gflat
        self._grad_offsets = None
        self._gv_cache = None

    def flat_offsets(self):
        """{parameter name: (start, numel)} in the flat buffer (parameter order: stem first, head last)."""
        out, off = {}, 0
        for n, p in self.named_parameters():
            out[n] = (off, p.numel())
            off += p.numel()
        return out

    def _grad_views(self):
        """-> (name -> grad tensor, accumulate?, attach). The flat buffer's gradient views are built
        once per buffer. After zero_grad(set_to_none=True) the backward OVERWRITES them (accumulate
        False) and attach() makes them the parameters' .grad again: the caller calls it after it has
        enqueued the backward kernels, so the host-side .grad assignments (one per parameter) run
        while the GPU works instead of delaying the first backward launch (profiles/r03x_*: a 0.2 ms
        GPU bubble per step). Some grads None, some not: the None ones are zeroed and attached first
        and the backward accumulates."""
        c = self._gv_cache
        if c is None or c[0] is not self._flat_grad:
            items, off = [], 0
            for n, p in self.named_parameters():
                k = p.numel()
                items.append((n, p, self._flat_grad[off:off + k].view_as(p)))
                off += k
            c = self._gv_cache = (self._flat_grad, items, {n: v for n, _, v in items})
        _, items, views = c
        missing = [(p, v) for _, p, v in items if p.grad is None]
        if not missing:
            return {n: p.grad for n, p, _ in items}, True, _noop
        if len(missing) == len(items):
            def attach():
                for p, v in missing:
                    p.grad = v
            return views, False, attach
        for p, v in missing:
            v.zero_()
            p.grad = v
        return {n: p.grad for n, p, _ in items}, True, _noop

    def _engine_for(self, images: torch.Tensor) -> CRNNEngine:
        L.require_device(images)
        dev = images.device
        if self._engine is None or self._engine.device != dev or self._flat_param is None \
                or self._flat_param.device != dev:
            if next(self.parameters()).device != dev:
                raise RuntimeError("model parameters and images must be on the same HIP device")
            self.flatten_parameters_()
            self._engine = CRNNEngine(self._param_dict(), self._buffer_dict(), self.hidden_size,
                                      self.num_classes, self.num_rnn_layers, self.compute_dtype,
                                      version_source=self._param_version)
        return self._engine

    def _param_version(self) -> int:
        # torch optimizers / load_state_dict modify parameters in place, bumping _version
        return sum(p._version for p in self.parameters())

    def mark_params_changed(self):
        """call after modifying parameters in place (optimizer steps do this via hooks)."""
        if self._engine is not None:
            self._engine.mark_params_changed()
        self._attn_version = None   # the attention decoder re-reads its weights on next use

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.mark_params_changed()
        return r

    def _attn_decoder(self, device):
        from crnn_hip.attn import AttnDecoderHIP
        ver = sum(p._version for p in self.attn.parameters())
        if self._attn_dec is None or self._attn_version != ver or self._attn_dec.device != device:
            params = {k: v for k, v in self.attn.state_dict().items()}
            if self._attn_dec is not None and self._attn_dec.device == device:
                self._attn_dec.refresh(params)
            else:
                self._attn_dec = AttnDecoderHIP(params, self.num_classes, self.sos_id, self.blank_id, device,
                                                train_bf16=self.compute_dtype == torch.bfloat16)
            self._attn_version = ver
        return self._attn_dec

    def _attn_forward(self, x, text, is_train, batch_max_length):
        steps = batch_max_length + 1
        if is_train and text is None:
            raise ValueError("For training, `text` with <SOS> at text[:,0] is required")
        anchor = next(self.parameters())
        if is_train and torch.is_grad_enabled() and anchor.requires_grad:
            self._engine_for(x)
            return _AttnTrainFn.apply(anchor, x, text, self, steps)
        enc = self.encode(x)
        dec = self._attn_decoder(enc.device)
        if not is_train:
            return dec.run(enc, steps)
        return dec.run(enc, steps, text=text)

    # ------------------------------------------------------------------ reference API
    def encode(self, x):
        """RCNN.encode (model/model.py:215-221): [B,3,H,W] -> [B, W/8, hidden] (inference)."""
        eng = self._engine_for(x)
        kw = self._drop_kwargs()
        p = kw["dropout_p"]
        with torch.no_grad():
            eng.forward(x, train=self.training, save_for_backward=False, update_running=self.training, **kw)
        key = "enc.drop" if p > 0.0 else f"r{self.num_rnn_layers - 1}.out"   # after enc_dropout (model.py:220)
        return eng.ws.bufs[key].float().clone()

    def forward(self, x, text=None, is_train=True, batch_max_length=25):
        """decoder='ctc': CTC logits [B, T, num_classes] (fp32); `text` / `batch_max_length` are
        ignored (CTC is alignment-free). decoder='attn': the reference's RCNN.forward
        (model/model.py:223-227) — greedy-decode logits [B, batch_max_length+1, num_classes] when
        is_train is False, teacher-forced logits from `text` (<SOS> at text[:, 0]) otherwise; with
        grad enabled the teacher-forced path is differentiable end to end (decoder BPTT + encoder
        backward on the HIP path; attention-weight dropout p=attn_dropout_p in training mode)."""
        if self.decoder == "attn":
            return self._attn_forward(x, text, is_train, batch_max_length)
        self._engine_for(x)
        anchor = next(self.parameters())
        return _EncodeFn.apply(anchor, x, self, torch.is_grad_enabled() and anchor.requires_grad)
