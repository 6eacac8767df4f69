"""Attention decoder on the HIP path (fp32): the reference's shipping head, model/model.py:23-148
(AttentionCell, Attention._greedy_decode, teacher-forced Attention.forward), SURVEY §8(f) next-1.

The host loop runs one decoder step as 3 GEMMs (crnn_gemm_nt) + 3 small kernels
(csrc/attn.hip): proj_h, attention context, gates (one GEMM over [context | h]), the LSTM cell
with the one-hot input folded in as a weight column, logits, blank mask + argmax. The encoder
projection proj_H = enc W_i2h^T is computed once per decode. Forward only (inference and
teacher-forced logits); the decoder's backward is not on the HIP path yet.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib as L
from ._lib import call, ptr


class AttnDecoderHIP:
    """params: the reference Attention state_dict (attention_cell.*, generator.*), any device
    tensors; copied to fp32 device buffers (call refresh() after the weights change)."""

    def __init__(self, params: Dict[str, torch.Tensor], num_classes: int, sos_id: int,
                 blank_id: Optional[int], device):
        self.device = torch.device(device)
        self.V = num_classes
        self.Vpad = (num_classes + 7) // 8 * 8
        self.sos_id = sos_id
        self.blank = -1 if blank_id is None else int(blank_id)
        self.refresh(params)

    def refresh(self, params: Dict[str, torch.Tensor]):
        f = lambda k: params[k].detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        pre = "attention_cell."
        self.w_i2h = f(pre + "i2h.weight")            # [H, C]
        self.H, self.C = self.w_i2h.shape
        self.w_h2h = f(pre + "h2h.weight")            # [H, H]
        self.b_h2h = f(pre + "h2h.bias")
        self.score = f(pre + "score.weight").reshape(-1)
        self.w_ih = f(pre + "rnn.weight_ih")          # [4H, C + V]
        self.b_ih = f(pre + "rnn.bias_ih")
        self.b_hh = f(pre + "rnn.bias_hh")
        w_hh = f(pre + "rnn.weight_hh")               # [4H, H]
        self.w_cat = torch.cat([self.w_ih[:, : self.C], w_hh], 1).contiguous()  # [4H, C + H]
        gw, gb = f("generator.weight"), f("generator.bias")
        self.w_gen = torch.zeros(self.Vpad, self.H, device=self.device)
        self.w_gen[: self.V] = gw
        self.b_gen = torch.zeros(self.Vpad, device=self.device)
        self.b_gen[: self.V] = gb

    def _gemm(self, a, lda, w, ldw, out, ldo, bias, M, N, K):
        call("crnn_gemm_nt", L.F32, ptr(a), lda, ptr(w), ldw, ptr(out), ldo, ptr(bias), M, N, K, 1, 0,
             L.stream_ptr())

    def run(self, enc: torch.Tensor, steps: int, text: Optional[torch.Tensor] = None) -> torch.Tensor:
        """enc [B, T, C] -> logits [B, steps, V] (fp32): greedy decode (text None, model/model.py:91-112)
        or teacher forcing with text[:, t] as the input of step t (:114-148)."""
        enc = enc.to(self.device, torch.float32).contiguous()
        B, T, C = enc.shape
        H, V, Vp, dev = self.H, self.V, self.Vpad, self.device
        if C != self.C:
            raise ValueError(f"encoder width {C} != decoder input size {self.C}")
        s = L.stream_ptr()
        projH = torch.empty(B * T, H, device=dev)
        self._gemm(enc, C, self.w_i2h, C, projH, H, None, B * T, H, C)
        h = torch.zeros(B, H, device=dev)
        c = torch.zeros(B, H, device=dev)
        hx = torch.zeros(B, C + H, device=dev)           # [context | h] rows of the gates GEMM
        projh = torch.empty(B, H, device=dev)
        gates = torch.empty(B, 4 * H, device=dev)
        if text is None:
            ch = torch.full((B,), self.sos_id, dtype=torch.int32, device=dev)
            logits_t = torch.empty(B, Vp, device=dev)
            out = torch.empty(B, steps, V, device=dev)
            for t in range(steps):
                self._step(enc, projH, h, c, hx, projh, gates, ch, 1, None, 0, B, T)
                self._gemm(h, H, self.w_gen, H, logits_t, Vp, self.b_gen, B, Vp, H)
                call("crnn_attn_out", ptr(logits_t), Vp, B, V, self.blank, ptr(out[:, t]), steps * V, ptr(ch), s)
            return out
        txt = text.to(dev, torch.int32).contiguous()
        if txt.shape[1] < steps:
            raise ValueError("text needs batch_max_length + 1 columns")
        hs = torch.empty(B, steps, H, device=dev)
        for t in range(steps):
            self._step(enc, projH, h, c, hx, projh, gates, txt[:, t:], txt.shape[1], hs[:, t], steps * H, B, T)
        lg = torch.empty(B * steps, Vp, device=dev)
        self._gemm(hs, H, self.w_gen, H, lg, Vp, self.b_gen, B * steps, Vp, H)
        out = torch.empty(B, steps, V, device=dev)
        scratch = torch.empty(B * steps, dtype=torch.int32, device=dev)
        call("crnn_attn_out", ptr(lg), Vp, B * steps, V, self.blank, ptr(out), V, ptr(scratch), s)
        return out

    def _step(self, enc, projH, h, c, hx, projh, gates, ch, ch_stride, hs, ld_hs, B, T):
        H, C, s = self.H, self.C, L.stream_ptr()
        self._gemm(h, H, self.w_h2h, H, projh, H, self.b_h2h, B, H, H)
        call("crnn_attn_context", ptr(projH), ptr(projh), ptr(self.score), ptr(enc), ptr(hx), C + H, None,
             B, T, H, C, s)
        self._gemm(hx, C + H, self.w_cat, C + H, gates, 4 * H, None, B, 4 * H, C + H)
        call("crnn_attn_cell", ptr(gates), ptr(self.b_ih), ptr(self.b_hh), ptr(self.w_ih), C + self.V, ptr(ch),
             ch_stride, ptr(h), ptr(c), ptr(hx), C + H, ptr(hs), ld_hs, B, H, C, s)
