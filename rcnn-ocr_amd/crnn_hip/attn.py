"""Attention decoder on the HIP path (fp32): the reference's shipping head, model/model.py:23-148
(AttentionCell, Attention._greedy_decode, teacher-forced Attention.forward), SURVEY §8(f) next-1.

The host loop runs one decoder step as 3 GEMMs (crnn_gemm_nt) + 3 small kernels
(csrc/attn.hip): proj_h, attention context, gates (one GEMM over [context | h]), the LSTM cell
with the one-hot input folded in as a weight column, logits, blank mask + argmax. The encoder
projection proj_H = enc W_i2h^T is computed once per decode. Forward only (inference and
teacher-forced logits) and the teacher-forced backward (BPTT through the cell and the attention,
run_train / backward): per step a cell-backward kernel, one GEMM for d[context | h], an attention
backward kernel (per-sample d attention logits, d proj_h) and one GEMM for the h2h path; d enc,
d proj_H and the weight gradients are computed once over all steps afterwards (the forward keeps
the one-hot inputs as extra columns of its saved [context | h] rows, so W_ih and W_hh's gradients
are one GEMM).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib as L
from ._lib import call, ptr


class AttnDecoderHIP:
    """params: the reference Attention state_dict (attention_cell.*, generator.*), any device
    tensors; copied to fp32 device buffers (call refresh() after the weights change).
    train_bf16: the training pass (run_train / backward) runs its GEMMs on bf16 MFMA with fp32 accumulation
    over the fp32 operands (CRNN_F32_BF16MMA, converted while staged) — the reference trains this head under
    fp16 autocast (training/train.py:499-505). Inference (run) keeps the exact-fp32 GEMMs."""

    def __init__(self, params: Dict[str, torch.Tensor], num_classes: int, sos_id: int,
                 blank_id: Optional[int], device, train_bf16: bool = False):
        self.device = torch.device(device)
        self.tdt = L.F32_BF16MMA if train_bf16 else L.F32   # the training pass's GEMM dtype code
        self._saved = None
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
        # gate-interleaved copies for the fused gate GEMM + cell (crnn_attn_gates_cell): row 4u + q = row q*H + u
        H = self.H
        il = torch.arange(4 * H, device=self.device).view(4, H).t().reshape(-1)
        self.w_cat_il = self.w_cat.index_select(0, il).contiguous()
        self.b_ih_il = self.b_ih.index_select(0, il).contiguous()
        self.b_hh_il = self.b_hh.index_select(0, il).contiguous()
        self.wv_il = self.w_ih[:, self.C:].index_select(0, il).t().contiguous()   # [V][4H]
        gw, gb = f("generator.weight"), f("generator.bias")
        self.w_gen = torch.zeros(self.Vpad, self.H, device=self.device)
        self.w_gen[: self.V] = gw
        self.b_gen = torch.zeros(self.Vpad, device=self.device)
        self.b_gen[: self.V] = gb

    def _gemm(self, a, lda, w, ldw, out, ldo, bias, M, N, K, dt=None):
        call("crnn_gemm_nt", L.F32 if dt is None else dt, ptr(a), lda, ptr(w), ldw, ptr(out), ldo, ptr(bias), M, N, K,
             1, 0, L.stream_ptr())

    def _bf16(self, x: torch.Tensor) -> torch.Tensor:
        """bf16 copy of a contiguous fp32 tensor (crnn_cast_f32)"""
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        call("crnn_cast_f32", L.BF16, ptr(x), ptr(out), x.numel(), L.stream_ptr())
        return out

    def _tn(self, A, lda, Bm, ldb, C, ldc, M, N, K, bf=None):
        """C (fp32) = A^T B over K rows. Training with train_bf16: bf16 operands (bf = their bf16 copies) through the
        deterministic split-K slab GEMM (crnn_gemm_tn_slab, fp32 accumulation); else crnn_gemm_tn in fp32."""
        s = L.stream_ptr()
        if bf is None:
            call("crnn_gemm_tn", L.F32, ptr(A), lda, ptr(Bm), ldb, ptr(C), ldc, M, N, K, 0, s)
            return
        need = L.lib().crnn_gemm_tn_workspace(M, N, K)
        ws = torch.empty(need // 4 + 4, device=C.device)
        call("crnn_gemm_tn_slab", bf[0], lda, bf[1], ldb, ptr(C), ldc, M, N, K, 0, ptr(ws), ws.numel() * 4, s)

    def run_train(self, enc: torch.Tensor, steps: int, text: torch.Tensor, drop_p: float = 0.0,
                  seed: int = 0) -> torch.Tensor:
        """teacher-forced forward that saves what backward() needs -> logits [B, steps, V].
        drop_p: the training-mode F.dropout on the attention weights (model/model.py:38; the
        reference's RCNN uses 0.1); step t's mask comes from the counter hash with seed + t."""
        mix = self.tdt == L.F32_BF16MMA
        enc_in = enc
        enc = enc.to(self.device, torch.float32).contiguous()
        B, T, C = enc.shape
        H, V, Vp, dev = self.H, self.V, self.Vpad, self.device
        s = L.stream_ptr()
        txt = text.to(dev, torch.int32).contiguous()
        if txt.shape[1] < steps:
            raise ValueError("text needs batch_max_length + 1 columns")
        projH = torch.empty(B * T, H, device=dev)
        self._gemm(enc, C, self.w_i2h, C, projH, H, None, B * T, H, C, self.tdt)
        encb = projHb = None
        if mix:   # the attention reads enc and proj_H as bf16 every step (crnn_attn_context_bf16)
            encb = (enc_in.to(dev).contiguous() if enc_in.dtype == torch.bfloat16 else self._bf16(enc))
            projHb = self._bf16(projH)
        LX = C + H + Vp                                     # [context_t | h_{t-1} | onehot(text_t)] per step
        Xs = torch.zeros(steps + 1, B, LX, device=dev)
        call("crnn_attn_onehot_rows", ptr(txt), txt.shape[1], steps, B, V, ptr(Xs), LX, C + H, s)
        Gs = torch.empty(steps, B, 4 * H, device=dev)       # activated gates
        Cs = torch.empty(steps, B, H, device=dev)           # cell states
        Ph = torch.empty(steps, B, H, device=dev)           # proj_h per step
        As = torch.empty(steps, B, T, device=dev)           # attention weights per step
        hs = torch.empty(B, steps, H, device=dev)
        h = torch.zeros(B, H, device=dev)
        c = torch.zeros(B, H, device=dev)
        for t in range(steps):
            self._gemm(h, H, self.w_h2h, H, Ph[t], H, self.b_h2h, B, H, H, self.tdt)
            if mix:
                call("crnn_attn_context_bf16", ptr(projHb), ptr(Ph[t]), ptr(self.score), ptr(encb), ptr(Xs[t]), LX,
                     ptr(As[t]), B, T, H, C, drop_p, (seed + t) & (2 ** 64 - 1), s)
            else:
                call("crnn_attn_context", ptr(projH), ptr(Ph[t]), ptr(self.score), ptr(enc), ptr(Xs[t]), LX,
                     ptr(As[t]), B, T, H, C, drop_p, (seed + t) & (2 ** 64 - 1), s)
            # gate GEMM + LSTM cell in one launch (gate-interleaved weights); h_t into the next step's X row
            call("crnn_attn_gates_cell", self.tdt, ptr(Xs[t]), LX, ptr(self.w_cat_il), C + H, ptr(self.b_ih_il),
                 ptr(self.b_hh_il), ptr(self.wv_il), ptr(txt[:, t:]), txt.shape[1], ptr(h), ptr(c), ptr(Xs[t + 1]), LX,
                 ptr(hs[:, t]), steps * H, ptr(Gs[t]), ptr(Cs[t]), B, H, C, s)
        lg = torch.empty(B * steps, Vp, device=dev)
        self._gemm(hs, H, self.w_gen, H, lg, Vp, self.b_gen, B * steps, Vp, H, self.tdt)
        out = torch.empty(B, steps, V, device=dev)
        scratch = torch.empty(B * steps, dtype=torch.int32, device=dev)
        call("crnn_attn_out", ptr(lg), Vp, B * steps, V, self.blank, ptr(out), V, ptr(scratch), s)
        self._saved = dict(enc=enc, encb=encb, projH=projH, projHb=projHb, Xs=Xs, Gs=Gs, Cs=Cs, Ph=Ph, As=As, hs=hs, txt=txt, steps=steps,
                           drop=(drop_p, seed))
        return out

    def backward(self, dlogits: torch.Tensor, grads: Dict[str, torch.Tensor], accumulate: bool) -> torch.Tensor:
        """BPTT of run_train's forward. dlogits [B, steps, V]; grads: fp32 tensors keyed by the
        reference's Attention parameter names, written (or added to, if accumulate). -> d enc [B, T, C]"""
        sv = self._saved
        if sv is None:
            raise RuntimeError("run_train must precede backward")
        enc, projH, Xs, Gs, Cs, Ph, As, hs, txt, steps = (sv[k] for k in
                                                           ("enc", "projH", "Xs", "Gs", "Cs", "Ph", "As", "hs", "txt",
                                                            "steps"))
        drop_p, seed = sv["drop"]
        B, T, C = enc.shape
        H, V, Vp, dev, s = self.H, self.V, self.Vpad, self.device, L.stream_ptr()
        F32 = self.tdt   # GEMMs only (crnn_colsum keeps L.F32)
        dL = torch.zeros(B * steps, Vp, device=dev)
        dL[:, :V] = dlogits.reshape(B * steps, V).to(dev, torch.float32)
        if self.blank >= 0:
            dL[:, self.blank] = 0.0   # the masked column is a constant (model/model.py:87-89)
        dHs = torch.empty(B * steps, H, device=dev)
        call("crnn_gemm_nn", F32, ptr(dL), Vp, ptr(self.w_gen), H, ptr(dHs), H, B * steps, H, Vp, 1, 0, s)
        mix = F32 == L.F32_BF16MMA
        bfp = (lambda *xs: tuple(ptr(x) for x in xs)) if mix else (lambda *xs: None)  # noqa: E731
        keep = []   # bf16 copies live until the stream has used them
        if mix:
            keep += [self._bf16(dL), self._bf16(hs)]
        gw = torch.empty(Vp, H, device=dev)
        self._tn(dL, Vp, hs, H, gw, H, Vp, H, B * steps, bfp(*keep[-2:]) if mix else None)
        gb = torch.empty(Vp, device=dev)
        call("crnn_colsum", L.F32, ptr(dL), Vp, B * steps, Vp, ptr(gb), 0, 1, s)
        dG = torch.empty(steps, B, 4 * H, device=dev)
        dPh = torch.empty(steps, B, H, device=dev)
        De = torch.empty(steps, B, T, device=dev)           # d attention logits per step
        dscore = torch.zeros(B, H, device=dev)
        dX = torch.empty(steps, B, C + H, device=dev)       # d [context | h_{t-1}] per step
        dc = [torch.zeros(B, H, device=dev), torch.empty(B, H, device=dev)]
        dh_rec, ld_rec = None, 0
        for t in reversed(range(steps)):
            call("crnn_attn_cell_bwd", ptr(Gs[t]), ptr(Cs[t]), ptr(Cs[t - 1]) if t > 0 else None, ptr(dh_rec), ld_rec,
                 ptr(dHs.view(B, steps, H)[:, t]), steps * H, ptr(dc[0]), ptr(dG[t]), ptr(dc[1]), B, H, s)
            dc.reverse()
            call("crnn_gemm_nn", F32, ptr(dG[t]), 4 * H, ptr(self.w_cat), C + H, ptr(dX[t]), C + H, B, C + H, 4 * H, 1,
                 0, s)
            if mix:
                call("crnn_attn_bwd_bf16", ptr(dX[t]), C + H, ptr(As[t]), ptr(sv["encb"]), ptr(sv["projHb"]), ptr(Ph[t]),
                     ptr(self.score), ptr(De[t]), ptr(dPh[t]), ptr(dscore), B, T, H, C, drop_p,
                     (seed + t) & (2 ** 64 - 1), s)
            else:
                call("crnn_attn_bwd", ptr(dX[t]), C + H, ptr(As[t]), ptr(enc), ptr(projH), ptr(Ph[t]), ptr(self.score),
                     ptr(De[t]), ptr(dPh[t]), ptr(dscore), B, T, H, C, drop_p, (seed + t) & (2 ** 64 - 1), s)
            # dh_{t-1} = d(h part of [context | h]) + dproj_h W_h2h   (accumulated into dX[t][:, C:])
            call("crnn_gemm_nn", F32, ptr(dPh[t]), H, ptr(self.w_h2h), H, ptr(dX[t][:, C:]), C + H, B, H, H, 1, 1, s)
            dh_rec, ld_rec = dX[t][:, C:], C + H
        # encoder-side gradients of the attention, all steps at once
        denc = torch.empty(B, T, C, device=dev)
        call("crnn_attn_denc", ptr(dX), C + H, ptr(As), steps, B, T, C, drop_p, seed & (2 ** 64 - 1), ptr(denc), s)
        dProjH = torch.empty(B * T, H, device=dev)
        if mix:
            call("crnn_attn_dproj_enc_bf16", ptr(Ph), ptr(De), ptr(sv["projHb"]), ptr(self.score), steps, B, T, H,
                 ptr(dProjH), s)
        else:
            call("crnn_attn_dproj_enc", ptr(Ph), ptr(De), ptr(projH), ptr(self.score), steps, B, T, H, ptr(dProjH), s)
        # weight gradients, batched over steps
        # [dW_ih[:, :C] | dW_hh | dW_ih[:, C:]] in one GEMM over the saved [context | h | onehot] rows
        LX = C + H + Vp
        wfull = torch.empty(4 * H, LX, device=dev)
        if mix:
            keep += [self._bf16(dG), self._bf16(Xs[:steps]), self._bf16(dPh), self._bf16(dProjH)]
            dGb, Xsb, dPhb, dPjb = keep[-4:]
            encb = sv["encb"]
        self._tn(dG, 4 * H, Xs, LX, wfull, LX, 4 * H, LX, steps * B, bfp(dGb, Xsb) if mix else None)
        dwih = torch.cat([wfull[:, :C], wfull[:, C + H:C + H + V]], 1)
        db = torch.empty(4 * H, device=dev)
        call("crnn_colsum", L.F32, ptr(dG), 4 * H, steps * B, 4 * H, ptr(db), 0, 1, s)
        wh2h = torch.empty(H, H, device=dev)
        self._tn(dPh, H, Xs[:, :, C:], LX, wh2h, H, H, H, steps * B,
                 (ptr(dPhb), ptr(Xsb) + 2 * C) if mix else None)
        bh2h = torch.empty(H, device=dev)
        call("crnn_colsum", L.F32, ptr(dPh), H, steps * B, H, ptr(bh2h), 0, 1, s)
        wi2h = torch.empty(H, C, device=dev)
        self._tn(dProjH, H, enc, C, wi2h, C, H, C, B * T, bfp(dPjb, encb) if mix else None)
        call("crnn_gemm_nn", F32, ptr(dProjH), H, ptr(self.w_i2h), C, ptr(denc), C, B * T, C, H, 1, 1, s)
        dsc = torch.empty(H, device=dev)
        call("crnn_colsum", L.F32, ptr(dscore), H, B, H, ptr(dsc), 0, 1, s)
        pre = "attention_cell."
        out = {pre + "i2h.weight": wi2h, pre + "h2h.weight": wh2h, pre + "h2h.bias": bh2h,
               pre + "score.weight": dsc.view(1, H), pre + "rnn.weight_ih": dwih, pre + "rnn.weight_hh": wfull[:, C:C + H],
               pre + "rnn.bias_ih": db, pre + "rnn.bias_hh": db, "generator.weight": gw[:V], "generator.bias": gb[:V]}
        for k, v in out.items():
            g = grads[k]
            if accumulate:
                g.add_(v.reshape(g.shape))
            else:
                g.copy_(v.reshape(g.shape))
        self._saved = None
        return denc

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
        # [context | h] rows of the gate GEMM, two buffers: step t reads hxs[t % 2] while its fused cell writes h_t
        # into hxs[(t + 1) % 2]
        hxs = torch.zeros(2, B, C + H, device=dev)
        projh = torch.empty(B, H, device=dev)
        if text is None:
            ch = torch.full((B,), self.sos_id, dtype=torch.int32, device=dev)
            logits_t = torch.empty(B, Vp, device=dev)
            out = torch.empty(B, steps, V, device=dev)
            for t in range(steps):
                self._step(enc, projH, h, c, hxs[t % 2], hxs[(t + 1) % 2], projh, ch, 1, None, 0, B, T)
                self._gemm(h, H, self.w_gen, H, logits_t, Vp, self.b_gen, B, Vp, H)
                call("crnn_attn_out", ptr(logits_t), Vp, B, V, self.blank, ptr(out[:, t]), steps * V, ptr(ch), s)
            return out
        txt = text.to(dev, torch.int32).contiguous()
        if txt.shape[1] < steps:
            raise ValueError("text needs batch_max_length + 1 columns")
        hs = torch.empty(B, steps, H, device=dev)
        for t in range(steps):
            self._step(enc, projH, h, c, hxs[t % 2], hxs[(t + 1) % 2], projh, txt[:, t:], txt.shape[1], hs[:, t],
                       steps * H, B, T)
        lg = torch.empty(B * steps, Vp, device=dev)
        self._gemm(hs, H, self.w_gen, H, lg, Vp, self.b_gen, B * steps, Vp, H)
        out = torch.empty(B, steps, V, device=dev)
        scratch = torch.empty(B * steps, dtype=torch.int32, device=dev)
        call("crnn_attn_out", ptr(lg), Vp, B * steps, V, self.blank, ptr(out), V, ptr(scratch), s)
        return out

    def _step(self, enc, projH, h, c, hx, hx_next, projh, ch, ch_stride, hs, ld_hs, B, T):
        H, C, s = self.H, self.C, L.stream_ptr()
        self._gemm(h, H, self.w_h2h, H, projh, H, self.b_h2h, B, H, H)
        call("crnn_attn_context", ptr(projH), ptr(projh), ptr(self.score), ptr(enc), ptr(hx), C + H, None,
             B, T, H, C, 0.0, 0, s)
        call("crnn_attn_gates_cell", L.F32, ptr(hx), C + H, ptr(self.w_cat_il), C + H, ptr(self.b_ih_il),
             ptr(self.b_hh_il), ptr(self.wv_il), ptr(ch), ch_stride, ptr(h), ptr(c), ptr(hx_next), C + H, ptr(hs),
             ld_hs, None, None, B, H, C, s)


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, ignore_index):
        L.require_device(logits)
        V = logits.shape[-1]
        x = logits.detach().reshape(-1, V)
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError("cross_entropy: logits must be contiguous fp32")
        M = x.shape[0]
        tg = targets.reshape(-1).to(x.device, torch.int32).contiguous()
        if tg.numel() != M:
            raise ValueError("cross_entropy: one target per logits row")
        loss = torch.empty((), device=x.device)
        d = torch.empty_like(x)
        ws = torch.empty(M + 1, device=x.device)
        call("crnn_attn_xent", ptr(x), V, ptr(tg), M, V, int(ignore_index), ptr(loss), ptr(d), V, ptr(ws),
             L.stream_ptr())
        ctx.save_for_backward(d)
        ctx.shape = logits.shape
        return loss

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d.mul_(g).view(ctx.shape), None, None


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor, ignore_index: int = 0) -> torch.Tensor:
    """nn.CrossEntropyLoss(ignore_index=PAD)(logits.reshape(-1, V), targets.reshape(-1)) — the
    attention head's training loss (training/train.py:289,503) — on the HIP path (one fused
    log-softmax / NLL / gradient kernel, csrc/attn.hip)."""
    return _XentFn.apply(logits, targets, ignore_index)
