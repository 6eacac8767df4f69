"""CTC loss and greedy decoding on the HIP path.

ctc_loss: torch.nn.functional.ctc_loss(log_softmax(logits), blank=0, reduction='mean',
          zero_infinity) semantics (the reference has no CTC loss);
ctc_greedy_decoder / decode: training/utils.py:122-162 API (alphabet[p-1] indexing,
          blank 0), but with an explicit layout argument instead of the reference's
          `shape[0] < shape[1]` guess. The argmax + collapse runs on device.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from . import _lib as L
from ._lib import call, ptr


class _CTCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, lengths, zero_infinity):
        B, T, C = logits.shape
        lg = logits.contiguous().float()
        tg = targets.to(device=lg.device, dtype=torch.int32).contiguous()
        ln = lengths.to(device=lg.device, dtype=torch.int32).contiguous()
        if tg.dim() == 1:  # concatenated targets -> padded [B, Lmax]
            lens = ln.tolist()
            lmax = max(1, max(lens))
            pad = torch.zeros(B, lmax, dtype=torch.int32, device=lg.device)
            off = 0
            for b, n in enumerate(lens):
                pad[b, :n] = tg[off:off + n]
                off += n
            tg = pad
        loss_b = torch.empty(B, dtype=torch.float32, device=lg.device)
        grad = torch.empty_like(lg) if logits.requires_grad else None
        s = L.stream_ptr()
        call("crnn_ctc_loss", ptr(lg), C, B, T, C, ptr(tg), tg.shape[1], ptr(ln), ptr(loss_b), ptr(grad),
             1 if zero_infinity else 0, s)
        out = torch.empty(1, dtype=torch.float32, device=lg.device)
        call("crnn_ctc_reduce_mean", ptr(loss_b), ptr(ln), B, ptr(out), s)
        ctx.save_for_backward(grad if grad is not None else torch.empty(0))
        return out[0]

    @staticmethod
    def backward(ctx, go):
        (g,) = ctx.saved_tensors
        return g * go, None, None, None


def ctc_loss(logits: torch.Tensor, targets: torch.Tensor, target_lengths: torch.Tensor,
             zero_infinity: bool = True) -> torch.Tensor:
    """mean-reduced CTC loss of logits [B, T, C] (batch-first, pre-softmax), blank = 0,
    input length T for every sample; differentiable wrt logits."""
    L.require_device(logits)
    return _CTCFn.apply(logits, targets, target_lengths, zero_infinity)


def ctc_greedy_decode(logits: torch.Tensor, layout: str = "BTC") -> List[List[int]]:
    """argmax over C, collapse repeats, drop blank 0 -> label id lists (device kernel)."""
    L.require_device(logits)
    if layout == "TBC":
        logits = logits.permute(1, 0, 2)
    elif layout != "BTC":
        raise ValueError("layout must be 'BTC' or 'TBC'")
    lg = logits.contiguous().float()
    B, T, C = lg.shape
    ids = torch.empty(B, T, dtype=torch.int32, device=lg.device)
    lens = torch.empty(B, dtype=torch.int32, device=lg.device)
    call("crnn_ctc_greedy", ptr(lg), C, B, T, C, ptr(ids), ptr(lens), L.stream_ptr())
    ids_h, lens_h = ids.cpu().tolist(), lens.cpu().tolist()
    return [row[:n] for row, n in zip(ids_h, lens_h)]


def ctc_greedy_decoder(logits: torch.Tensor, alphabet: Sequence[str], blank: int = 0,
                       layout: str = "BTC") -> Tuple[List[str], List[List[int]]]:
    """training/utils.py:122-150 return contract: (texts, seqs), alphabet[p-1]."""
    if blank != 0:
        raise NotImplementedError("the HIP decoder uses blank = 0 (SURVEY D5)")
    seqs = ctc_greedy_decode(logits, layout)
    texts = ["".join(alphabet[p - 1] for p in s) for s in seqs]
    return texts, seqs


def decode(ctc_out, alphabet: Sequence[str], method: str = "greedy", layout: str = "BTC"):
    """training/utils.py:153-162: log_softmax is monotone per row, so argmax on logits is identical."""
    if isinstance(ctc_out, tuple):
        ctc_out = ctc_out[0]
    if method != "greedy":
        raise ValueError(f"Unsupported decode method: {method}")
    return ctc_greedy_decoder(ctc_out, alphabet, layout=layout)
