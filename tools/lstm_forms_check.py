"""Persistent BiLSTM forward forms (CRNN_OPT_LSTM_HANDOFF: 1 = K-split waves, 2 = unit-complete waves,
3 = unit-complete, 8 waves) on the same inputs: max |difference| of h / saved gates / cell against form 1
and the fp32 recurrence on the host, error word and counters.   python tools/lstm_forms_check.py [B T H]"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def host_ref(xg, whh, B, T, H):
    """fp32 recurrence over the packed (gate-interleaved) layout: gates[4u+q]"""
    xg, whh = xg.float().cpu(), whh.float().cpu()
    hs = torch.zeros(B, T, 2 * H)
    for d in range(2):
        h = torch.zeros(B, H)
        c = torch.zeros(B, H)
        for s in range(T):
            t = s if d == 0 else T - 1 - s
            gt = xg[:, t, d] + h @ whh[d].t()
            gt = gt.view(B, H, 4)
            i, f, g, o = gt[..., 0].sigmoid(), gt[..., 1].sigmoid(), gt[..., 2].tanh(), gt[..., 3].sigmoid()
            c = f * c + i * g
            h = (o * c.tanh()).bfloat16().float()
            hs[:, t, d * H:(d + 1) * H] = h
    return hs


def main():
    B, T, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 32, 512)
    dev = torch.device("cuda")
    st = L.stream_ptr()
    g = torch.Generator().manual_seed(0)
    xg = (torch.randn(B, T, 2, 4 * H, generator=g) * 0.7).to(dev, torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    S, U = ctypes.c_int(0), ctypes.c_int(0)
    L.lib().crnn_lstm_seq_config(B, H, 0, ctypes.byref(S), ctypes.byref(U))
    outs = {}
    for form in [int(f) for f in os.environ.get("FORMS", "1,2,3").split(",")]:
        L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, form)
        hseq = torch.full((B, T, 2 * H), 3.0, dtype=torch.bfloat16, device=dev)
        gsv = torch.full((2, T, B, 4 * H), 3.0, dtype=torch.bfloat16, device=dev)
        csv = torch.full((2, T, B, H), 3.0, device=dev)
        ws = torch.full((L.lib().crnn_lstm_seq_workspace(B) // 4,), 7, dtype=torch.int32, device=dev)
        L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(), gsv.data_ptr(), csv.data_ptr(),
               ws.data_ptr(), B, T, H, st)
        torch.cuda.synchronize()
        e = int(ws[2 * (B // 16 + 1)].item())
        cnt = int(ws[: 2 * (B // S.value)].min().item())
        outs[form] = (hseq.float().cpu(), gsv.float().cpu(), csv.cpu())
        print(f"form {form}: err word {e}, counters min {cnt} (want {H // U.value * T}), finite "
              f"{all(torch.isfinite(x).all().item() for x in outs[form])}", flush=True)
    L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, 3)   # the default
    ref = host_ref(xg, whh, B, T, H)
    for form, (h, gs, cs) in outs.items():
        a = outs[min(outs)]
        print(f"form {form}: vs first form max|dh| {(h - a[0]).abs().max():.3e} max|dgates| {(gs - a[1]).abs().max():.3e} "
              f"max|dc| {(cs - a[2]).abs().max():.3e}; vs fp32 host max|dh| {(h - ref).abs().max():.3e} "
              f"mean|dh| {(h - ref).abs().mean():.3e}", flush=True)


if __name__ == "__main__":
    main()
