"""Forward-sweep timing per CRNN_OPT_LSTM_HANDOFF form, with and without the saved-forward stores (gsv/csv = null
is the inference form), interleaved rounds in one process. (r06 also ran diagnostic forms without the hand-off
poll — compute alone — that are no longer in the library: profiles/r06/r06k_lstm_diag.log, r06m_lstm_diag.log.)
    python tools/lstm_diag.py [B T H] [forms]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def main():
    B, T, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 32, 512)
    forms = [int(f) for f in (sys.argv[4] if len(sys.argv) > 4 else "1,3").split(",")]
    dev = torch.device("cuda")
    st = L.stream_ptr()
    g = torch.Generator().manual_seed(0)
    xg = (torch.randn(B, T, 2, 4 * H, generator=g) * 0.5).to(dev, torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    hseq = torch.zeros(B, T, 2 * H, device=dev, dtype=torch.bfloat16)
    gsv = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
    csv = torch.zeros(2, T, B, H, device=dev)
    ws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4 + 4, dtype=torch.int32, device=dev)
    res = {}
    for rnd in range(3):
        for form in forms:
            L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, form)
            for save in (True, False):
                fn = lambda: L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(),  # noqa
                                    gsv.data_ptr() if save else None, csv.data_ptr() if save else None, ws.data_ptr(),
                                    B, T, H, st)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((form, save), []).append(e0.elapsed_time(e1) / 20 * 1e3 / T)
    L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, 3)   # the default
    for (form, save), xs in sorted(res.items()):
        print(f"B={B} T={T} H={H} form {form} {'saved stores' if save else 'no saved stores'}: us/step median "
              f"{sorted(xs)[len(xs) // 2]:.3f} ({', '.join(f'{x:.3f}' for x in xs)})")


if __name__ == "__main__":
    main()
