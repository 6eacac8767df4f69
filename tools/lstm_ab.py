"""In-process A/B of the persistent BiLSTM sweeps under crnn_set_option variants (interleaved rounds).
    python tools/lstm_ab.py KEY=V0,V1[,...] [B T H]
    LSTM_AB_COLD=1: each timed launch alone, after a 1 GiB scratch write (weights, x-gates and workspace out of
    L2 / MALL, as inside the train step) — the per-launch time then includes the cold prologue."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
import torch  # noqa: E402

from crnn_hip import _lib as L  # noqa: E402


def main():
    ks, vs = sys.argv[1].split("=")
    key, vals = int(ks), [int(v) for v in vs.split(",")]
    B, T, H = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (256, 32, 512)
    dev = torch.device("cuda")
    st = L.stream_ptr()
    g = torch.Generator(device="cpu").manual_seed(0)
    xg = (torch.randn(B, T, 2, 4 * H, generator=g) * 0.5).to(dev, torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    whh_t = whh.transpose(1, 2).contiguous()
    hseq = torch.zeros(B, T, 2 * H, device=dev, dtype=torch.bfloat16)
    gsv = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
    csv = torch.zeros(2, T, B, H, device=dev)
    dg = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
    ws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4 + 4, dtype=torch.int32, device=dev)
    fns = {
        "fwd": lambda: L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(), gsv.data_ptr(),
                              csv.data_ptr(), ws.data_ptr(), B, T, H, st),
        "bwd": lambda: L.call("crnn_lstm_seq_bwd", hseq.data_ptr(), whh_t.data_ptr(), gsv.data_ptr(), csv.data_ptr(),
                              dg.data_ptr(), ws.data_ptr(), B, T, H, st),
    }
    res = {}
    cold = os.environ.get("LSTM_AB_COLD") == "1"
    scratch = torch.empty(1 << 28, device=dev) if cold else None
    for rnd in range(3):
        for v in vals:
            L.call("crnn_set_option", key, v)
            for name, fn in fns.items():
                for _ in range(3):
                    fn()
                if cold:
                    ts = []
                    for _ in range(10):
                        scratch.fill_(float(rnd))
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        fn()
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3 / T)
                    res.setdefault((name, v), []).append(sorted(ts)[len(ts) // 2])
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, v), []).append(e0.elapsed_time(e1) / 20 * 1e3 / T)
    L.call("crnn_set_option", key, vals[0])
    for (name, v), xs in sorted(res.items()):
        print(f"B={B} T={T} H={H} {'cold ' if cold else ''}{name} opt{key}={v}: us/step median {sorted(xs)[len(xs) // 2]:.3f} "
              f"(rounds {', '.join(f'{x:.3f}' for x in xs)})")


if __name__ == "__main__":
    main()
