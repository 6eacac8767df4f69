"""A/B microbenchmark of the BiLSTM / linear GEMM entry points at the bench shapes (B=256, T=32,
H=512): crnn_set_option(KEY, v) for v in VALS, timed in one process.
    python tools/gemmbench.py [KEY=V0,V1] [--set KEY=V ...]  (--set: fixed options for every variant)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def main():
    key, vals = 2, [0, 1]
    args = sys.argv[1:]
    fixed = []
    while "--set" in args:
        i = args.index("--set")
        k, v = args[i + 1].split("=")
        fixed.append((int(k), int(v)))
        del args[i:i + 2]
    if args:
        k, v = args[0].split("=")
        key, vals = int(k), [int(x) for x in v.split(",")]
    for k, v in fixed:
        L.call("crnn_set_option", k, v)
    dev = torch.device("cuda")
    st = L.stream_ptr()
    B, T, H, In = 256, 32, 512, 512
    M = B * T
    bf = torch.bfloat16
    x = torch.randn(M, In, device=dev).to(bf)
    wih = (torch.randn(8 * H, In, device=dev) * 0.05).to(bf)
    bias = torch.randn(8 * H, device=dev)
    xg = torch.empty(M, 8 * H, device=dev, dtype=bf)
    hseq = torch.randn(M, 2 * H, device=dev).to(bf)
    lin = (torch.randn(H, 2 * H, device=dev) * 0.05).to(bf)
    out = torch.empty(M, H, device=dev, dtype=bf)
    dx = torch.randn(M, H, device=dev).to(bf)
    dh = torch.empty(M, 2 * H, device=dev, dtype=bf)
    dlw = torch.empty(H, 2 * H, device=dev)
    dg = torch.randn(2, T, B, 4 * H, device=dev).to(bf)
    dW = torch.empty(2, 4 * H, H, device=dev)
    dxl = torch.empty(B, T, In, device=dev, dtype=bf)
    dW4 = torch.empty(4, 4 * H, H, device=dev)
    tnneed = L.lib().crnn_gemm_tn_workspace(H, 2 * H, M)
    tnw = torch.empty(tnneed // 4 + 4, device=dev)
    need = L.lib().crnn_lstm_wgrad_workspace(B, T, H, In)
    wgw = torch.empty(need // 4 + 4, device=dev)
    ops = {
        "xg nt 8192x4096x512": lambda: L.call("crnn_gemm_nt", L.BF16, x.data_ptr(), In, wih.data_ptr(), In, xg.data_ptr(),
                                              8 * H, bias.data_ptr(), M, 8 * H, In, 0, 0, st),
        "lin fwd nt 8192x512x1024": lambda: L.call("crnn_gemm_nt", L.BF16, hseq.data_ptr(), 2 * H, lin.data_ptr(), 2 * H,
                                                   out.data_ptr(), H, None, M, H, 2 * H, 0, 0, st),
        "lin bwd nn 8192x1024x512": lambda: L.call("crnn_gemm_nn", L.BF16, dx.data_ptr(), H, lin.data_ptr(), 2 * H,
                                                   dh.data_ptr(), 2 * H, M, 2 * H, H, 0, 0, st),
        "lin wgrad tn 512x1024x8192": lambda: L.call("crnn_gemm_tn", L.BF16, dx.data_ptr(), H, hseq.data_ptr(), 2 * H,
                                                     dlw.data_ptr(), 2 * H, H, 2 * H, M, 0, st),
        "lin wgrad tn slab": lambda: L.call("crnn_gemm_tn_slab", dx.data_ptr(), H, hseq.data_ptr(), 2 * H,
                                            dlw.data_ptr(), 2 * H, H, 2 * H, M, 0, tnw.data_ptr(), tnneed, st),
        "dwhh (2 dirs)": lambda: L.call("crnn_lstm_dwhh", L.BF16, dg.data_ptr(), hseq.data_ptr(), dW[0].data_ptr(),
                                        dW[1].data_ptr(), B, T, H, 0, st),
        "dwih (2 dirs)": lambda: L.call("crnn_lstm_dwih", L.BF16, dg.data_ptr(), x.data_ptr(), dW[0].data_ptr(),
                                        dW[1].data_ptr(), B, T, H, In, 0, st),
        "lstm wgrad batched (4)": lambda: L.call("crnn_lstm_wgrad", dg.data_ptr(), x.data_ptr(), hseq.data_ptr(),
                                                 dW4[0].data_ptr(), dW4[1].data_ptr(), dW4[2].data_ptr(),
                                                 dW4[3].data_ptr(), wgw.data_ptr(), need, B, T, H, In, 0, st),
        "lstm dx": lambda: L.call("crnn_lstm_dx", L.BF16, dg.data_ptr(), wih.data_ptr(), dxl.data_ptr(), B, T, H, In, st),
    }
    # the same products through torch.matmul (hipBLASLt), bf16 in and out: the vendor reference per shape
    dgf = dg.permute(0, 2, 1, 3).reshape(2, M, 4 * H)       # [d][b*T + t][4H] (layout irrelevant for timing)
    xb = x.view(M, In)
    hb = hseq.view(M, 2 * H)
    vendor = {
        "xg nt 8192x4096x512": lambda: torch.addmm(bias.to(bf), xb, wih.t()),
        "lin fwd nt 8192x512x1024": lambda: hb @ lin.t(),
        "lin bwd nn 8192x1024x512": lambda: dx @ lin,
        "lin wgrad tn 512x1024x8192": lambda: dx.t() @ hb,
        "dwhh (2 dirs)": lambda: torch.bmm(dgf.transpose(1, 2), hb[:, :H].unsqueeze(0).expand(2, M, H)),
        "dwih (2 dirs)": lambda: torch.bmm(dgf.transpose(1, 2), xb.unsqueeze(0).expand(2, M, In)),
        "lstm dx": lambda: dgf.transpose(0, 1).reshape(M, 8 * H) @ wih,
    }
    for name, fn in ops.items():
        line = f"{name:28s}"
        if os.environ.get("GEMMBENCH_VENDOR") and name in vendor:
            vf = vendor[name]
            for _ in range(3):
                vf()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                vf()
            e1.record()
            torch.cuda.synchronize()
            line += f" | hipBLASLt: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us"
        for v in vals:
            L.call("crnn_set_option", key, v)
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            line += f" | opt{key}={v}: {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
