"""Microbenchmark of the SE MLP kernels (warm back-to-back vs after an L2/MALL-flushing write).
    python tools/sebench.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    st = L.stream_ptr()
    flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)   # 1 GiB
    for B, C in ((256, 512), (256, 256)):
        Cr = C // 16
        pooled = torch.randn(B, C, device=dev)
        w1 = torch.randn(Cr, C, device=dev) * 0.05
        w2 = torch.randn(C, Cr, device=dev) * 0.05
        hid = torch.empty(B, Cr, device=dev)
        s = torch.empty(B, C, device=dev)
        ds = torch.randn(B, C, device=dev)
        dsig, dpool = torch.empty(B, C, device=dev), torch.empty(B, C, device=dev)
        dhid = torch.empty(B, Cr, device=dev)
        dw1, dw2 = torch.empty(Cr, C, device=dev), torch.empty(C, Cr, device=dev)
        fns = {
            "mlp_fwd": lambda: L.call("crnn_se_mlp_fwd", pooled.data_ptr(), w1.data_ptr(), w2.data_ptr(), hid.data_ptr(),
                                      s.data_ptr(), B, C, Cr, st),
            "mlp_bwd+wgrad": lambda: L.call("crnn_se_mlp_bwd", ds.data_ptr(), pooled.data_ptr(), hid.data_ptr(), s.data_ptr(),
                                            w1.data_ptr(), w2.data_ptr(), dsig.data_ptr(), dhid.data_ptr(),
                                            dpool.data_ptr(), dw1.data_ptr(), dw2.data_ptr(), B, C, Cr, 8, 0, st),
        }
        for name, fn in fns.items():
            for _ in range(5):
                fn()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
            for _ in range(200):
                fn()
            e[1].record()
            torch.cuda.synchronize()
            warm = e[0].elapsed_time(e[1]) / 200 * 1e3
            cold = 0.0
            for _ in range(10):
                flush.fill_(1.0)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                torch.cuda.synchronize()
                cold += a.elapsed_time(b) * 1e3 / 10
            print(f"B={B} C={C} {name:14s} warm {warm:7.2f} us   after-flush {cold:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
