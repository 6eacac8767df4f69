"""A/B of the stem BN -> ReLU -> 2x2 max-pool (B=256, 32x256x128 bf16 -> 16x128x128): CRNN_OPT_POOL2 0 / 1,
alternated in one process, with the HBM rate of its algorithmic bytes.   python tools/pool_ab.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, H, W, C = 256, 32, 256, 128
    z = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.2
    y = torch.empty(B, H // 2, W // 2, C, dtype=torch.bfloat16, device=dev)
    st = L.stream_ptr()
    nbytes = z.numel() * 2 + y.numel() * 2
    res = {0: [], 1: []}
    for rnd in range(4):
        for opt in (0, 1):
            L.call("crnn_set_option", L.OPT_POOL2, opt)
            for _ in range(3):
                L.call("crnn_bn_relu_maxpool", L.BF16, z.data_ptr(), sc.data_ptr(), sh.data_ptr(), y.data_ptr(), B, H, W,
                       C, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                L.call("crnn_bn_relu_maxpool", L.BF16, z.data_ptr(), sc.data_ptr(), sh.data_ptr(), y.data_ptr(), B, H, W,
                       C, st)
            e1.record()
            torch.cuda.synchronize()
            res[opt].append(e0.elapsed_time(e1) / 20 * 1e3)
    for opt, v in res.items():
        med = sorted(v)[len(v) // 2]
        print(f"bn_relu_maxpool CRNN_OPT_POOL2={opt}: median {med:.1f} us = {nbytes / med / 1e6:.2f} TB/s "
              f"({', '.join(f'{t:.1f}' for t in v)})", flush=True)
    L.call("crnn_set_option", L.OPT_POOL2, 1)


if __name__ == "__main__":
    main()
