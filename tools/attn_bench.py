"""Greedy attention decode throughput on the HIP path (crnn_hip/attn.py): B=256 encoder rows of
T=32 x 512 (the cfg2 encoder output), 26 steps (batch_max_length 25), C=194; random weights.
    python tools/attn_bench.py [B]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip.attn import AttnDecoderHIP  # noqa: E402
from model.model import _AttentionParams  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    H, T, V, steps = 512, 32, 194, 26
    torch.manual_seed(0)
    p = _AttentionParams(H, H, V).state_dict()
    dec = AttnDecoderHIP(p, V, sos_id=1, blank_id=3, device="cuda")
    enc = torch.randn(B, T, H, device="cuda")
    for _ in range(3):
        dec.run(enc, steps)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        dec.run(enc, steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"attn greedy decode B={B} T={T} H={H} steps={steps}: {dt * 1e3:.3f} ms/batch = {B / dt:.0f} lines/s "
          f"({dt / steps * 1e6:.1f} us/step, 6 launches/step)")


if __name__ == "__main__":
    main()
