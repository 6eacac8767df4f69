"""Reference point for the conv GEMM kernels: hipBLASLt (torch.matmul, bf16) on plain GEMMs of the
same M x N x K as the SE-ResNet31 convs (no im2col gather), TFLOP/s.  python tools/blas_ref.py"""
import torch

SHAPES = [  # (name, M, N, K): fwd = (B*Ho*Wo, Co, 9*Ci)
    ("stem1 fwd", 256 * 32 * 256, 128, 576),
    ("b0.c2 fwd", 256 * 8 * 64, 256, 2304),
    ("b3.c2 fwd", 256 * 4 * 32, 512, 4608),
    ("b0.c2 wgrad", 256, 2304, 256 * 8 * 64),
    ("b3.c2 wgrad", 512, 4608, 256 * 4 * 32),
    ("lstm xg", 256 * 32, 4096, 512),
    ("lstm dx", 256 * 32, 512, 4096),
]


def main():
    dev = torch.device("cuda")
    for name, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.matmul(a, b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.matmul(a, b)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name:14s} M={M:8d} N={N:5d} K={K:7d}: {us:8.1f} us  {2 * M * N * K / us / 1e6:7.0f} TFLOP/s")


if __name__ == "__main__":
    main()
