"""Decoder-shape GEMM timings (attention decoder per-step products, crnn_hip/attn.py): crnn_gemm_nt / nn with
CRNN_F32_BF16MMA (linear.hip run_mix's plan), bf16 operands on the library's bf16 path, and torch bf16 / fp32 matmul
(hipBLASLt) for reference. (r06w measured the alternative tile / stage plans through a temporary switch, since
removed: profiles/r06/r06w_gemm_mix_plans.log.)
    python tools/gemm_mix_bench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))

SHAPES = [("nn", 256, 1280, 1024), ("nt", 256, 1024, 1280), ("nn", 256, 256, 256), ("nt", 256, 256, 256)]


def child():
    import torch
    from crnn_hip import _lib as L
    dev = torch.device("cuda")
    st = L.stream_ptr()
    for kind, M, N, K in SHAPES:
        A = torch.randn(M, K, device=dev)
        Bm = torch.randn(N, K, device=dev) if kind == "nt" else torch.randn(K, N, device=dev)
        C = torch.empty(M, N, device=dev)
        Ab, Bb = A.bfloat16(), Bm.bfloat16()

        def lib(dt, a, b):
            if kind == "nt":
                return lambda: L.call("crnn_gemm_nt", dt, a.data_ptr(), K, b.data_ptr(), K, C.data_ptr(), N, None, M, N,
                                      K, 1, 0, st)
            return lambda: L.call("crnn_gemm_nn", dt, a.data_ptr(), K, b.data_ptr(), N, C.data_ptr(), N, M, N, K, 1, 0,
                                  st)
        fns = {"lib mixed": lib(L.F32_BF16MMA, A, Bm), "lib fp32": lib(L.F32, A, Bm), "lib bf16": lib(L.BF16, Ab, Bb),
               "torch bf16": (lambda: Ab @ Bb.t()) if kind == "nt" else (lambda: Ab @ Bb),
               "torch fp32": (lambda: A @ Bm.t()) if kind == "nt" else (lambda: A @ Bm)}
        for name, fn in fns.items():
            for _ in range(5):
                fn()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 20 * 1e3)
            us = sorted(ts)[2]
            print(f"{kind} {M}x{N}x{K} {name:14s} {us:7.2f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    child()
