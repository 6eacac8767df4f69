"""The 256-row kernel on plain bf16 GEMMs (square and conv-like tall-skinny) (crnn_gemm_nt, RowMajorK loaders both sides) next
to torch.matmul (hipBLASLt), uniform random [-1, 1) operands: the template's own rate, without the
conv loaders and epilogues.   python tools/gemm_square.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


def main():
    st = L.stream_ptr()
    if len(sys.argv) > 1:   # KEY=V: a crnn_set_option for this run
        k, v = sys.argv[1].split("=")
        L.call("crnn_set_option", int(k), int(v))
    shapes = [(4096, 4096, 4096), (8192, 8192, 8192),
              # conv-like tall-skinny: M = batch x pixels, N = Co, K = 9 Ci (b3.c2, b0.c2, stem1 fwd)
              (32768, 512, 4608), (131072, 256, 2304), (131072, 128, 576)]
    for m, n, k in shapes:
        A = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        f = 2.0 * m * n * k
        t1 = timeit(lambda: L.call("crnn_gemm_nt", L.BF16, A.data_ptr(), k, B.data_ptr(), k, C.data_ptr(), n, None,
                                   m, n, k, 0, 0, st))
        t2 = timeit(lambda: torch.matmul(A, B.t()))
        rows = torch.randperm(m, device="cuda")[:256]   # rows from every tile position
        ref = torch.matmul(A.float()[rows], B.float().t())
        err = float((C[rows].float() - ref).abs().max())
        print(f"{m}x{n}x{k}: crnn 256-row kernel {f / t1 / 1e12:7.1f} TF   hipBLASLt {f / t2 / 1e12:7.1f} TF   "
              f"(max err {err:.3f})")

if __name__ == "__main__":
    main()
