"""Microbenchmark of the BN finalize / backward-finalize launches at the bench's shapes, next to a
trivial launch (the per-launch floor). python tools/bnbench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = "cuda"
    L.lib()
    st = L.stream_ptr()
    fws = torch.zeros(L.lib().crnn_bn_finalize_workspace(512) // 4, device=dev)
    x = torch.randn(512, device=dev)
    y = torch.empty(512, dtype=torch.bfloat16, device=dev)
    print(f"trivial launch        {timeit(lambda: L.call('crnn_cast_f32', L.BF16, x.data_ptr(), y.data_ptr(), 512, st)):7.2f} us")
    for C, rows, rpp in [(512, 256, 128), (512, 512, 128), (256, 1024, 128), (256, 2048, 128), (128, 2048, 128),
                         (64, 16384, 128), (128, 16384, 128)]:
        ps, pq = torch.rand(rows, C, device=dev), torch.rand(rows, C, device=dev)
        gm, bt = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        o = [torch.empty(C, device=dev) for _ in range(4)]
        count = rows * rpp
        f = lambda: L.call("crnn_bn_finalize", ps.data_ptr(), pq.data_ptr(), rows, rpp, C, count, gm.data_ptr(),
                           bt.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, 1, o[0].data_ptr(), o[1].data_ptr(),
                           o[2].data_ptr(), o[3].data_ptr(), fws.data_ptr(), st)
        g = lambda: L.call("crnn_bn_bwd_finalize", ps.data_ptr(), pq.data_ptr(), rows, C, count, o[0].data_ptr(),
                           o[1].data_ptr(), o[2].data_ptr(), o[3].data_ptr(), 0, fws.data_ptr(), st)
        print(f"C={C:3d} rows={rows:5d}  fwd finalize {timeit(f):7.2f} us   bwd finalize {timeit(g):7.2f} us")


if __name__ == "__main__":
    main()
