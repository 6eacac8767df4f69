"""Which kernels of this library give run-to-run different results while ANOTHER process runs this
library on the same GPU? This process repeats two conv forwards through the C ABI and checks each
output (and the BN partial sums of the epilogue) bit for bit against its first run:
  gemm: 3x3 256->256 at B=64, 16x64 (the 256-row LDS-DMA GEMM, gemm256.hpp)
  halo: the stem's 64->128 3x3 at B=16, 16x256 (conv_halo.hip: LDS tiles, no LDS-DMA)
    python tools/conv_only_check.py [seconds]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
import torch  # noqa: E402


def setup(L, B, Ci, H, W, Co, seed):
    g = torch.Generator().manual_seed(seed)
    dev = "cuda"
    d = L.ConvDesc(B, H, W, Ci, H, W, Co, 3, 3, 1, 1, 1, 1, Ci)
    x = torch.randn(B, H, W, Ci, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Co, 3, 3, Ci, generator=g) / 24).to(dev, torch.bfloat16)
    y = torch.empty(B, H, W, Co, dtype=torch.bfloat16, device=dev)
    rows = L.lib().crnn_conv_stat_rows(L.BF16, d)
    ps = torch.empty(rows, Co, device=dev)
    pq = torch.empty(rows, Co, device=dev)
    st = L.stream_ptr()

    def run():
        L.call("crnn_conv_fwd", L.BF16, d, x.data_ptr(), w.data_ptr(), y.data_ptr(), ps.data_ptr(), pq.data_ptr(), st)
        return y, ps, pq
    return run


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    from crnn_hip import _lib as L
    L.lib()
    cases = {"gemm": setup(L, 64, 256, 16, 64, 256, 1), "halo": setup(L, 16, 64, 16, 256, 128, 2)}
    ref = {k: [t.clone() for t in f()] for k, f in cases.items()}
    torch.cuda.synchronize()
    t0, n = time.time(), 0
    bad = {k: 0 for k in cases}
    while time.time() - t0 < secs:
        n += 1
        for k, f in cases.items():
            for _ in range(4):
                out = f()
                nd = [i for i, (t, r) in enumerate(zip(out, ref[k])) if not torch.equal(t, r)]
                if nd:
                    bad[k] += 1
                    y, r = out[0].float(), ref[k][0].float()
                    print(f"round {n} {k}: outputs {nd} differ (y: {int((y != r).sum())} elements, "
                          f"max |diff| {float((y - r).abs().max()):.3e})", flush=True)
        torch.cuda.synchronize()
        if n % 200 == 0:
            print(f"round {n}: {bad}", flush=True)
    print(f"{n} rounds x 4 launches each: differing launches {bad}", flush=True)


if __name__ == "__main__":
    main()
