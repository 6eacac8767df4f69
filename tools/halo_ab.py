"""A/B of the stem halo convs (B=256, 32x256: 8 -> 64 and 64 -> 128 forward, 64 -> 128 input gradient) under a
tuning switch, alternated in one process.   python tools/halo_ab.py [KEY]   (KEY: a CRNN_OPT_* index, default
CRNN_OPT_HALO_ROW16)"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402


def main():
    key = int(sys.argv[1]) if len(sys.argv) > 1 else L.OPT_HALO_ROW16
    dev = torch.device("cuda")
    B, H, W = 256, 32, 256
    st = L.stream_ptr()
    g = torch.Generator().manual_seed(3)
    cases = {}
    for Ci, Co in ((8, 64), (64, 128)):
        x = torch.randn(B, H, W, Ci, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(Co, Ci, 3, 3, generator=g) / 24).to(dev)
        dy = torch.randn(B, H, W, Co, generator=g).to(dev, torch.bfloat16)
        d = L.ConvDesc(B, H, W, Ci, H, W, Co, 3, 3, 1, 1, 1, 1, Ci)
        wd = torch.empty(Co, 3, 3, Ci, dtype=torch.bfloat16, device=dev)
        L.call("crnn_pack_conv_weight", L.BF16, w.data_ptr(), wd.data_ptr(), Co, Ci, 3, 3, Ci, st)
        rows = L.lib().crnn_conv_stat_rows(L.BF16, d)
        y = torch.empty(B, H, W, Co, dtype=torch.bfloat16, device=dev)
        ps, pq = torch.empty(rows, Co, device=dev), torch.empty(rows, Co, device=dev)
        keep = (x, w, dy, d, wd, y, ps, pq)
        cases[f"fwd {Ci}->{Co}"] = (keep, lambda k=keep: L.call("crnn_conv_fwd", L.BF16, k[3], k[0].data_ptr(), k[4].data_ptr(),
                                                                  k[5].data_ptr(), k[6].data_ptr(), k[7].data_ptr(), st))
        wsb = torch.empty(2 * 512 * Co * Ci * 9 + 16, device=dev)      # room for one slab per band
        dw = torch.empty(Co, Ci, 3, 3, device=dev)
        keep3 = keep + (wsb, dw)
        cases[f"wgrad {Ci}->{Co}"] = (keep3, lambda k=keep3: L.call("crnn_conv_wgrad", L.BF16, k[3], k[2].data_ptr(),
                                                                      k[0].data_ptr(), k[9].data_ptr(), k[8].data_ptr(),
                                                                      k[8].numel() * 4, 0.0, st))
        if Ci == 64:
            dx = torch.empty(B, H, W, Ci, dtype=torch.bfloat16, device=dev)
            keep2 = keep + (dx,)
            cases[f"dgrad {Co}->{Ci}"] = (keep2, lambda k=keep2: L.call("crnn_conv_dgrad", L.BF16, k[3], k[2].data_ptr(),
                                                                       k[4].data_ptr(), k[8].data_ptr(), None, None, 0, st))
    for name, (_, fn) in cases.items():
        res = {0: [], 1: []}
        for rnd in range(4):
            for opt in (0, 1):
                L.call("crnn_set_option", key, opt)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[opt].append(e0.elapsed_time(e1) / 20 * 1e3)
        line = f"{name:14s}"
        for opt, v in res.items():
            med = sorted(v)[len(v) // 2]
            line += f" | opt{key}={opt}: median {med:7.1f} us ({', '.join(f'{t:.1f}' for t in v)})"
        print(line, flush=True)
    L.call("crnn_set_option", key, 0)


if __name__ == "__main__":
    main()
