"""Where a 256-row conv GEMM launch spends its time, per workgroup (diagnostic library only):
    SRCS=conv.hip tools/build_variant.sh stamps -DCRNN_GEMM_STAMPS=1
    CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_stamps.so python tools/gemm_stamps.py
Each workgroup stamps s_memrealtime (10 ns) at entry (t0), after the prologue's first barrier (t1),
after the K loop (t2), after issuing the epilogue (t3) and after its stores completed (t4); plus its
XCC id. Prints, per conv geometry and op, the launch span and the median / p90 of each phase, the
number of dispatch rounds (start-time clusters) and the blocks per XCC."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

from crnn_hip import _lib as L  # noqa: E402
from kbench import geometries  # noqa: E402

SLOTS, NBLK = 6, 8192


def read_stamps():
    buf = (ctypes.c_ulonglong * (SLOTS * NBLK))()
    rc = L.lib().crnn_diag_gemm_stamps(buf, NBLK)
    assert rc == 0, rc
    return np.frombuffer(buf, dtype=np.uint64).reshape(NBLK, SLOTS).copy()


def analyse(name, a, b):
    new = np.nonzero(b[:, 0] != a[:, 0])[0]
    if len(new) == 0:
        return f"{name}: no 256-row GEMM blocks"
    st = b[new].astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st[:, :5] - t0) * 10 / 1000.0   # microseconds
    span = rel[:, 4].max()
    pro, loop, issue, drain = (rel[:, 1] - rel[:, 0], rel[:, 2] - rel[:, 1], rel[:, 3] - rel[:, 2],
                               rel[:, 4] - rel[:, 3])
    starts = np.sort(rel[:, 0])
    rounds = 1 + int(np.sum(np.diff(starts) > 2.0))
    xcc = np.bincount((st[:, 5] >> 32).astype(np.int64) & 15, minlength=8)
    q = lambda v: f"{np.median(v):6.1f}/{np.percentile(v, 90):6.1f}"  # noqa: E731
    late = np.percentile(rel[:, 0], 90)
    return (f"{name:28s} blocks {len(new):4d} span {span:7.1f}us rounds {rounds} | start p90 {late:6.1f} | "
            f"prologue {q(pro)} | loop {q(loop)} | epi-issue {q(issue)} | epi-drain {q(drain)} | "
            f"end p10/p50/max {np.percentile(rel[:, 4], 10):6.1f}/{np.median(rel[:, 4]):6.1f}/{span:6.1f} | "
            f"xcc {xcc.tolist()}")


def main():
    B = int(os.environ.get("B", "256"))
    dev = torch.device("cuda")
    T = torch.bfloat16
    s = L.stream_ptr()
    for li, (name, cs, h, w) in enumerate(geometries(B, 32, 256)):
        d = cs.desc(B, h, w)
        x = torch.randn(B, h, w, cs.ci, device=dev).to(T)
        wt = (torch.randn(cs.co, cs.kh, cs.kw, cs.ci, device=dev) * 0.05).to(T)
        y = torch.empty(B, d.Ho, d.Wo, cs.co, device=dev, dtype=T)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        rows = max(L.lib().crnn_conv_stat_rows(L.BF16, d), 2 * ((B * d.Ho * d.Wo + 63) // 64))
        ps = torch.empty(rows, cs.co, device=dev)
        pq = torch.empty(rows, cs.co, device=dev)
        need = L.lib().crnn_conv_wgrad_workspace(L.BF16, d)
        ws = torch.empty(need // 4 + 1, device=dev)
        dw = torch.empty(cs.co, cs.ci_real, cs.kh, cs.kw, device=dev)
        twt = wt.flip(1, 2).permute(3, 1, 2, 0).contiguous() if L.lib().crnn_conv_dgrad_tw_rows(L.BF16, d) else None
        ops = {
            "fwd": lambda: L.call("crnn_conv_fwd", L.BF16, d, x.data_ptr(), wt.data_ptr(), y.data_ptr(),
                                  ps.data_ptr(), pq.data_ptr(), s),
            "dgrad": lambda: L.call("crnn_conv_dgrad", L.BF16, d, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(),
                                    None, None, 0, s),
            "dgradtw": (lambda: L.call("crnn_conv_dgrad_tw", L.BF16, d, dy.data_ptr(), twt.data_ptr(),
                                       dx.data_ptr(), None, None, 0, s)) if twt is not None else None,
            "wgrad": lambda: L.call("crnn_conv_wgrad", L.BF16, d, dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                    ws.data_ptr(), need, 0.0, s),
        }
        for k, fn in ops.items():
            if fn is None or (k == "dgrad" and name == "stem0"):
                continue
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            a = read_stamps()
            fn()
            torch.cuda.synchronize()
            b = read_stamps()
            print(analyse(f"{name} {k}", a, b), flush=True)


if __name__ == "__main__":
    main()
