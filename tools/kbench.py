"""Per-layer conv microbenchmark on the HIP path (bf16, B=256, 32x256 geometry).
Prints TFLOP/s for fwd / dgrad / wgrad of each distinct conv geometry in SE-ResNet31.
    python tools/kbench.py [--iters 20] [--only fwd|dgrad|wgrad] [--layer N]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
import torch  # noqa: E402

from crnn_hip import _lib as L  # noqa: E402
from crnn_hip.engine import backbone_specs  # noqa: E402


def geometries(B, H, W):
    stem0, stem1, blocks, co0, co1 = backbone_specs()
    out = []
    h, w = H, W
    out.append(("stem0", stem0, h, w)); h, w = stem0.out_hw(h, w)
    out.append(("stem1", stem1, h, w)); h, w = stem1.out_hw(h, w)
    h, w = h // 2, w // 2
    seen = set()
    for i, b in enumerate(blocks):
        for nm, cs, hh, ww in [("c1", b.conv1, h, w), ("c2", b.conv2, *b.conv1.out_hw(h, w))] + \
                ([("ds", b.ds, h, w)] if b.ds is not None else []):
            key = (cs.ci, cs.co, cs.kh, cs.sh, hh, ww)
            if key not in seen:
                seen.add(key)
                out.append((f"b{i}.{nm}", cs, hh, ww))
        h, w = b.conv1.out_hw(h, w)
    out.append(("co0", co0, h, w)); h, w = co0.out_hw(h, w)
    out.append(("co1", co1, h, w))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default=None)
    ap.add_argument("--layer", type=int, default=None)
    ap.add_argument("--opt", default=None, help="A/B a crnn_set_option key: KEY=V0,V1 (e.g. 0=0,1)")
    ap.add_argument("--set", action="append", default=[], help="fixed crnn_set_option KEY=V for every variant")
    a = ap.parse_args()
    dev = torch.device("cuda")
    T = torch.bfloat16
    s = L.stream_ptr()
    tot = {}
    key, variants = None, [("", None)]
    for kv in a.set:
        k_, v_ = kv.split("=")
        L.call("crnn_set_option", int(k_), int(v_))
    if a.opt:
        ks, vs = a.opt.split("=")
        key = int(ks)
        variants = [(f"[{v}]", int(v)) for v in vs.split(",")]
    for li, (name, cs, h, w) in enumerate(geometries(a.batch, 32, 256)):
        if a.layer is not None and li != a.layer:
            continue
        d = cs.desc(a.batch, h, w)
        x = torch.randn(a.batch, h, w, cs.ci, device=dev).to(T)
        wt = (torch.randn(cs.co, cs.kh, cs.kw, cs.ci, device=dev) * 0.05).to(T)
        y = torch.empty(a.batch, d.Ho, d.Wo, cs.co, device=dev, dtype=T)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        # BN partial rows: sized for the smallest tile (an --opt variant may change the kernel's tile)
        rows = max(L.lib().crnn_conv_stat_rows(L.BF16, d), 2 * ((a.batch * d.Ho * d.Wo + 63) // 64))
        ps = torch.empty(rows, cs.co, device=dev)
        pq = torch.empty(rows, cs.co, device=dev)
        need = L.lib().crnn_conv_wgrad_workspace(L.BF16, d)
        ws = torch.empty(need // 4 + 1, device=dev)
        dw = torch.empty(cs.co, cs.ci_real, cs.kh, cs.kw, device=dev)
        flop = 2.0 * a.batch * d.Ho * d.Wo * cs.co * cs.ci_real * cs.kh * cs.kw
        twt = None
        if L.lib().crnn_conv_dgrad_tw_rows(L.BF16, d) > 0:   # the forward-path dgrad's transposed kernel
            twt = wt.flip(1, 2).permute(3, 1, 2, 0).contiguous()
        ops = {
            "fwd": lambda: L.call("crnn_conv_fwd", L.BF16, d, x.data_ptr(), wt.data_ptr(), y.data_ptr(),
                                  ps.data_ptr(), pq.data_ptr(), s),
            "dgrad": lambda: L.call("crnn_conv_dgrad", L.BF16, d, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), None,
                                    None, 0, s),
            "dgradtw": (lambda: L.call("crnn_conv_dgrad_tw", L.BF16, d, dy.data_ptr(), twt.data_ptr(), dx.data_ptr(),
                                       None, None, 0, s)) if twt is not None else None,
            "wgrad": lambda: L.call("crnn_conv_wgrad", L.BF16, d, dy.data_ptr(), x.data_ptr(), dw.data_ptr(),
                                    ws.data_ptr(), need, 0.0, s),
        }
        line = f"{li:2d} {name:8s} Ci={cs.ci:3d} Co={cs.co:3d} k={cs.kh}x{cs.kw} s={cs.sh},{cs.sw} in={h}x{w} " \
               f"GF={flop / 1e9:7.1f} |"
        for k, fn in ops.items():
            if fn is None or (a.only and k not in a.only.split(",")):
                continue
            if k == "dgrad" and name == "stem0":
                continue
            for tag, val in variants:
                if key is not None:
                    L.call("crnn_set_option", key, val)
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                tot[k + tag] = tot.get(k + tag, 0.0) + ms
                line += f" {k}{tag} {ms * 1e3:7.1f}us {flop / ms / 1e9:6.0f}TF |"
        print(line, flush=True)
    print("sum of distinct-geometry times (ms):", {k: round(v, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()
