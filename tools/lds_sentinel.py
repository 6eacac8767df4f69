"""In-process LDS cross-talk probe (VERDICT r04 "next 1"): a side stream keeps LDS sentinel workgroups
(crnn_diag_lds_sentinel: fill LDS with a pattern, re-check it) resident while the main stream runs ONE
kind of aggressor kernel at a time — this library's LDS-DMA GEMMs (the 256-row conv fwd / dgrad / wgrad,
the W-halo conv), the halo stem convs, or hipBLASLt (torch.matmul). Any sentinel word that changes is an
LDS write from outside its workgroup's allocation.
    python tools/lds_sentinel.py [--rounds 20] [--lds 4096,16384,32768] [--only NAME,...]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

from crnn_hip import _lib as L  # noqa: E402
from kbench import geometries  # noqa: E402


def aggressors(B, s):
    dev = torch.device("cuda")
    T = torch.bfloat16
    out = {}
    keep = []
    for name, cs, h, w in geometries(B, 32, 256):
        if name not in ("stem1", "b0.c1", "b1.c2", "b3.c2", "b5.c2", "co0"):
            continue
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
        keep += [d, x, wt, y, dy, dx, ps, pq, ws, dw]
        out[f"{name}.fwd"] = (lambda d=d, x=x, wt=wt, y=y, ps=ps, pq=pq: L.call(
            "crnn_conv_fwd", L.BF16, d, x.data_ptr(), wt.data_ptr(), y.data_ptr(), ps.data_ptr(), pq.data_ptr(), s))
        out[f"{name}.dgrad"] = (lambda d=d, dy=dy, wt=wt, dx=dx: L.call(
            "crnn_conv_dgrad", L.BF16, d, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), None, None, 0, s))
        out[f"{name}.wgrad"] = (lambda d=d, dy=dy, x=x, dw=dw, ws=ws, need=need: L.call(
            "crnn_conv_wgrad", L.BF16, d, dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), need, 0.0, s))
    # the BiLSTM recurrence kernels at cfg2 (B = 256, T = 32, H = 512): per-step (gemm_oneshot LDS-DMA burst
    # + cell kernels) and persistent (lstm_seq.hip)
    Tn, H = 32, 512
    xg = (torch.randn(B, Tn, 2, 4 * H, device=dev) * 0.1).to(T)
    whh = (torch.randn(2, 4 * H, H, device=dev) * 0.05).to(T)
    whh_t = whh.transpose(1, 2).contiguous()
    hseq = (torch.randn(B, Tn, 2 * H, device=dev) * 0.1).to(T)
    gsv = torch.rand(2, Tn, B, 4 * H, device=dev).to(T)
    csv = torch.randn(2, Tn, B, H, device=dev)
    dhseq = (torch.randn(B, Tn, 2 * H, device=dev) * 0.1).to(T)
    dgates = (torch.randn(2, Tn, B, 4 * H, device=dev) * 0.1).to(T)
    dc = torch.zeros(2, B, H, device=dev)
    bws = torch.empty(L.lib().crnn_lstm_bptt_workspace(B, H) // 4 + 1, device=dev)
    sws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4 + 1, device=dev, dtype=torch.int32)
    keep += [xg, whh, whh_t, hseq, gsv, csv, dhseq, dgates, dc, bws, sws]
    out["lstm.step_fwd"] = lambda: L.call("crnn_lstm_step_fwd", L.BF16, xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(),
                                          gsv.data_ptr(), csv.data_ptr(), B, Tn, H, 5, s)
    out["lstm.step_bwd"] = lambda: L.call("crnn_lstm_step_bwd", L.BF16, dhseq.data_ptr(), whh.data_ptr(),
                                          whh_t.data_ptr(), gsv.data_ptr(), csv.data_ptr(), dgates.data_ptr(),
                                          dc.data_ptr(), bws.data_ptr(), B, Tn, H, 5, s)
    out["lstm.seq_fwd"] = lambda: L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(),
                                         gsv.data_ptr(), csv.data_ptr(), sws.data_ptr(), B, Tn, H, s)
    out["lstm.seq_bwd"] = lambda: L.call("crnn_lstm_seq_bwd", dhseq.data_ptr(), whh_t.data_ptr(), gsv.data_ptr(),
                                         csv.data_ptr(), dgates.data_ptr(), sws.data_ptr(), B, Tn, H, s)
    dx = torch.empty(B, Tn, 512, device=dev, dtype=T)
    keep.append(dx)
    out["lstm.dx"] = lambda: L.call("crnn_lstm_dx", L.BF16, dgates.data_ptr(), whh.data_ptr(), dx.data_ptr(), B, Tn,
                                    H, 512, s)
    a = torch.randn(4096, 4096, device=dev).to(T)
    b = torch.randn(4096, 4096, device=dev).to(T)
    c = torch.empty(4096, 4096, device=dev, dtype=T)
    keep += [a, b, c]
    out["hipblaslt.matmul"] = lambda: torch.matmul(a, b, out=c)
    out["none"] = lambda: None
    return out, keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lds", default="4096,16384,32768")
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--sleep", type=int, default=1)
    ap.add_argument("--launches", type=int, default=4, help="aggressor launches per round")
    ap.add_argument("--only", default=None)
    ap.add_argument("--mode", type=int, default=0, help="sentinel mode bits: 1 rewrite per check, 2 shuffle check")
    a = ap.parse_args()
    torch.cuda.init()
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    ops, _keep = aggressors(a.batch, main_s.cuda_stream)
    nw = L.lib().crnn_diag_lds_sentinel_words()
    out = torch.zeros(nw, dtype=torch.int32, device="cuda")
    total = {}
    for name, fn in ops.items():
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        for lds in [int(v) for v in a.lds.split(",")]:
            bad = waves = checks = 0
            recs = []
            for r in range(a.rounds):
                out.zero_()
                torch.cuda.synchronize()
                # alternate who is queued first, so both orders of arrival on the CUs occur
                if r % 2 == 0:
                    for _ in range(a.launches // 2):
                        fn()
                side.wait_stream(main_s)
                with torch.cuda.stream(side):
                    L.call("crnn_diag_lds_sentinel", out.data_ptr(), a.blocks, lds, a.iters, 1234 + r, a.sleep,
                           a.mode, side.cuda_stream)
                for _ in range(a.launches - (a.launches // 2 if r % 2 == 0 else 0)):
                    fn()
                torch.cuda.synchronize()
                o = out.cpu().numpy().view("uint32")
                bad += int(o[0])
                waves += int(o[2])
                checks += int(o[3])
                for k in range(min(int(o[1]), 64)):
                    if len(recs) < 6:
                        recs.append([hex(int(v)) for v in o[8 + 8 * k: 16 + 8 * k]])
            total[(name, lds)] = bad
            print(f"{name:18s} lds {lds:6d}: {bad:8d} corrupted words, {waves:5d} waves hit, {checks} block-checks",
                  flush=True)
            for rr in recs:
                print("    rec {index, got, expected, HW_ID, LDS_ALLOC, XCC_ID, check, block}:", rr, flush=True)
    hit = {k: v for k, v in total.items() if v}
    print("SUMMARY:", "no corruption" if not hit else f"corruption under {sorted(hit)}", flush=True)


if __name__ == "__main__":
    main()
