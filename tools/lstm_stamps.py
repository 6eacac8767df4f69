"""Phase timing of the persistent BiLSTM kernels (lstm_seq.hip) from in-kernel s_memrealtime
stamps (10 ns ticks). Prints per-phase medians and the hand-off latency (last producer's signal of
step s-1 -> consumer past its wait at step s), for every workgroup tile (CRNN_OPT_LSTM_TILE) the
shape supports, in one process.   python tools/lstm_stamps.py [B T H]
STAMPS_COLD=1: the stamped launch runs after a 1 GiB scratch write (weights, x-gates and ring out of L2 / MALL,
as inside the train step)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rcnn-ocr_amd"))
from crnn_hip import _lib as L  # noqa: E402

PH = ["start", "waited", "mfma+part", "reduced", "epilogue", "stored", "published"]


def run(kind, B, T, H, save=True):
    dev = torch.device("cuda")
    st = L.stream_ptr()
    g = torch.Generator(device="cpu").manual_seed(0)
    xg = (torch.randn(B, T, 2, 4 * H, generator=g) * 0.5).to(dev, torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, generator=g) / H ** 0.5).to(dev, torch.bfloat16)
    whh_t = whh.transpose(1, 2).contiguous()
    hseq = torch.zeros(B, T, 2 * H, device=dev, dtype=torch.bfloat16)
    gsv = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
    csv = torch.zeros(2, T, B, H, device=dev)
    dg = torch.zeros(2, T, B, 4 * H, device=dev, dtype=torch.bfloat16)
    ws = torch.zeros(L.lib().crnn_lstm_seq_workspace(B) // 4 + 4, dtype=torch.int32, device=dev)
    S, U = ctypes.c_int(0), ctypes.c_int(0)
    if not L.lib().crnn_lstm_seq_config(B, H, int(kind == "bwd"), ctypes.byref(S), ctypes.byref(U)):
        return
    S, U = S.value, U.value
    grid = 2 * (B // S) * (H // U)
    stamps = torch.zeros(grid * T * 8, dtype=torch.int64, device=dev)

    def fwd():
        L.call("crnn_lstm_seq_fwd", xg.data_ptr(), whh.data_ptr(), hseq.data_ptr(), gsv.data_ptr() if save else None,
               csv.data_ptr() if save else None, ws.data_ptr(), B, T, H, st)

    def bwd():
        L.call("crnn_lstm_seq_bwd", hseq.data_ptr(), whh_t.data_ptr(), gsv.data_ptr(), csv.data_ptr(), dg.data_ptr(),
               ws.data_ptr(), B, T, H, st)

    save0, save = save, True
    fwd()
    save = save0
    fn = fwd if kind == "fwd" else bwd
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    L.call("crnn_lstm_seq_debug_stamps", stamps.data_ptr())
    cold = os.environ.get("STAMPS_COLD") == "1"
    if cold:
        scratch = torch.empty(1 << 28, device=dev)
        scratch.fill_(1.0)
        torch.cuda.synchronize()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    if cold:
        print(f"  (stamped launch after a 1 GiB scratch write: {e0.elapsed_time(e1) * 1e3:.1f} us)")
    L.call("crnn_lstm_seq_debug_stamps", None)
    s = stamps.view(grid, T, 8).cpu().numpy().astype(np.int64)
    ho = {0: "counter", 1: "granule", 2: "unit-complete", 3: "unit-complete 8w"}.get(HANDOFF, str(HANDOFF))
    print(f"{kind}: B={B} T={T} H={H} tile {S}x{U} grid={grid} hand-off {ho if kind == 'fwd' else 'counter'}: "
          f"{'' if save else '(inference, nothing saved) '}{us:.1f} us/sweep = {us / T:.2f} us/step (no stamps)")
    steps = slice(2, T - 1)
    d = s[:, steps, :]
    for p in range(1, 7):
        if p in (1, 2, 3):   # only for s > 0
            pass
        dt = (d[:, :, p] - d[:, :, p - 1]) * 10 / 1e3
        print(f"  {PH[p - 1]:>10s} -> {PH[p]:<10s} median {np.median(dt):6.3f} us  p90 {np.percentile(dt, 90):6.3f}")
    per_step = (s[:, 1:, 0] - s[:, :-1, 0]) * 10 / 1e3
    print(f"  step period median {np.median(per_step):.3f} us")
    # hand-off: group = same (d, bs); physical block -> logical via the same xcd remap is not needed:
    # use all producers' published stamps of step s-1 vs this block's waited stamp at s (upper bound)
    nb = s.shape[0]
    last_pub = s[:, :-1, 6].max(axis=0)   # over all blocks
    wait_done = s[:, 1:, 1]
    lat = (wait_done - last_pub[None, :]) * 10 / 1e3
    print(f"  last publish (any block, step s-1) -> waited (step s): median {np.median(lat):.3f} us")
    # launch ramp and prologue: slot 7 of step 0 = the workgroup's entry stamp
    ent = s[:, 0, 7]
    if (ent > 0).all():
        t0 = ent.min()
        us_ = lambda v: (v - t0) * 10 / 1e3
        print(f"  entry spread (first -> last workgroup) {us_(ent.max()):.2f} us; entry -> step-0 start median "
              f"{np.median((s[:, 0, 0] - ent) * 10 / 1e3):.2f} us max {np.max((s[:, 0, 0] - ent) * 10 / 1e3):.2f}; "
              f"first entry -> last step-0 publish {us_(s[:, 0, 6].max()):.2f} us; first entry -> last step end "
              f"{us_(s[:, -1, 6].max()):.2f} us; steps 1..T-1 {(s[:, -1, 6].max() - s[:, 0, 6].max()) * 10 / 1e3 / (T - 1):.3f} us each")


HANDOFF = 1

if __name__ == "__main__":
    # forward under both hand-off forms (CRNN_OPT_LSTM_HANDOFF), each tile, in one process
    B, T, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 32, 512)
    if os.environ.get("STAMPS_FORMS"):
        # the given forward forms (CRNN_OPT_LSTM_HANDOFF values) at the default tile, alternated twice, then the BPTT
        # (phases of the unit-complete forms 2 / 3: waited = own K-slice polled, mfma+part = slice written to LDS,
        # reduced = past the barrier, epilogue = MFMAs + cell done, stored = granules published)
        forms = [int(v) for v in os.environ["STAMPS_FORMS"].split(",")]
        for _ in range(2):
            for HANDOFF in forms:
                L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, HANDOFF)
                run("fwd", B, T, H)
        run("bwd", B, T, H)
        sys.exit(0)
    if os.environ.get("STAMPS_BWD_FORMS"):
        # the BPTT under CRNN_OPT_LSTM_BWD_PART values (0: counter form, 1: partial-sum form; phases of form 1:
        # waited = partials gathered, mfma+part = cell done, reduced = past the barrier, epilogue = partial tiles
        # multiplied and published)
        for _ in range(2):
            for v in (int(x) for x in os.environ["STAMPS_BWD_FORMS"].split(",")):
                L.call("crnn_set_option", L.OPT_LSTM_BWD_PART, v)
                print(f"BPTT form CRNN_OPT_LSTM_BWD_PART={v}")
                run("bwd", B, T, H)
        L.call("crnn_set_option", L.OPT_LSTM_BWD_PART, 0)
        sys.exit(0)
    if os.environ.get("STAMPS_SAVE_AB"):
        # default tile and hand-off: saved-forward stores on / off (the BPTT operands' cost per step),
        # then the default BPTT
        for save in (True, False, True):
            run("fwd", B, T, H, save)
        run("bwd", B, T, H)
        sys.exit(0)
    for force in (1, 2, 3):
        L.call("crnn_set_option", L.OPT_LSTM_TILE, force)
        for HANDOFF in (1, 0, 1):
            L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, HANDOFF)
            run("fwd", B, T, H)
        run("bwd", B, T, H)
    L.call("crnn_set_option", L.OPT_LSTM_TILE, 0)
    L.call("crnn_set_option", L.OPT_LSTM_HANDOFF, 3)   # the default
