"""Load-sensitivity check of the training step: the same step repeated while a side stream keeps
the device busy (device copies, pinned D2H / H2D copies) must give bit-identical parameter
gradients to a quiet run. A kernel whose result depends on wave / workgroup timing (float atomics,
an unsynchronised LDS or cross-workgroup hand-off) shows up as parameters that differ.
    python tools/race_check.py [B H W hidden reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402


def main():
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    a = [int(v) for v in sys.argv[1:6]] if len(sys.argv) > 5 else [16, 32, 128, 64, 12]
    B, H, W, hid, reps = a
    m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(hid, 194), 5), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(B, H, W, W // 8, 194, seed=100)
    x = x.cuda()
    m(x)
    offs = m.flat_offsets()

    def step():
        for p in m.parameters():
            p.grad = None
        ctc_loss(m(x), tg, tl).backward()

    def where(d, ref):
        out = []
        for k, (s, n) in offs.items():
            v = float(d[s:s + n].abs().max())
            if v > 0:
                out.append((round(v / (float(ref[s:s + n].abs().max()) + 1e-30), 7), k))
        return len(out), sorted(out, reverse=True)[:5]

    step()
    torch.cuda.synchronize()
    g0 = m._flat_grad.detach().clone()
    side = torch.cuda.Stream()
    big = torch.empty(32 << 20, device="cuda")
    big2 = torch.empty_like(big)
    host = torch.empty(8 << 20, pin_memory=True)
    dev_small = torch.empty(8 << 20, device="cuda")
    nbad = 0
    for i in range(reps):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(6):
                big2.copy_(big)
                host.copy_(dev_small, non_blocking=True)
                dev_small.copy_(host, non_blocking=True)
        step()
        torch.cuda.synchronize()
        n, top = where(m._flat_grad - g0, g0)
        nbad += n > 0
        print(f"rep {i}: {n} params differ from the quiet step {top}", flush=True)
    print(f"B={B} {H}x{W} hidden {hid}: {nbad} of {reps} loaded steps differ", flush=True)


if __name__ == "__main__":
    main()
