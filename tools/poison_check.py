"""Uninitialised-read check of the training step: run the step once, overwrite the engine's
workspace buffers and / or the flat gradient with garbage (NaN or random finite values), run the
identical step again and compare the parameter gradients. A kernel that reads memory it did not
write this step (stale partials, unwritten padding, a grad region it only partly overwrites)
shows up as a difference. Prints the workspace buffers a difference traces to when single
buffers are poisoned one at a time.
    python tools/poison_check.py [B H W hidden]"""
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
    B, H, W, hid = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (16, 32, 128, 64)))
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
        torch.cuda.synchronize()
        return m._flat_grad.detach().clone()

    def poison(t, kind):
        if t.is_floating_point():
            if kind == "nan":
                t.fill_(float("nan"))
            else:
                t.copy_((torch.randn(t.shape, device=t.device) * 3.0).to(t.dtype))
        else:
            t.copy_(torch.randint(-1000, 1000, t.shape, device=t.device).to(t.dtype))

    def where(d):
        out = []
        for k, (s, n) in offs.items():
            v = float(d[s:s + n].abs().nan_to_num(nan=float("inf")).max())
            if v > 0:
                out.append((v, k))
        return sorted(out, reverse=True)[:5]

    g0 = step()
    # the persistent BiLSTM's counters / status and the BN finalize tickets are zeroed once at
    # allocation and re-armed by their kernels: not scratch, never poisoned
    ws = {k: v for k, v in m._engine.ws.bufs.items() if k not in ("rnn.seq_ws", "bn.fin_ws")}
    print(f"B={B} {H}x{W} hidden {hid}: {len(ws)} workspace buffers, {m._engine.ws.nbytes() / 1e6:.1f} MB; "
          f"repeat step bit-identical: {bool(torch.equal(step(), g0))}", flush=True)
    for kind in ("nan", "rand"):
        for target in ("grad", "workspace", "both"):
            if target in ("grad", "both"):
                poison(m._flat_grad.detach(), kind)
            if target in ("workspace", "both"):
                for t in ws.values():
                    poison(t, kind)
            torch.cuda.synchronize()
            g = step()
            d = (g - g0)
            bad = where(d)
            print(f"poison {kind:4s} {target:9s}: {len(bad)} params differ {bad}", flush=True)
            if target == "workspace" and bad:
                for name, t in list(ws.items()):
                    step()
                    poison(t, kind)
                    torch.cuda.synchronize()
                    b1 = where(step() - g0)
                    if b1:
                        print(f"    buffer {name} {tuple(t.shape)} {t.dtype}: {b1[:3]}", flush=True)
            step()


if __name__ == "__main__":
    main()
