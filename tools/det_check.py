"""Determinism check of the training backward: the same step twice in one process must give
bit-identical parameter gradients. Prints the parameters whose gradients differ (max abs diff,
relative to the gradient's max), for the default engine and with single features switched off.
    python tools/det_check.py [B H W hidden]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402


def run(B, H, W, hidden, **flags):
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(hidden, 194), 5), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(B, H, W, W // 8, 194, seed=100)
    x = x.cuda()
    m(x)
    for k, v in flags.items():
        setattr(m._engine, k, v)
    m._engine._pack_jobs = None
    m._engine.packed_version = None
    if flags.get("dgrad_tw") is False:
        for k in [k for k in m._engine.packed if k.endswith(".t")]:
            del m._engine.packed[k]
    outs = []
    for _ in range(3):
        m.zero_grad(set_to_none=True)
        ctc_loss(m(x), tg, tl).backward()
        torch.cuda.synchronize()
        outs.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
    bad = []
    for k in outs[0]:
        for o in outs[1:]:
            d = float((o[k] - outs[0][k]).abs().max())
            if d > 0:
                bad.append((k, d / (float(outs[0][k].abs().max()) + 1e-30)))
                break
    return bad


def main():
    B, H, W, hid = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (16, 32, 128, 64)))
    for flags in ({}, {"pool_out_reduce": False}, {"dgrad_tw": False}, {"use_seq": False}):
        bad = run(B, H, W, hid, **flags)
        print(f"B={B} {H}x{W} hidden {hid} flags {flags}: {len(bad)} parameters differ between identical steps",
              sorted(bad, key=lambda t: -t[1])[:6], flush=True)


if __name__ == "__main__":
    main()
