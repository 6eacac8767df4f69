"""Do our kernels disturb OTHER kernels that share the CUs with them? A side stream runs deterministic
torch work (bf16 GEMMs through hipBLASLt, fp32 reductions, an elementwise chain) over and over while
the bench train step (B, 32x256, hidden 512, bf16) runs on the compute stream; every side result must
be bit-identical to the one computed on an idle device. Mode "self": the same check on a copy of
our own step's gradients computed alone. Prints the number of differing side results.
    python tools/cohab_check.py [iters] [B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402


def side_work(a, b, x):
    c = a @ b                          # hipBLASLt GEMM (LDS tiles)
    s = x.sum(dim=1)                   # torch reduction kernels (LDS trees)
    m = x.amax(dim=0)
    e = torch.tanh(x[:4096] * 1.37 + 0.5).sum()
    return c, s, m, e


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    g = torch.Generator().manual_seed(3)
    a = torch.randn(4096, 4096, generator=g).cuda().bfloat16()
    b = torch.randn(4096, 4096, generator=g).cuda().bfloat16()
    x = torch.randn(16384, 4096, generator=g).cuda()
    torch.cuda.synchronize()
    ref = [t.clone() for t in side_work(a, b, x)]
    torch.cuda.synchronize()
    m = RCNN(num_classes=194, hidden_size=512, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(512, 194), 5), strict=False)
    m = m.cuda().train()
    xs, _, tg, tl = synthetic_batch(B, 32, 256, 32, 194, seed=100)
    xs = xs.cuda()
    m(xs)
    side = torch.cuda.Stream()
    bad = 0
    for i in range(iters):
        m.zero_grad(set_to_none=True)
        outs = []
        side.wait_stream(torch.cuda.current_stream())
        loss = ctc_loss(m(xs), tg, tl)
        with torch.cuda.stream(side):
            for _ in range(3):
                outs.append(side_work(a, b, x))
        loss.backward()
        with torch.cuda.stream(side):
            for _ in range(6):
                outs.append(side_work(a, b, x))
        torch.cuda.synchronize()
        nd = sum(1 for o in outs for t, r in zip(o, ref) if not torch.equal(t, r))
        bad += nd > 0
        print(f"iter {i}: {nd} of {len(outs) * 4} side results differ from the idle-device run", flush=True)
    print(f"{bad} of {iters} iterations with a differing side result", flush=True)


if __name__ == "__main__":
    main()
