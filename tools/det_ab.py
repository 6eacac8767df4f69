"""A/B of the BN finalize forms under an in-process CU-occupying side stream (r04): the r01-r03
ticketed chunk fold (CRNN_OPT_FIN_TICKET = 1) against the one-launch form without a hand-off (0).
For each form: the finalize alone (SE-block shape, 200 launches) and the bench train step
(B, 32x256, hidden 512, bf16; 8 steps), counting launches / steps whose results differ from the
first. Prints one line per case.
    python tools/det_ab.py [B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

from test_gpu_determinism import SideLoad  # noqa: E402


def fin_case(L, opt, rows=256, C=256, n=200):
    L.call("crnn_set_option", 17, opt)
    g = torch.Generator().manual_seed(1)
    pg, pgx = torch.randn(rows, C, generator=g).cuda(), torch.randn(rows, C, generator=g).cuda()
    fws = torch.zeros((L.lib().crnn_bn_finalize_workspace(512) + 3) // 4, device="cuda")
    outs = [torch.empty(C, device="cuda") for _ in range(4)]
    load = SideLoad()
    ref, bad = None, 0
    for i in range(n):
        load.issue(3)
        L.call("crnn_bn_bwd_finalize", pg.data_ptr(), pgx.data_ptr(), rows, C, rows * 64, outs[0].data_ptr(),
               outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(), 0, fws.data_ptr(), L.stream_ptr())
        got = torch.cat([o.clone() for o in outs])
        torch.cuda.synchronize()
        if ref is None:
            ref = got
        elif not torch.equal(got, ref):
            bad += 1
    print(f"finalize opt {opt}: {bad} of {n - 1} launches differ from the first", flush=True)


def step_case(L, opt, B, steps=8):
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    L.call("crnn_set_option", 17, opt)
    m = RCNN(num_classes=194, hidden_size=512, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(512, 194), 5), strict=False)
    m = m.cuda().train()
    x, _, tg, tl = synthetic_batch(B, 32, 256, 32, 194, seed=100)
    x = x.cuda()
    m(x)
    load = SideLoad(n=4096)
    order = {k: n for n, (k, _) in enumerate(m.named_parameters())}
    ref, bad = None, 0
    for i in range(steps):
        m.zero_grad(set_to_none=True)
        load.issue(4)
        loss = ctc_loss(m(x), tg, tl)
        load.issue(12)
        loss.backward()
        torch.cuda.synchronize()
        g = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        if ref is None:
            ref = g
            continue
        diff = [k for k in g if not torch.equal(g[k], ref[k])]
        if diff:
            bad += 1
            near = sorted(diff, key=lambda k: order[k])[-4:]
            print(f"  opt {opt} step {i}: {len(diff)} gradients differ; nearest the loss {near}", flush=True)
    print(f"train step opt {opt} (B={B}): {bad} of {steps - 1} steps differ from the first", flush=True)


def main():
    from crnn_hip import _lib as L
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for opt in (1, 0):
        fin_case(L, opt)
    for opt in (1, 0):
        step_case(L, opt, B)


if __name__ == "__main__":
    main()
