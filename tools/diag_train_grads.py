"""Diagnostic: per-parameter gradient error of (CPU fp32 oracle) and (HIP fp32 path)
against a float64 oracle, on a train-golden case. Separates conditioning from bugs."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))
import crnn_oracle as O  # noqa: E402
from helpers import case_params, load, pixels_to_images  # noqa: E402


def oracle_grads(sd, x, tg, tl, dtype):
    p = {k: (v.to(dtype).clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.to(dtype) if v.is_floating_point() else v)) for k, v in sd.items()}
    logits = O.head(O.encode(x.to(dtype), p, O.Ctx(train=True)), p)
    loss = O.ctc_loss(logits, tg, tl)
    loss.backward()
    return {k: v.grad.double() for k, v in p.items() if v.is_floating_point() and v.grad is not None}, float(loss)


def main(case="b4_32x128_h256"):
    torch.set_num_threads(16)
    z = load(f"train_{case}.npz")
    sd, hidden = case_params(z, with_running=False)
    x = pixels_to_images(z["pixels"])
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    g64, l64 = oracle_grads(sd, x, tg, tl, torch.float64)
    g32, l32 = oracle_grads(sd, x, tg, tl, torch.float32)
    from model.model import RCNN
    from crnn_hip.ctc import ctc_loss
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    m = m.cuda().train()
    loss = ctc_loss(m(x.cuda()), tg, tl)
    loss.backward()
    torch.cuda.synchronize()
    gh = {k: v.grad.double().cpu() for k, v in m.named_parameters()}
    print(f"loss fp64 {l64:.8f} cpu32 {l32:.8f} hip32 {float(loss):.8f}")
    worst = []
    for k in g64:
        r = g64[k]
        n = float(r.norm()) + 1e-30
        e32 = float((g32[k] - r).norm()) / n
        eh = float((gh[k] - r).norm()) / n
        worst.append((eh, e32, k))
    worst.sort(reverse=True)
    for eh, e32, k in worst[:25]:
        print(f"{k:45s} hip32 {eh:.2e}  cpu32 {e32:.2e}")
    print("median hip32", np.median([w[0] for w in worst]), "median cpu32", np.median([w[1] for w in worst]))


if __name__ == "__main__" and (len(sys.argv) == 1 or sys.argv[1] not in ("stages", "bwd", "local")):
    main(*sys.argv[1:])


def stages(case="b4_32x128_h256", train="1"):
    """forward activation error per stage, HIP fp32 and CPU fp32 vs fp64 oracle."""
    z = load(f"train_{case}.npz")
    sd, hidden = case_params(z, with_running=False)
    x = pixels_to_images(z["pixels"])
    tr = train == "1"
    res = {}
    for dt in (torch.float64, torch.float32):
        p = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in sd.items()}
        ctx = O.Ctx(train=tr, record=True)
        with torch.no_grad():
            O.encode(x.to(dt), p, ctx)
        res[dt] = ctx.acts
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    m = m.cuda().train(tr)
    with torch.no_grad():
        m(x.cuda())
    eng = m._engine
    pairs = {"stem": "s1.pool", "layer1": "b0.y", "layer2": "b2.y", "layer3": "b7.y", "layer4": "b10.y"}
    for k, b in pairs.items():
        ref = res[torch.float64][k]
        got = eng.ws.bufs[b].double().permute(0, 3, 1, 2).cpu()
        c32 = res[torch.float32][k].double()
        print(f"{k:8s} hip {float((got-ref).norm()/ref.norm()):.2e} cpu32 {float((c32-ref).norm()/ref.norm()):.2e}")
    for k, b in [("seq", "seq"), ("rnn0", "r0.out"), ("rnn1", "r1.out")]:
        ref = res[torch.float64][k]
        got = eng.ws.bufs[b].double().cpu()
        c32 = res[torch.float32][k].double()
        print(f"{k:8s} hip {float((got-ref).norm()/ref.norm()):.2e} cpu32 {float((c32-ref).norm()/ref.norm()):.2e}")
    # first conv output (pre-BN) directly
    zz = eng.ws.bufs["s0.z"].double().permute(0, 3, 1, 2).cpu()
    import torch.nn.functional as F
    ref = F.conv2d(x.double(), sd["cnn.conv0.0.weight"].double(), padding=1)
    print("s0.z", float((zz - ref).norm() / ref.norm()))
    for nm in ["s0.mean", "s0.inv"]:
        print(nm, eng.ws.bufs[nm][:4].cpu().tolist())
    mu = ref.mean(dim=(0, 2, 3))
    var = ref.var(dim=(0, 2, 3), unbiased=False)
    print("ref mean", mu[:4].tolist(), "ref inv", (1 / torch.sqrt(var + 1e-5))[:4].tolist())


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "stages":
    stages(*sys.argv[2:])


def bwd_stages(case="b4_32x128_h256"):
    """upstream-gradient error per block boundary, HIP fp32 vs fp64 oracle (and CPU fp32)."""
    z = load(f"train_{case}.npz")
    sd, hidden = case_params(z, with_running=False)
    x = pixels_to_images(z["pixels"])
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    acts = {}
    for dt in (torch.float64, torch.float32):
        p = {k: (v.to(dt).clone().requires_grad_(True) if v.is_floating_point() and "running" not in k
                 else (v.to(dt) if v.is_floating_point() else v)) for k, v in sd.items()}
        ctx = O.Ctx(train=True, record=True)
        logits = O.head(O.encode(x.to(dt), p, ctx), p)
        O.ctc_loss(logits, tg, tl).backward()
        acts[dt] = ctx.acts
    from model.model import RCNN
    from crnn_hip.ctc import ctc_loss
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    m = m.cuda().train()
    m._engine_for(x.cuda()).debug = True
    ctc_loss(m(x.cuda()), tg, tl).backward()
    torch.cuda.synchronize()
    dbg = m._engine.dbg
    ref, c32 = acts[torch.float64]["seq"].grad, acts[torch.float32]["seq"].grad.double()
    got = dbg["dseq"].double().cpu()
    print(f"dseq      hip {float((got-ref).norm()/ref.norm()):.2e} cpu32 {float((c32-ref).norm()/ref.norm()):.2e}")
    names = [f"{st}.{i}" for st, n, *_ in O.STAGES for i in range(n)]
    for bi in reversed(range(len(names))):
        ref = acts[torch.float64][names[bi]].grad
        c32 = acts[torch.float32][names[bi]].grad.double()
        got = dbg[f"dy.b{bi}"].double().permute(0, 3, 1, 2).cpu()
        print(f"{names[bi]:9s} hip {float((got-ref).norm()/ref.norm()):.2e} "
              f"cpu32 {float((c32-ref).norm()/ref.norm()):.2e}")
    ref = acts[torch.float64]["stem"].grad
    got = dbg["dpool"].double().view(ref.shape[0], ref.shape[2], ref.shape[3], ref.shape[1]).permute(0, 3, 1, 2).cpu()
    print(f"stem      hip {float((got-ref).norm()/ref.norm()):.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "bwd":
    bwd_stages(*sys.argv[2:])


def block_local(case="b4_32x128_h256"):
    """per-block decision-consistent local errors (tests/blockcheck.py)."""
    from blockcheck import block_errors
    z = load(f"train_{case}.npz")
    sd, hidden = case_params(z, with_running=False)
    x = pixels_to_images(z["pixels"])
    tg, tl = torch.from_numpy(z["targets"]), torch.from_numpy(z["target_lengths"])
    from model.model import RCNN
    from crnn_hip.ctc import ctc_loss
    m = RCNN(num_classes=194, hidden_size=hidden, blank_id=None, compute_dtype=torch.float32)
    m.load_state_dict(sd, strict=False)
    m = m.cuda().train()
    m._engine_for(x.cuda()).debug = True
    ctc_loss(m(x.cuda()), tg, tl).backward()
    torch.cuda.synchronize()
    params = dict(m.named_parameters())
    for bi, e in block_errors(m._engine, params, {k: v.grad for k, v in params.items()}):
        print(f"block {bi:2d} " + " ".join(f"{k}={v:.1e}" for k, v in e.items()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "local":
    block_local(*sys.argv[2:])
