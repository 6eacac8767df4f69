"""In-process version of the r04 two-process probe (VERDICT r04 "next 1": no two-process runs): a second
model of this library (its own engine, buffers and batch: the bf16 bench step with every LDS-DMA GEMM,
the W-halo and halo stem convs) trains on a SIDE stream while the victim model repeats one bf16 train
step (B=256, 32x256, hidden 512) on the compute stream. Every victim gradient must be bit-identical to
the one it computed on an idle device; the aggressor's own gradients are checked the same way.
    python tools/cohab_model.py [iters] [victim_seq 0|1] [aggressor_seq 0|1]
CRNN_OPTS="key=value,..." sets crnn_set_option switches first."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402


def make(seed, B, use_seq):
    import crnn_oracle as O
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    m = RCNN(num_classes=194, hidden_size=512, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
    m.load_state_dict(recipe_state_dict(O.param_shapes(512, 194), seed), strict=False)
    m = m.cuda().train()
    xs, _, tg, tl = synthetic_batch(B, 32, 256, 32, 194, seed=100 + seed)
    xs = xs.cuda()
    m(xs)
    m._engine.use_seq = use_seq
    return m, xs, tg, tl


def grads(m):
    return {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


def diff(g, ref):
    """(differing elements, max |d|, the differing parameters nearest the loss)"""
    bad = [k for k in g if not torch.equal(g[k], ref[k])]
    n = sum(int((g[k] != ref[k]).sum()) for k in bad)
    mx = max((float((g[k] - ref[k]).abs().max()) for k in bad), default=0.0)
    return n, mx, bad[::-1][:4]


def step(m, xs, tg, tl):
    from crnn_hip.ctc import ctc_loss
    m.zero_grad(set_to_none=True)
    ctc_loss(m(xs), tg, tl).backward()


def snaps(m):
    """the engine's debug snapshots of the SE chain (engine.debug), kernel order within each block"""
    return {k: v for k, v in m._engine.dbg.items() if k.startswith("se.")}


def first_diff(sn, ref):
    """per block (backward order): the first snapshot that differs from the reference run"""
    out = []
    blocks = sorted({k.split(".")[1] for k in sn}, key=lambda b: -int(b[1:]))
    for b in blocks:
        keys = [k for k in sn if k.split(".")[1] == b]
        bad = [k for k in keys if not torch.equal(sn[k], ref[k])]
        if bad:
            k = bad[0]   # the first differing snapshot: how many elements, how far, where
            d = (sn[k].float() - ref[k].float()).reshape(-1)
            idx = (d != 0).nonzero().reshape(-1)
            rel = float(d.abs().max() / (ref[k].float().abs().max() + 1e-30))
            out.append((b, [x.split(".", 2)[2] for x in bad],
                        f"first {k.split('.', 2)[2]}: {idx.numel()} of {d.numel()} elements differ, max rel "
                        f"{rel:.2e}, at {idx[:8].tolist()}, got {sn[k].reshape(-1)[idx[:4]].tolist()} "
                        f"ref {ref[k].reshape(-1)[idx[:4]].tolist()}"))
    return out[:2]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    victim_seq = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    aggr_seq = bool(int(sys.argv[3])) if len(sys.argv) > 3 else False
    kind = sys.argv[4] if len(sys.argv) > 4 else "model"
    from crnn_hip import _lib as L
    for kv in os.environ.get("CRNN_OPTS", "").split(","):
        if kv:
            L.call("crnn_set_option", *[int(v) for v in kv.split("=")])
    vm, vx, vtg, vtl = make(5, 256, victim_seq)
    am, ax, atg, atl = make(6, 256, aggr_seq)
    probe = os.environ.get("COHAB_PROBE") == "1"
    vm._engine.debug = am._engine.debug = probe
    step(vm, vx, vtg, vtl)
    torch.cuda.synchronize()
    vref = grads(vm)
    vsref = snaps(vm) if probe else {}
    step(am, ax, atg, atl)
    torch.cuda.synchronize()
    aref = grads(am)
    asref = snaps(am) if probe else {}
    side = torch.cuda.Stream()
    vbad = abad = 0
    for i in range(iters):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                step(am, ax, atg, atl)   # the aggressor's forward + backward overlap the victim's step
        step(vm, vx, vtg, vtl)
        torch.cuda.synchronize()
        vg, ag = grads(vm), grads(am)
        vd, vmx, vnames = diff(vg, vref)
        ad, amx, anames = diff(ag, aref)
        vbad += vd > 0
        abad += ad > 0
        print(f"iter {i}: victim {vd} gradient elements differ (max |d| {vmx:.3e}) {vnames}; "
              f"aggressor {ad} ({amx:.3e}) {anames}", flush=True)
        if probe and vd:
            print("    victim SE chain, first differing snapshots per block:", first_diff(snaps(vm), vsref), flush=True)
        if probe and ad:
            print("    aggressor SE chain, first differing snapshots per block:", first_diff(snaps(am), asref),
                  flush=True)
    print(f"SUMMARY {kind} opts={os.environ.get('CRNN_OPTS', '')} victim_seq={int(victim_seq)} aggressor_seq={int(aggr_seq)}: victim differs in {vbad} of {iters} "
          f"iterations, aggressor in {abad}", flush=True)


if __name__ == "__main__":
    main()
