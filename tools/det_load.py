"""Determinism of the training backward UNDER LOAD: the same step several times in this process
while a second process keeps the GPU busy (bench.py), the condition of the two-rank rehearsal
(tests/test_gpu_dp.py). Prints the parameters whose gradients differ from the first step's.
    python tools/det_load.py [steps] [B H W hidden]"""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    B, H, W, hid = (int(a) for a in (sys.argv[2:6] if len(sys.argv) > 5 else (16, 32, 128, 64)))
    import crnn_oracle as O
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    from crnn_hip import _lib as L
    # CRNN_DET_SET="KEY=V,KEY=V": library options for this process only (crnn_set_option), e.g. 0=0
    # turns the 256-row GEMM's wave-half stagger off
    for kv in filter(None, os.environ.get("CRNN_DET_SET", "").split(",")):
        k, v = kv.split("=")
        L.call("crnn_set_option", int(k), int(v))
        print("option", k, "=", v, flush=True)
    load = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline", "--steps", "3000",
                             "--warmup", "2", "--batch", "128"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
        m.load_state_dict(recipe_state_dict(O.param_shapes(hid, 194), 5), strict=False)
        m = m.cuda().train()
        x, _, tg, tl = synthetic_batch(B, H, W, W // 8, 194, seed=100)
        x = x.cuda()
        m(x)
        time.sleep(12)   # the load process is past its start-up
        ref = None
        for i in range(steps):
            m.zero_grad(set_to_none=True)
            ctc_loss(m(x), tg, tl).backward()
            torch.cuda.synchronize()
            g = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
            # every engine workspace buffer's final state too: the first producer that differs
            g.update({"ws:" + k: v.detach().clone() for k, v in m._engine.ws.bufs.items()
                      if v.is_floating_point() and not k.startswith("rnn.seq_ws")})
            if ref is None:
                ref = g
                continue
            bad = sorted(((float((g[k].float() - ref[k].float()).abs().max()), k) for k in g
                          if g[k].shape == ref[k].shape and not torch.equal(g[k], ref[k])), reverse=True)
            wsb = [b for b in bad if b[1].startswith("ws:")]
            pb = [b for b in bad if not b[1].startswith("ws:")]
            order = {k: n for n, (k, _) in enumerate(m.named_parameters())}
            deep = sorted((order[k], k) for _, k in pb)[-6:]   # the ones nearest the loss: the origin
            print(f"step {i}: {len(pb)} parameters differ from step 0 {pb[:4]}; nearest the loss "
                  f"{[k for _, k in deep]}; workspace buffers {wsb[:8]}", flush=True)
    finally:
        load.kill()
        load.wait()


if __name__ == "__main__":
    main()
