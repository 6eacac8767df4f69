"""Run-to-run determinism of the SE weight gradient under a second process's load (the condition of
tests/test_gpu_dp.py at hidden 512, B = 128), with the diagnostic library that records what every
se_wgrad block READ (fixed-order sums of dsig, pooled, hid, dhid) and what it WROTE (dw2, dw1 sums):
    SRCS="bn.hip" tools/build_variant.sh seprobe -DCRNN_SE_PROBE=1
    CRNN_HIP_LIB=$PWD/rcnn-ocr_amd/crnn_hip/libcrnn_hip_seprobe.so python tools/se_probe.py [steps]
For each step that differs from step 0: the se_wgrad launches (backward order, 0 = the last block)
whose inputs differ and those whose outputs differ."""
import ctypes
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    B, H, W, hid = 128, 32, 256, 512
    import crnn_oracle as O
    from crnn_hip import _lib as L
    from crnn_hip.ctc import ctc_loss
    from crnn_hip.recipe import recipe_state_dict, synthetic_batch
    from model.model import RCNN
    lib = L.lib()
    probe = lib.crnn_diag_se_probe
    probe.argtypes = [ctypes.c_void_p, ctypes.c_int]
    NL, NB, NV = 32, 64, 6
    buf = np.zeros(NL * NB * NV, dtype=np.float32)
    env = dict(os.environ)
    env.pop("CRNN_HIP_LIB", None)   # the load process runs the default library
    if os.environ.get("SE_PROBE_LOAD") == "matmul":   # a load process with no kernel of this library
        cmd = [sys.executable, "-c", "import torch\na=torch.randn(4096,4096,device='cuda',dtype=torch.bfloat16)\n"
               "while True:\n  b=a@a\n  torch.cuda.synchronize()"]
    else:
        cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline", "--steps", "3000", "--warmup", "2",
               "--batch", "128"]
        if os.environ.get("SE_PROBE_LOAD") == "fp32":   # this library, but no LDS-DMA GEMM (fp32 kernels)
            cmd += ["--dtype", "fp32"]
    load = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
    try:
        if os.environ.get("SE_PROBE_SHIFT") == "1":
            # this process's device allocations at different virtual addresses from the load process's
            # (the two run the same allocation sequence otherwise): a test for cross-process aliasing
            pad = torch.empty((37 << 20) + 4096 * 7, dtype=torch.uint8, device="cuda")   # noqa: F841
        m = RCNN(num_classes=194, hidden_size=hid, blank_id=None, compute_dtype=torch.bfloat16, enc_dropout_p=0.0)
        m.load_state_dict(recipe_state_dict(O.param_shapes(hid, 194), 5), strict=False)
        m = m.cuda().train()
        m._engine = None
        x, _, tg, tl = synthetic_batch(B, H, W, W // 8, 194, seed=100)
        x = x.cuda()
        m(x)
        m._engine.use_seq = False   # per-step BiLSTM: the persistent sweeps need the whole chip
        time.sleep(12)
        ref = refp = None
        nbad = 0
        for i in range(steps):
            torch.cuda.synchronize()
            probe(buf.ctypes.data, 0)   # reset the launch count
            m.zero_grad(set_to_none=True)
            ctc_loss(m(x), tg, tl).backward()
            torch.cuda.synchronize()
            probe(buf.ctypes.data, buf.size)
            p = buf.reshape(NL, NB, NV).copy()
            g = {k: q.grad.detach().clone() for k, q in m.named_parameters()}
            if ref is None:
                ref, refp = g, p
                continue
            bad = [k for k in g if not torch.equal(g[k], ref[k])]
            din = sorted({int(l) for l, _ in zip(*np.nonzero((p[:, :, :4] != refp[:, :, :4]).any(-1)))})
            dout = sorted({int(l) for l, _ in zip(*np.nonzero((p[:, :, 4:] != refp[:, :, 4:]).any(-1)))})
            if bad or din or dout:
                nbad += 1
            order = {k: n for n, (k, _) in enumerate(m.named_parameters())}
            near = sorted(bad, key=lambda k: order[k])[-4:]   # the differing parameters nearest the loss
            print(f"step {i}: {len(bad)} gradients differ, nearest the loss {near}; se_wgrad launches with "
                  f"different INPUTS {din}, different OUTPUTS {dout}", flush=True)
        print(f"{nbad} of {steps - 1} steps differ", flush=True)
    finally:
        load.kill()
        load.wait()


if __name__ == "__main__":
    main()
