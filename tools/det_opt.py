"""Co-scheduling determinism probe under a tuning switch: a victim model's bf16 train step beside this library's
own step on a side stream (tests/test_gpu_determinism.py's set-up), counting the iterations whose gradients
differ from the idle-device result, per option value.   python tools/det_opt.py KEY V0,V1 [ITERS]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("rcnn-ocr_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))
from crnn_hip import _lib as L  # noqa: E402
from test_gpu_determinism import _bench_model, _grads  # noqa: E402


def main():
    key, vals = int(sys.argv[1]), [int(v) for v in sys.argv[2].split(",")]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    for v in vals:
        L.call("crnn_set_option", key, v)
        vm, vx, vtg, vtl = _bench_model(5, True)
        am, ax, atg, atl = _bench_model(6, False)
        _grads(vm, vx, vtg, vtl)
        torch.cuda.synchronize()
        vref = {k: p.grad.detach().clone() for k, p in vm.named_parameters()}
        _grads(am, ax, atg, atl)
        torch.cuda.synchronize()
        aref = {k: p.grad.detach().clone() for k, p in am.named_parameters()}
        side = torch.cuda.Stream()
        nv = na = 0
        names = {}
        for i in range(iters):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    _grads(am, ax, atg, atl)
            _grads(vm, vx, vtg, vtl)
            torch.cuda.synchronize()
            vbad = [k for k, p in vm.named_parameters() if not torch.equal(p.grad, vref[k])]
            abad = [k for k, p in am.named_parameters() if not torch.equal(p.grad, aref[k])]
            nv += bool(vbad)
            na += bool(abad)
            for k in vbad + abad:
                names[k] = names.get(k, 0) + 1
        print(f"option {key}={v}: victim differs in {nv} of {iters} iterations, side model in {na}; "
              f"gradients {sorted(names.items(), key=lambda t: -t[1])[:6]}", flush=True)
        del vm, am
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
