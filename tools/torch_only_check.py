"""Cross-process counterpart of tools/cohab_check.py: this process runs only torch work (bf16 GEMMs,
fp32 reductions, an elementwise chain) and checks every result bit for bit against its first run,
while another process (the caller's choice, e.g. bench.py) loads the same GPU.
    python tools/torch_only_check.py [seconds]"""
import sys
import time

import torch

from cohab_check import side_work


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    g = torch.Generator().manual_seed(3)
    a = torch.randn(4096, 4096, generator=g).cuda().bfloat16()
    b = torch.randn(4096, 4096, generator=g).cuda().bfloat16()
    x = torch.randn(16384, 4096, generator=g).cuda()
    ref = [t.clone() for t in side_work(a, b, x)]
    torch.cuda.synchronize()
    t0, n, bad = time.time(), 0, 0
    while time.time() - t0 < secs:
        outs = [side_work(a, b, x) for _ in range(8)]
        torch.cuda.synchronize()
        nd = sum(1 for o in outs for t, r in zip(o, ref) if not torch.equal(t, r))
        n += 1
        bad += nd > 0
        if nd or n % 20 == 0:
            print(f"round {n}: {nd} of {len(outs) * 4} results differ", flush=True)
    print(f"{bad} of {n} rounds with a differing result", flush=True)


if __name__ == "__main__":
    main()
