"""Per-dispatch HBM bytes of the conv kernels from tools/gpu_pmc_kbench.sh, in dispatch order, with the
kernel family; 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md gfx950 correction). Prints one line per
dispatch (kbench runs each op 3 + 2 times per layer: warm-up then timed).
    python tools/pmc_kbench_summary.py gpurun_out/pmck_F gpurun_out/pmck_W"""
import csv
import glob
import sys
from collections import defaultdict


def read(d, ctr):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    out = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        did = int(r["Dispatch_Id"])
        out[did] += float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    return out, names


f, names = read(sys.argv[1], "FETCH_SIZE")
w, _ = read(sys.argv[2], "WRITE_SIZE")
for did in sorted(f):
    n = names[did]
    if not any(k in n for k in ("gemm", "halo", "wgrad_reduce")):
        continue
    fam = ("fwd" if "FwdA" in n else "dgrad" if "Dgrad" in n else "wgrad" if "Wgrad" in n or "wgrad" in n
           else "halo" if "halo" in n else "gemm")
    print(f"{did:5d} {fam:6s} fetch {2 * f[did] / 1024:8.1f} MB  write {w.get(did, 0) / 1024:7.1f} MB  {n[:70]}")
