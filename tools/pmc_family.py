"""Per-family split of the conv launches' measured HBM traffic from the same rocprofv3
PMC passes as tools/pmc_traffic.py: mean bytes per launch of each GEMM / kernel family over the traced steps,
with the same correction (2 x FETCH_SIZE + WRITE_SIZE).   python tools/pmc_family.py gpurun_out/pmc_1 gpurun_out/pmc_2"""
import re
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_traffic import read  # noqa: E402

FAMILIES = [
    ("wgrad (256-row GEMM, fp32 split-K slabs)", re.compile(r"gemm256.*WgradAF|gemm4w.*WgradAF")),
    ("wgrad slab reduce", re.compile(r"wgrad_reduce")),
    ("fwd 3x3 s1 (W-halo)", re.compile(r"gemm256hw_kernel.*FwdEpi")),
    ("dgrad 3x3 s1 (W-halo)", re.compile(r"gemm256hw_kernel.*Dgrad")),
    ("fwd (256-row, K-tile images)", re.compile(r"gemm256_kernel.*FwdA.*FwdEpi")),
    ("dgrad + BN reduce (256-row)", re.compile(r"gemm256_kernel.*DgradBnEpi")),
    ("dgrad (256-row)", re.compile(r"gemm256_kernel.*DgradEpi")),
    ("strided dgrad class groups", re.compile(r"dgrad_cls_group")),
    ("stem halo fwd / dgrad", re.compile(r"halo3x3_kernel")),
    ("stem halo wgrad", re.compile(r"halo3x3_wgrad")),
    ("128-row / small conv GEMMs", re.compile(r"gemm_kernel.*(FwdA|DgradA|WgradA)")),
]


def main(p_fetch, p_write):
    acc = defaultdict(lambda: defaultdict(float))
    for path, ctr in ((p_fetch, "FETCH_SIZE"), (p_write, "WRITE_SIZE")):
        rows, names = read(path)
        for did, cs in rows.items():
            for fam, rx in FAMILIES:
                if rx.search(names[did]):
                    acc[fam][ctr] += cs[ctr] * 1024.0
                    acc[fam]["n_" + ctr] += 1
                    break
    print(f"{'family':45s} {'launches':>8s} {'read MB':>9s} {'write MB':>9s} {'HBM MB/launch':>14s}")
    for fam, _ in FAMILIES:
        a = acc.get(fam)
        if not a or not a["n_FETCH_SIZE"]:
            continue
        n = a["n_FETCH_SIZE"]
        rd = 2 * a["FETCH_SIZE"] / n / 1e6
        wr = a["WRITE_SIZE"] / max(1, a["n_WRITE_SIZE"]) / 1e6
        print(f"{fam:45s} {int(n):8d} {rd:9.1f} {wr:9.1f} {rd + wr:14.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
