"""Summarize tools/gpu_pmc_gemm.sh: per kernel family (crnn gemm / hipBLASLt Cijk), the SQ counter
ratios of its largest dispatches.   python tools/pmc_gemm_summary.py gpurun_out/pmcg_0 [...]"""
import csv
import glob
import sys
from collections import defaultdict


def main(dirs):
    for d in dirs:
        f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
        if not f:
            print(d, "no csv"); continue
        rows = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f[0])):
            did = int(r["Dispatch_Id"])
            rows[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = r["Kernel_Name"]
        fam = defaultdict(lambda: defaultdict(float))
        for did, cs in rows.items():
            n = names[did]
            k = "crnn4w" if "gemm4w" in n else "crnn8w" if "gemm256" in n else "hipblaslt" if "Cijk" in n else None
            if k is None or cs["SQ_WAVE_CYCLES"] < 1e8:   # large dispatches only
                continue
            for c, v in cs.items():
                fam[k][c] += v
            fam[k]["n"] += 1
        print(d)
        for k, c in fam.items():
            w = c["SQ_WAVE_CYCLES"]
            print(f"  {k:10s} n={int(c['n']):3d} wait_any {c['SQ_WAIT_ANY'] / w:.3f} wait_inst {c['SQ_WAIT_INST_ANY'] / w:.3f}"
                  f" active_inst {c['SQ_ACTIVE_INST_ANY'] / w:.3f} lds_conflict/lds_active "
                  f"{c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f} mfma_busy/wave_cyc "
                  f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / w:.3f} insts_lds/wave_cyc {c['SQ_INSTS_LDS'] / w:.4f}")


if __name__ == "__main__":
    main(sys.argv[1:])
