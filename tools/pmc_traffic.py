"""Per-launch HBM traffic (and MFMA busy share) of the hot kernels from rocprofv3 PMC passes
(tools/gpu_pmc.sh): FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is doubled for the wide 16-B/lane
streaming reads these kernels issue (MI355X_MICROARCH.md § HBM: gfx950 tallies 128-B requests at
64 B). Writes the JSON bench.py reports as roofline.traffic.
    python tools/pmc_traffic.py gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_3 > profiles/<tag>_pmc_traffic.json"""
import csv
import json
import re
import sys
from collections import defaultdict

CONV = re.compile(r"(FwdA|DgradA|DgradClsA|WgradA)")


def kind(name):
    if "lstm_seq_fwd" in name:
        return "lstm_fwd"
    if "lstm_seq_bwd" in name:
        return "lstm_bwd"
    if ("gemm" in name and CONV.search(name)) or "halo3x3" in name or "dgrad_cls_group" in name:
        return "conv"
    if "wgrad_reduce" in name:   # the split-K slab reduce: part of its wgrad launch (bench.py times both)
        return "conv_aux"
    return None


def read(d):
    rows = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    names = {}
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            did = int(r["Dispatch_Id"])
            rows[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = r["Kernel_Name"]
    return rows, names


def main(p_fetch, p_write, p_mfma):
    sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "rcnn-ocr_amd"))
    from crnn_hip._lib import source_hash
    out = {"source": "rocprofv3 --pmc passes over `bench.py --steps 3 --warmup 1` (tools/gpu_pmc.sh)",
           "source_hash": source_hash(),
           "correction": "hbm = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane streaming reads) + WRITE_SIZE"}
    acc = defaultdict(lambda: defaultdict(float))
    for path, ctr in ((p_fetch, "FETCH_SIZE"), (p_write, "WRITE_SIZE")):
        rows, names = read(path)
        for did, cs in rows.items():
            k = kind(names[did])
            if k:
                acc[k][ctr] += cs[ctr] * 1024.0
                acc[k]["n_" + ctr] += 1
    rows, names = read(p_mfma)
    for did, cs in rows.items():
        k = kind(names[did])
        if k:
            acc[k]["mfma_busy"] += cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            acc[k]["gui_active"] += cs.get("GRBM_GUI_ACTIVE", 0.0)
    aux = acc.pop("conv_aux", None)
    if aux is not None and "conv" in acc:   # per conv launch as bench.py counts them (reduce included)
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            acc["conv"][ctr] += aux[ctr]
    for k, a in acc.items():
        n = max(1.0, a["n_FETCH_SIZE"])
        fetch = a["FETCH_SIZE"] / n
        write = a["WRITE_SIZE"] / max(1.0, a["n_WRITE_SIZE"])
        out[k] = {"launches_sampled": int(n), "fetch_bytes_per_launch_raw": fetch,
                  "write_bytes_per_launch": write, "hbm_bytes_per_launch": 2 * fetch + write,
                  # MFMA busy cycles over (GUI-active cycles / 8 XCDs x 1024 SIMDs): share of the
                  # matrix pipes busy while the kernels ran (SQ_VALU_MFMA_BUSY_CYCLES counts per SIMD)
                  "mfma_busy_frac": (a["mfma_busy"] / (a["gui_active"] / 8.0 * 1024.0)) if a["gui_active"] else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
