"""Sum rocprofv3 --pmc counters per kernel (name substring filter) from a counter_collection.csv.
    python tools/pmc_kernels.py <dir> [substring]"""
import csv
import sys
from collections import defaultdict


def main(d, sub=""):
    tot = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            if sub not in k:
                continue
            k = k[:90]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    for k, cs in tot.items():
        m = len(n[k])
        print(f"{k}  (dispatches {m})")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {v / m:16.0f} per dispatch")


if __name__ == "__main__":
    main(*sys.argv[1:])
