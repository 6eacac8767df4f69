"""Per-kernel-name averages of the counters in a rocprofv3 --pmc CSV directory (kernel-trace run).
    python tools/pmc_sq_summary.py DIR [name-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if sub not in n:
        continue
    per[n[:90]][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[n[:90]].add(r["Dispatch_Id"])
for n, cs in per.items():
    k = len(cnt[n])
    print(f"{k:3d} x {n}")
    print("     " + "  ".join(f"{c}={v / k:.4g}" for c, v in sorted(cs.items())))
