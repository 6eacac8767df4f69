"""GPU idle time between kernels per training step, from a rocprofv3 --kernel-trace database:
steps are delimited by the optimizer kernel; prints per-step span, idle total and the largest
bubbles with the kernels on both sides.   python tools/step_gaps.py run_results.db"""
import sqlite3
import sys

import numpy as np


def main(path):
    db = sqlite3.connect(path)
    cur = db.cursor()

    def table(prefix):
        return [r[0] for r in cur.execute(f"select name from sqlite_master where type='table' and name like '{prefix}%'")][0]

    kd, ks = table("rocpd_kernel_dispatch"), table("rocpd_info_kernel_symbol")
    names = {r[0]: r[1] for r in cur.execute(f"select id, kernel_name from {ks}")}
    rows = list(cur.execute(f"select start, end, kernel_id from {kd} order by start"))
    marks = [i for i, r in enumerate(rows) if "adam" in names[r[2]] or "sgd_kernel" in names[r[2]]]
    worst = []
    for a, b in zip(marks[:-1], marks[1:]):
        seg = rows[a:b + 1]
        end, gaps = seg[0][1], []
        for i in range(1, len(seg)):
            if seg[i][0] > end:
                gaps.append((seg[i][0] - end, names[seg[i - 1][2]][:50], names[seg[i][2]][:50]))
            end = max(end, seg[i][1])
        g = np.array([x[0] for x in gaps]) if gaps else np.zeros(1)
        print(f"step: span {(seg[-1][1] - seg[0][1]) / 1e3:8.0f} us, kernels {len(seg) - 1}, idle {g.sum() / 1e3:6.0f} us "
              f"({len(gaps)} gaps, {(g > 3000).sum()} over 3 us)")
        worst = gaps
    for g, x, y in sorted(worst, key=lambda t: -t[0])[:8]:
        print(f"  last step: {g / 1e3:7.1f} us idle between {x} and {y}")


if __name__ == "__main__":
    main(sys.argv[1])
