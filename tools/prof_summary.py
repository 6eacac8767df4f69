"""Kernel-time summary from a rocprofv3 SQLite result (rocpd schema): per kernel name,
calls, total / average duration, share. Usage: prof_summary.py <run_results.db> [steps]"""
import sqlite3
import sys


def summary(db, steps=None, top=40):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels group by name").fetchall()
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    out = [f"total kernel time {tot / 1e6:.3f} ms" + (f"  ({tot / 1e6 / steps:.3f} ms/step over {steps} steps)" if steps else "")]
    out.append(f"{'calls':>7} {'total_ms':>9} {'avg_us':>9} {'pct':>6}  kernel")
    for name, n, t, a in rows[:top]:
        out.append(f"{n:7d} {t / 1e6:9.3f} {a / 1e3:9.2f} {100 * t / tot:6.2f}  {name[:150]}")
    return "\n".join(out)




def markdown(db, steps, title, top=45):
    """per-step markdown table (the form committed under profiles/)."""
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels group by name").fetchall()
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    out = [f"# {title}", "", f"Total kernel time per step: {tot / 1e6 / steps:.2f} ms ({steps} traced steps).", "",
           "| ms/step | launches/step | avg us | kernel |", "|---:|---:|---:|---|"]
    for name, n, t, a in rows[:top]:
        out.append(f"| {t / 1e6 / steps:.3f} | {n / steps:.1f} | {a / 1e3:.1f} | `{name[:140]}` |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[1] == "--md":
        print(markdown(sys.argv[2], int(sys.argv[3]), " ".join(sys.argv[4:]) or "rocprofv3 kernel summary"))
    else:
        print(summary(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None))
