"""Packed-fp32 WAR scan: in a device assembly listing (hipcc --cuda-device-only
-S, built WITH packed fp32 ops, i.e. csrc/Makefile NOPK=), find every v_pk_{add,mul,fma}_f32 whose SOURCE VGPRs are
overwritten by a later LDS or memory load (ds_* / buffer_load / global_load return) within the next WINDOW
instructions, with no s_nop between them. Such a pair is race-free only if the packed instruction has read its
sources before the load's data returns.
    python tools/pk_war_scan.py bn_pk.s [WINDOW]"""
import re
import sys
from collections import Counter

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def regs(tok):
    out = set()
    for m in REG.finditer(tok):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main():
    path = sys.argv[1]
    win = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    lines = open(path).read().split("\n")
    fn, per_fn, examples = None, Counter(), {}
    insts = []
    for l in lines:
        m = re.match(r"^(_Z\w+):", l)
        if m:
            fn = m.group(1)
            insts = []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        insts.append(t)
        # check the instruction WINDOW back: a v_pk whose sources this load overwrites
        op = t.split()[0]
        if op.startswith(("ds_read", "ds_bpermute", "ds_permute", "ds_swizzle", "buffer_load", "global_load")):
            dst = regs(t.split()[1].rstrip(","))
            for back in range(2, min(win + 2, len(insts) + 1)):
                p = insts[-back]
                if p.startswith("s_nop") or p.startswith("s_waitcnt"):
                    break
                if p.startswith("v_pk_") and "_f32" in p.split()[0]:
                    ops = [x.rstrip(",") for x in p.split()[1:4]]
                    srcs = set().union(*(regs(x) for x in ops[1:]))
                    hit = dst & srcs
                    if hit:
                        per_fn[fn] += 1
                        examples.setdefault(fn, (p, t))
    total = sum(per_fn.values())
    print(f"{path}: {total} packed-fp32 source -> load-destination WAR pairs within {win} instructions, "
          f"{len(per_fn)} kernels")
    for f, n in per_fn.most_common(12):
        print(f"  {n:4d}  {f[:90]}")
        print(f"        e.g. {examples[f][0]}  ->  {examples[f][1]}")


if __name__ == "__main__":
    main()
