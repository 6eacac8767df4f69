"""Scan hipcc assembly (.s) for the inline-asm MFMA operand hazard the compiler does not pad
(cdna_hip_programming.md §5.7 item 2): a VALU instruction (v_mov, v_accvgpr_write, v_perm, ...) writes a
register that the next few instructions later an MFMA reads as its A or B operand, with fewer than
MIN_WS wait states between them. The compiler pads its own MFMAs (builtins); an MFMA issued from asm
gets nothing, so such a pair reads a stale operand now and then.
    python tools/asm_hazard_scan.py file.s [substring-of-kernel-name] [min_wait_states=2]"""
import re
import sys


def regs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def scan(text, want="", min_ws=2):
    parts = re.split(r"\n(_Z\S+):[^\n]*\n", text)
    out = {}
    for name, body in zip(parts[1::2], parts[2::2]):
        if want not in name:
            continue
        ins = [l.strip() for l in body.split("\n")]
        ins = [l for l in ins if l and not l.startswith((";", ".")) and not l.endswith(":")]
        hz = []
        for k, l in enumerate(ins):
            if not l.startswith("v_mfma"):
                continue
            ops = [o.strip() for o in l.split(" ", 1)[1].split(",")]
            src = regs(ops[1]) | regs(ops[2])
            ws = 0
            for j in range(k - 1, max(-1, k - 8), -1):
                p = ins[j]
                if p.startswith("s_nop"):
                    ws += int(p.split()[1]) + 1
                elif p.startswith("v_") and not p.startswith("v_mfma") and " " in p:
                    if regs(p.split(" ", 1)[1].split(",")[0].strip()) & src and ws < min_ws:
                        hz.append((k, p, l, ws))
                    ws += 1
                else:
                    ws += 1
                if ws >= min_ws:
                    break
        n_mfma = sum(1 for l in ins if l.startswith("v_mfma"))
        out[name] = (n_mfma, hz)
    return out


if __name__ == "__main__":
    res = scan(open(sys.argv[1]).read(), sys.argv[2] if len(sys.argv) > 2 else "",
               int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    tot = 0
    for name, (n, hz) in res.items():
        if hz:
            tot += len(hz)
            print(f"{name[:110]}: {len(hz)} of {n} MFMAs; e.g. {hz[0][1]!r} -> {hz[0][2]!r} ({hz[0][3]} wait states)")
    print(f"kernels scanned {len(res)}, MFMAs {sum(n for n, _ in res.values())}, hazards {tot}")


def scan_asm_loads(text, want=""):
    """asm ds_read destinations (uncounted by hipcc) read by any instruction before an lgkmcnt(0) wait, and
    asm ds_read destinations overwritten while an MFMA issued at most WAR_WIN instructions earlier reads them"""
    WAR_WIN = 4
    parts = re.split(r"\n(_Z\S+):[^\n]*\n", text)
    out = {}
    for name, body in zip(parts[1::2], parts[2::2]):
        if want not in name:
            continue
        lines = [l.strip() for l in body.split("\n")]
        pend, early, war, in_asm, recent = set(), [], [], False, []
        for l in lines:
            if l.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if l.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not l or l.startswith((";", ".")) or l.endswith(":"):
                continue
            if l.startswith("s_waitcnt") and ("lgkmcnt(0)" in l):
                pend = set()
            op = l.split(" ", 1)
            args = [a.strip() for a in op[1].split(",")] if len(op) > 1 else []
            if l.startswith("ds_read") and in_asm:
                d = regs(args[0])
                for (k, srcs) in recent[-WAR_WIN:]:
                    if d & srcs:
                        war.append((l, k))
                pend |= d
                continue
            reads = set()
            for a in args[1:] if args else []:
                reads |= regs(a)
            if l.startswith("v_mfma"):
                reads = regs(args[1]) | regs(args[2])
                recent.append((l, reads))
            if pend & reads:
                early.append(l)
        out[name] = (early, war)
    return out


if __name__ == "__main__" and len(sys.argv) > 4 and sys.argv[4] == "loads":
    for name, (early, war) in scan_asm_loads(open(sys.argv[1]).read(), sys.argv[2]).items():
        if early or war:
            print(f"{name[:110]}: {len(early)} reads of un-waited asm-load registers (e.g. {early[:1]}), "
                  f"{len(war)} WAR overwrites within a few instructions of an MFMA reading them (e.g. {war[:1]})")
    print("asm-load scan done")


def cfg_blocks(lines):
    """basic blocks of one function body (file order) with successor lists"""
    blocks, cur, label_of = [], {"label": None, "ins": []}, {}
    for l in lines:
        if re.match(r"\.LBB\S+:", l):
            if cur["ins"] or cur["label"] is not None:
                blocks.append(cur)
            cur = {"label": l.split(":")[0], "ins": []}
            continue
        cur["ins"].append(l)
        if l[2:].startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = {"label": None, "ins": []}
    if cur["ins"] or cur["label"] is not None:
        blocks.append(cur)
    for i, b in enumerate(blocks):
        if b["label"]:
            label_of[b["label"]] = i
    for i, b in enumerate(blocks):
        succ = []
        last = b["ins"][-1][2:] if b["ins"] else ""
        m = re.match(r"s_c?branch\S*\s+(\.LBB\S+)", last)
        if m and m.group(1) in label_of:
            succ.append(label_of[m.group(1)])
        if not last.startswith(("s_branch", "s_endpgm", "s_setpc")) and i + 1 < len(blocks):
            succ.append(i + 1)
        b["succ"] = succ
    return blocks


def scan_pending_clobber(text, want=""):
    """CFG-aware: registers written by an inline-asm ds_read (hipcc does not count it) stay 'pending' until an
    s_waitcnt lgkmcnt(0); a compiler instruction (outside asm) that WRITES or READS a pending register is a
    hazard — the late LDS return overwrites the compiler's value, or the compiler reads what has not landed
    (cdna_hip_programming.md §5.7 item 1). Returns {kernel: [(instruction, registers)]}."""
    parts = re.split(r"\n(_Z\S+):[^\n]*\n", text)
    out = {}
    for name, body in zip(parts[1::2], parts[2::2]):
        if want not in name:
            continue
        raw = [l.strip() for l in body.split("\n")]
        lines, in_asm = [], False
        for l in raw:   # tag asm lines
            if l.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if l.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not l or (l.startswith((";", ".")) and not re.match(r"\.LBB\S+:", l)):
                continue
            lines.append(("A " if in_asm else "C ") + l if not re.match(r"\.LBB\S+:", l) else l)
        blocks = cfg_blocks(lines)
        entry = [set() for _ in blocks]
        work = list(range(len(blocks)))
        hits = {}
        while work:
            i = work.pop(0)
            pend = set(entry[i])
            for tl in blocks[i]["ins"]:
                kind, l = tl[:1], tl[2:]
                if l.startswith("s_waitcnt") and "lgkmcnt(0)" in l:
                    pend = set()
                    continue
                op = l.split(" ", 1)
                args = [a.strip() for a in op[1].split(",")] if len(op) > 1 else []
                if kind == "A" and l.startswith("ds_read"):
                    pend |= regs(args[0])
                    continue
                if kind == "C" and args:
                    touched = set()
                    for a in args:
                        touched |= regs(a)
                    if touched & pend:
                        hits[l] = sorted(touched & pend)[:4]
            for sidx in blocks[i]["succ"]:
                if not pend <= entry[sidx]:
                    entry[sidx] |= pend
                    if sidx not in work:
                        work.append(sidx)
        out[name] = list(hits.items())
    return out


if __name__ == "__main__" and len(sys.argv) > 4 and sys.argv[4] == "pending":
    res = scan_pending_clobber(open(sys.argv[1]).read(), sys.argv[2])
    n = 0
    for name, h in res.items():
        if h:
            n += 1
            print(f"{name[:120]}: {len(h)} compiler instructions touch un-waited asm-load registers, e.g. {h[:2]}")
    print(f"kernels scanned {len(res)}, with hazards {n}")
