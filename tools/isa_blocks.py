#!/usr/bin/env python3
"""Basic blocks of one kernel in a hipcc device assembly (.s) file, with
instruction counts by class, loops (back edges) and the hot path's counts.

    python3 tools/isa_blocks.py FILE.s KERNEL_SYMBOL [--blocks]

Classes: valu (v_*), salu (s_* scalar ALU), smem (s_load/s_buffer_load),
vmem (global_/buffer_/flat_), lds (ds_*), wait (s_waitcnt), nop (s_nop),
branch (s_branch/s_cbranch*), other.  Used to read where a frame's issue
slots go (one wave per SIMD issues one instruction per cycle-slot)."""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks_of(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], {"label": sym, "ins": [], "line": start + 1}
    for i in range(start + 1, end):
        l = lines[i].split(";")[0].rstrip()
        if not l.strip():
            continue
        m = re.match(r"^(\.LBB\w+|\.L\w+):", l)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "ins": [], "line": i + 1}
            continue
        if l.startswith("\t.") or l.startswith("."):
            continue
        toks = l.split()
        if not toks:
            continue
        cur["ins"].append((toks[0], " ".join(toks[1:]), i + 1))
        if toks[0] in ("s_branch",) or toks[0].startswith("s_endpgm"):
            blocks.append(cur)
            cur = {"label": None, "ins": [], "line": i + 2}
    blocks.append(cur)
    return [b for b in blocks if b["ins"] or b["label"]]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    bl = blocks_of(path, sym)
    idx = {b["label"]: k for k, b in enumerate(bl) if b["label"]}
    total = Counter()
    for b in bl:
        b["cnt"] = Counter(classify(op) for op, _, _ in b["ins"])
        total.update(b["cnt"])
    print("kernel total:", dict(total))
    loops = []
    for k, b in enumerate(bl):
        for op, arg, ln in b["ins"]:
            if classify(op) == "branch" and arg.startswith(".L") and arg in idx and idx[arg] <= k:
                loops.append((idx[arg], k, op, ln))
    for a, z, op, ln in loops:
        c = Counter()
        for b in bl[a:z + 1]:
            c.update(b["cnt"])
        print(f"loop {bl[a]['label']} (line {bl[a]['line']}) .. block {z} ({op} at line {ln}): "
              f"{z - a + 1} blocks, {dict(c)}")
    if "--blocks" in sys.argv:
        for k, b in enumerate(bl):
            print(k, b["label"], b["line"], dict(b["cnt"]))


if __name__ == "__main__":
    main()
