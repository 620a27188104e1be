#!/usr/bin/env python3
"""Opcode histogram of one kernel in a hipcc -S (gfx950) listing.

usage: isa_hist.py LISTING.s SUBSTRING [--blocks]

SUBSTRING selects the kernel by its mangled name.  --blocks also prints each
basic block's VALU/LDS/VMEM counts, which is how the per-task loop body is
found (the largest block(s) inside the persistent loop).
"""
import collections
import re
import sys


def kernel_body(text, sub):
    for m in re.finditer(r"^(\S+):\s*; @", text, re.M):
        if sub in m.group(1):
            end = text.find(".Lfunc_end", m.end())
            return m.group(1), text[m.end():end]
    raise SystemExit(f"no kernel matching {sub!r}")


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return None


def main():
    text = open(sys.argv[1]).read()
    name, body = kernel_body(text, sys.argv[2])
    print(name)
    ops = collections.Counter()
    blocks = []
    cur = [None, collections.Counter()]
    for line in body.split("\n"):
        if re.match(r"^\.LBB\S+:", line):
            blocks.append(cur)
            cur = [line.split(":")[0], collections.Counter()]
            continue
        if not line.startswith("\t") or line.startswith("\t."):
            continue
        op = line.split()[0]
        k = classify(op)
        if k:
            ops[op] += 1
            cur[1][k] += 1
    blocks.append(cur)
    kinds = collections.Counter()
    for op, n in ops.items():
        kinds[classify(op)] += n
    print(dict(kinds))
    print([(o, n) for o, n in ops.most_common() if o.startswith("v_")][:45])
    if "--blocks" in sys.argv:
        for lbl, c in blocks:
            if sum(c.values()) >= 20:
                print(f"{lbl}: {dict(c)}")


if __name__ == "__main__":
    main()
