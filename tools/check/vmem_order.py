#!/usr/bin/env python3
"""Static checks of decode_kernel's coefficient prefetch in the BUILT library.

    python tools/check/vmem_order.py [path/to/libhjd.so]

1. Counted loop-head wait (the performance property).  The full-strip loop
   of decode_kernel (csrc/hjd_kernels.hpp) issues the next strip's
   coefficient loads (`global_load_dwordx4 ... nt`), then this strip's IDCT,
   colour math and output stores.  The wait for those loads at the next loop
   head must be `s_waitcnt vmcnt(S)`, S = the stores a strip issues after them
   (4 at 4:4:4, 8 at 4:2:0), so that the stores drain while the next strip
   computes.  The compiler's waitcnt pass only emits that count when every
   control-flow path from the loads to the loop head issues the S stores;
   one path with fewer (an edge-strip branch, stores inside a both-sided
   branch) turns it into vmcnt(0).  This script reports the wait in front of
   each kernel's coefficient staging (the run of six ds_write_b128) and fails
   if a 4:4:4/4:2:0 product kernel waits vmcnt(0) in its loop.

2. Prefetch registers untouched until covered (the correctness property,
   independent of the compiler's own analysis).  On every control-flow path
   from a prefetch load, its destination VGPRs may not be read, copied or
   overwritten before an `s_waitcnt vmcnt(j)` that covers it: j <= the vector
   memory instructions issued after that load on the path (a wave's vector
   memory operations are counted in order -- LLVM's own gfx950 model).  A
   forward data-flow analysis over each kernel's control-flow graph (built
   from the disassembly's branch targets) tracks, per in-flight VGPR, the
   fewest younger vector memory instructions over all paths.

Exit status 1 on any violation.
"""
from __future__ import annotations

import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from d16_order import DEFAULT_LIB, _regs, disassemble  # noqa: E402

_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<([^>+]+)(?:\+0x([0-9a-f]+))?>")
_VMEM = ("global_", "buffer_", "scratch_", "flat_")
KERNEL_SUBSTR = "decode_kernel"


def _is_prefetch(mn: str, ops: str) -> bool:
    return mn == "global_load_dwordx4" and re.search(r"\bnt\b", ops) is not None


def _functions(text: str):
    """{name: [(addr, mnemonic, operands, branch_target_or_None)]} for decode kernels."""
    funcs, cur, start = {}, None, 0
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            start, name = int(m.group(1), 16), m.group(2)
            cur = funcs.setdefault(name, []) if KERNEL_SUBSTR in name else None
            continue
        if cur is None:
            continue
        body, _, comment = line.partition("//")
        body = body.strip()
        if not body or body.endswith(":"):
            continue
        a = _ADDR.search(line)
        if not a:
            continue
        parts = body.split(None, 1)
        mn, ops = parts[0], (parts[1] if len(parts) > 1 else "")
        tgt = None
        if mn.startswith(("s_branch", "s_cbranch")):
            t = _TARGET.search(comment)
            if t:
                tgt = start + (int(t.group(2), 16) if t.group(2) else 0)
        cur.append((int(a.group(1), 16), mn, ops, tgt))
    return funcs


def _successors(insts, i, index_of):
    addr, mn, ops, tgt = insts[i]
    nxt = [i + 1] if i + 1 < len(insts) else []
    if mn == "s_endpgm":
        return []
    if mn == "s_branch":
        return [index_of[tgt]]
    if mn.startswith("s_cbranch"):
        return [index_of[tgt]] + nxt
    if mn.startswith(("s_setpc", "s_swappc")):
        raise ValueError(f"indirect branch at {addr:#x}")
    return nxt


def _join(a, b):
    """States are frozensets of (vgpr, younger VMEM ops since its load) --
    per register, like the compiler's own score brackets; join keeps every
    pending register with its fewest younger ops over the joining paths."""
    if a is None:
        return b
    if b is None:
        return a
    d = dict(a)
    for r, n in b:
        d[r] = min(n, d.get(r, n))
    return frozenset(d.items())


def _transfer(state, mn, ops, on_violation):
    pend = dict(state) if state else {}
    if _is_prefetch(mn, ops):
        dst, src = ops.split(",", 1)
        if _regs(src) & pend.keys() or _regs(dst) & pend.keys():
            on_violation()
        pend = {r: n + 1 for r, n in pend.items()}
        pend.update((r, 0) for r in _regs(dst))
        return frozenset(pend.items())
    if not pend:
        return None
    if mn == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", ops)
        if m:   # loads with >= j younger VMEM ops are complete once vmcnt <= j
            j = int(m.group(1))
            pend = {r: n for r, n in pend.items() if n < j}
        return frozenset(pend.items()) if pend else None
    if _regs(ops) & pend.keys():
        on_violation()
    if mn.startswith(_VMEM):
        pend = {r: n + 1 for r, n in pend.items()}
    return frozenset(pend.items())


def check_function(name, insts):
    """(number of prefetch loads, [violation strings]) for one kernel."""
    index_of = {a: i for i, (a, *_r) in enumerate(insts)}
    n_pf = sum(1 for _a, mn, ops, _t in insts if _is_prefetch(mn, ops))
    if n_pf == 0:
        return 0, []
    state_in = [None] * len(insts)
    seen = [False] * len(insts)
    work = [0]
    seen[0] = True
    errors = {}
    while work:
        i = work.pop()
        addr, mn, ops, _t = insts[i]

        def bad(i=i, addr=addr, mn=mn, ops=ops):
            errors[i] = f"{name}: `{mn} {ops}` at {addr:#x} touches a prefetch VGPR still in flight"

        out = _transfer(state_in[i], mn, ops, bad)
        for j in _successors(insts, i, index_of):
            new = _join(state_in[j], out)
            if not seen[j] or new != state_in[j]:
                seen[j] = True
                state_in[j] = new
                work.append(j)
    return n_pf, [errors[k] for k in sorted(errors)]


def check_text(text: str):
    """(prefetch loads checked, kernels checked, [violations])."""
    n, k, errors = 0, 0, []
    for name, insts in _functions(text).items():
        c, e = check_function(name, insts)
        if c:
            n, k = n + c, k + 1
        errors += e
    return n, k, errors


# product kernels of the benchmarked shapes (sampling 0/1, q16 input, variant
# bits 0-1 and the d16 gather): their full-strip loop must wait counted
_COUNTED = re.compile(r"decode_kernelILi([01])ELi0ELi(0|1|2|3|128|129)EE")


def staging_waits(name, insts):
    """vmcnt of the wait in front of each coefficient staging (six ds_write_b128)."""
    out = []
    for i, (_a, mn, _o, _t) in enumerate(insts):
        if mn != "ds_write_b128" or (i and insts[i - 1][1] == "ds_write_b128"):
            continue
        if sum(1 for x in insts[i:i + 8] if x[1] == "ds_write_b128") < 6:
            continue
        for j in range(i - 1, max(-1, i - 40), -1):
            mj, oj = insts[j][1], insts[j][2]
            if mj == "s_waitcnt" and "vmcnt" in oj:
                out.append(int(re.search(r"vmcnt\((\d+)\)", oj).group(1)))
                break
            if mj.startswith(("s_branch", "s_cbranch")):
                break
    return out


def check_counted(funcs):
    """([(kernel, waits)], [violations]) for the counted loop-head wait."""
    rows, errors = [], []
    for name, insts in funcs.items():
        if not _COUNTED.search(name):
            continue
        w = staging_waits(name, insts)
        rows.append((name, w))
        if not any(x > 0 for x in w):
            errors.append(f"{name}: no counted vmcnt wait before the loop's coefficient staging (waits {w})")
    return rows, errors


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    text = disassemble(lib)
    rows, errors = check_counted(_functions(text))
    for name, w in rows:
        print(f"{name[:60]}: staging waits vmcnt{w}")
    n, k, e2 = check_text(text)
    errors += e2
    for e in errors:
        print(e)
    print(f"{len(rows)} product kernels checked for a counted loop-head wait; {n} prefetch loads in {k} decode "
          f"kernels checked for uses before a covering wait; {len(errors)} violations")
    sys.exit(1 if errors or n == 0 or not rows else 0)


if __name__ == "__main__":
    main()
