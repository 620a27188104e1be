#!/usr/bin/env python3
"""Per-instruction VALU budget of the fused kernel's task loop (VERDICT r3
"Next" #3: a counter-backed budget of the 4:4:4 kernel).

    python tools/valu_budget.py [--kernel _ZN3hjd13decode_kernelILi0ELi0ELi128E] [--listing rt.s]

Compiles csrc/hjd_runtime.hip to gfx950 assembly (unless --listing is
given), takes the kernel's largest basic block (the six unrolled IDCT rounds
of one task) and splits it into rounds at each round's first coefficient
gather.  Every VALU instruction is classified by what the source says it is
for and priced with the microbenchmarked gfx950 issue costs
(profiles/r03_valu_rates2.txt: add/sub/and/or/xor/ashr ~2.4 cycles per wave64
instruction per SIMD at 4 waves per SIMD, every other op the kernel uses
3.7-4.2, taken as 4).  The colour units (four per task) are counted from
their own blocks.  Prints JSON.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST = ("v_add_u32", "v_sub_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_ashrrev_i32")

ROLE = [  # (opcode prefix, role) -- first match wins
    ("v_dot2_i32_i16", "row butterfly stage 1-2 (one dot2 per exact two-product sum)"),
    ("v_pk_mul_lo_u16", "dequant (two coefficients per op)"),
    ("v_or_b32", "d16 gather pair join / +4 rounding"),
    ("v_mad_i32_i24", "column stage 1-2 products (24-bit)"),
    ("v_mul_i32_i24", "column stage 1-2 products (24-bit)"),
    ("v_mul_lo_u32", "stage 3: 181*(a4 +- a5) (exceeds 24 bits)"),
    ("v_med3_i32", "column clamp [-256,255] (4x-scaled bounds)"),
    ("v_ashrrev_i32", "reference rounding shifts (>>8 row out, >>3 / >>6 column)"),
    ("v_and_b32", "4x-scale masks (& ~3)"),
    ("v_add_lshl_u32", "column odd sums at 4x scale"),
    ("v_lshl_add_u32", "column DC at 4x scale + rounding constant"),
    ("v_lshlrev_b32", "column x4 input scale"),
    ("v_add_u32", "butterfly sums / rounding constants"),
    ("v_sub_u32", "butterfly differences"),
]


def listing(path):
    if path:
        return open(path).read()
    out = os.path.join(tempfile.mkdtemp(prefix="hjd_budget_"), "rt.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{REPO}/include",
                    f"-I{REPO}/ocljpegdecoder_amd/csrc", "-S", "--cuda-device-only",
                    f"{REPO}/ocljpegdecoder_amd/csrc/hjd_runtime.hip", "-o", out], check=True, capture_output=True)
    return open(out).read()


def blocks(text, sub):
    m = next(m for m in re.finditer(r"^(\S+):\s*; @", text, re.M) if sub in m.group(1))
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    out, cur, name = [], [], "entry"
    for line in body.splitlines():
        lm = re.match(r"^(\.LBB\S+):", line)
        if lm:
            out.append((name, cur))
            name, cur = lm.group(1), []
            continue
        s = line.split(";", 1)[0].strip()
        if s:
            cur.append(s)
    out.append((name, cur))
    return m.group(1), out


def cost(op):
    return 2.4 if op.startswith(FAST) else 4.0


def role(op):
    return next((r for p, r in ROLE if op.startswith(p)), "other (addresses, colour unit merged into the block)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="_ZN3hjd13decode_kernelILi0ELi0ELi128E")
    ap.add_argument("--listing", default="")
    a = ap.parse_args()
    name, bl = blocks(listing(a.listing), a.kernel)
    big_name, big = max(bl, key=lambda b: sum(1 for i in b[1] if i.startswith("v_")))
    # rounds start at each round's first gather load
    starts = [i for i, ins in enumerate(big) if ins.startswith(("ds_read_u16_d16_hi", "ds_read_u16 ")) and
              (i == 0 or not big[i - 1].startswith("ds_read_u16"))]
    rounds = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(big)
        ops = [ins.split()[0] for ins in big[s:e] if ins.startswith("v_")]
        rounds.append(ops)
    full = [r for r in rounds[1:-1]] or rounds   # interior rounds: one whole round each
    r = full[len(full) // 2]
    by_role = collections.defaultdict(lambda: [0, 0.0])
    for op in r:
        by_role[role(op)][0] += 1
        by_role[role(op)][1] += cost(op)
    colour = [b for b in bl if sum(1 for i in b[1] if i.startswith("v_mul_i32_i24_sdwa")) >= 8 and b[0] != big_name]
    res = {"kernel": name, "loop_block": big_name,
           "loop_block_valu": sum(1 for i in big if i.startswith("v_")),
           "loop_block_lds": sum(1 for i in big if i.startswith("ds_")),
           "rounds_found": len(rounds), "valu_per_round": [len(x) for x in rounds],
           "one_interior_round": {"valu": len(r), "weighted_cycles": round(sum(cost(o) for o in r), 1),
                                  "by_role": {k: {"ops": v[0], "cycles": round(v[1], 1)} for k, v in
                                              sorted(by_role.items(), key=lambda kv: -kv[1][1])},
                                  "opcodes": dict(collections.Counter(r).most_common())},
           "colour_blocks": {b[0]: {"valu": sum(1 for i in b[1] if i.startswith("v_")),
                                    "weighted_cycles": round(sum(cost(i.split()[0]) for i in b[1]
                                                                 if i.startswith("v_")), 1)} for b in colour},
           "cost_model": "2.4 cycles: v_add/sub/and/or/xor_b32, v_ashrrev_i32; 4.0: every other VALU op "
                         "(profiles/r03_valu_rates2.txt)"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
