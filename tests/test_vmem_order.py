"""decode_kernel's coefficient prefetch, checked on the built library
(DESIGN.md s13.8).  The full-strip loop must wait for the next strip's
coefficient loads with a counted vmcnt (4 at 4:4:4, 8 at 4:2:0), so that the
previous strip's stores stay in flight; and no prefetch register may be
touched before a covering wait.  tools/check/vmem_order.py checks both in the
gfx950 code objects of libhjd.so; the synthetic listings below (objdump
format) show that it catches each way either property can break."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "check"))
import d16_order  # noqa: E402
import vmem_order  # noqa: E402

LIB = os.path.join(REPO, "ocljpegdecoder_amd", "lib", "libhjd.so")
NAME = "_ZN3hjd13decode_kernelILi1ELi0ELi0EEEvPKvPKiPKNS_8FrameDevEilPhll"


def listing(body_lines, name=NAME):
    """objdump-style text: one instruction per line with its address comment."""
    out, addr = [f"0000000000001000 <{name}>:"], 0x1000
    for ins in body_lines:
        ins, _, tgt = ins.partition(" <")   # objdump prints a branch target after the encoding
        out.append(f"\t{ins:<58}// {addr:012X}: 00000000" + (f" <{tgt}" if tgt else ""))
        addr += 8
    return "\n".join(out) + "\n"


def br(op, target_index, name=NAME):
    """branch to the instruction at target_index (8 bytes per instruction)."""
    return f"{op} 0 <{name}+0x{8 * target_index:x}>"


# loop: stage (wait, six ds_write_b128) -> prefetch next -> two stores -> back
LOOP = [
    "s_waitcnt vmcnt(2)",                                   # 0  loop head: counted
    "ds_write_b128 v40, v[2:5]",                            # 1
    "ds_write_b128 v40, v[6:9] offset:1152",                # 2
    "ds_write_b128 v40, v[10:13] offset:2304",              # 3
    "ds_write_b128 v40, v[14:17] offset:3456",              # 4
    "ds_write_b128 v40, v[18:21] offset:4608",              # 5
    "ds_write_b128 v40, v[22:25] offset:5760",              # 6
    "global_load_dwordx4 v[2:5], v26, s[2:3] nt",           # 7  prefetch
    "global_load_dwordx4 v[6:9], v26, s[2:3] offset:1024 nt",
    "global_load_dwordx4 v[10:13], v26, s[2:3] offset:2048 nt",
    "global_load_dwordx4 v[14:17], v26, s[2:3] offset:3072 nt",
    "global_load_dwordx4 v[18:21], v26, s[4:5] nt",
    "global_load_dwordx4 v[22:25], v26, s[4:5] offset:1024 nt",
    "v_add_u32_e32 v30, v31, v32",                          # 13 (the strip's math)
    "global_store_dwordx4 v33, v[34:37], s[6:7] nt",        # 14
    "global_store_dwordx4 v33, v[34:37], s[6:7] offset:512 nt",
    "s_cmp_lg_u32 s8, 0",                                   # 16
    br("s_cbranch_scc1", 0),                                # 17
    "s_endpgm",                                             # 18
]


def test_checker_accepts_counted_loop():
    funcs = vmem_order._functions(listing(LOOP))
    rows, errors = vmem_order.check_counted(funcs)
    assert rows == [(NAME, [2])] and errors == []
    n, k, errors = vmem_order.check_text(listing(LOOP))
    assert (n, k, errors) == (6, 1, [])


def test_checker_rejects_vmcnt0_loop_head():
    body = [("s_waitcnt vmcnt(0)" if i == 0 else x) for i, x in enumerate(LOOP)]
    rows, errors = vmem_order.check_counted(vmem_order._functions(listing(body)))
    assert rows == [(NAME, [0])] and errors


@pytest.mark.parametrize("mutate, what", [
    (lambda b: b[:14] + b[15:17] + [br("s_cbranch_scc1", 0)] + b[18:], "one store fewer than the count"),
    (lambda b: b[:13] + ["v_mov_b32_e32 v50, v25"] + b[14:], "copy of a prefetch register"),
    (lambda b: b[:13] + [br("s_cbranch_vccz", 16)] + b[14:], "path around the stores"),
    (lambda b: b[:13] + ["v_mov_b32_e32 v2, 0"] + b[13:], "overwrite of an in-flight register"),
])
def test_checker_catches_uncovered_use(mutate, what):
    body = mutate(list(LOOP))
    n, k, errors = vmem_order.check_text(listing(body))
    assert errors, what


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhjd.so not built")
def test_built_library_prefetch_is_counted_and_covered():
    text = d16_order.disassemble(LIB)
    rows, errors = vmem_order.check_counted(vmem_order._functions(text))
    # BGRX 4:4:4 and 4:2:0 q16 kernels with variant bits 0-3, plus the two
    # d16 4:4:4 product kernels
    assert len(rows) == 10 and errors == [], (rows, errors)
    counts = {name: max(w) for name, w in rows}
    assert all(c == (8 if "ILi1E" in name else 4) for name, c in counts.items()), counts
    n, k, errors = vmem_order.check_text(text)
    assert n > 0 and errors == [], errors[:5]
