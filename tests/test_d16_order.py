"""The 4:4:4 d16 gather's ordering, checked on the built library (ADVICE r3,
medium; DESIGN.md s3 "perm-free gathers").  The inline-asm ds_read_u16_d16_hi
results are only valid after a covering s_waitcnt lgkmcnt; a compiler that
copied, spilled or consumed a destination register earlier would corrupt
4:4:4 pixels silently.  tools/check/d16_order.py verifies every such load in
the gfx950 code objects of libhjd.so; the synthetic listings below show that
the checker catches each way the ordering can break."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "check"))
import d16_order  # noqa: E402

LIB = os.path.join(REPO, "ocljpegdecoder_amd", "lib", "libhjd.so")

GOOD = """
0000000000001000 <_ZN3hjd13decode_kernelILi0ELi0ELi128EEEvPKvPKiPKNS_8FrameDevEilPh>:
	ds_read_u16_d16_hi v26, v57                                // 0
	ds_read_u16_d16_hi v27, v58                                // 8
	ds_read_u16 v38, v72                                       // 10
	ds_read_u16 v54, v73                                       // 18
	s_waitcnt lgkmcnt(1)                                       // 20
	v_or_b32_e32 v26, v26, v38                                 // 24
	s_waitcnt lgkmcnt(0)                                       // 28
	v_or_b32_e32 v27, v27, v54                                 // 2c
	s_endpgm                                                   // 30
"""


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhjd.so not built")
def test_built_library_d16_loads_are_covered():
    n, errors = d16_order.check_text(d16_order.disassemble(LIB))
    # 24 d16 loads per kVarD16 kernel (4 per round x 6 rounds); at least the
    # BGRX and BGR24 4:4:4 product kernels carry them
    assert n >= 48, n
    assert errors == [], errors[:5]


def test_checker_accepts_covered_listing():
    assert d16_order.check_text(GOOD) == (2, [])


@pytest.mark.parametrize("mutation, what", [
    (("s_waitcnt lgkmcnt(1)", "s_waitcnt lgkmcnt(4)"), "wait too weak"),
    (("s_waitcnt lgkmcnt(1)                                       // 20\n",
      "v_mov_b32_e32 v90, v26                                     // 1c\n\ts_waitcnt lgkmcnt(1)"
      "                                       // 20\n"), "copy before the wait"),
    (("s_waitcnt lgkmcnt(1)", "s_cbranch_scc1 3"), "branch before the wait"),
    ("early wait", "wait issued before the younger DS ops it counts on"),
])
def test_checker_catches_broken_ordering(mutation, what):
    if mutation == "early wait":   # the lgkmcnt(1) moved up to right after the first d16 load
        lines = GOOD.splitlines(keepends=True)
        wait = next(l for l in lines if "lgkmcnt(1)" in l)
        lines.remove(wait)
        lines.insert(next(i for i, l in enumerate(lines) if "v26, v57" in l) + 1, wait)
        text = "".join(lines)
    else:
        text = GOOD.replace(*mutation)
    assert text != GOOD
    n, errors = d16_order.check_text(text)
    assert n == 2 and errors, what
