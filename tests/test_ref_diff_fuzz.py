"""Differential fuzz of the host decoder against the compiled reference
(tools/fuzz/ref_diff.py; oracle/_ref/libref.so, this container only): damaged
copies of the golden files -- byte and bit flips in the scan, 0xFF / RSTn
insertions, deletions, truncations -- decoded by the reference's load_jpg and
by hjd_jpeg_decode_coefs.  Pinned here: no mutant decodes to coefficients
other than the reference's, none is accepted by the host alone, and every
mutant only the reference accepts falls in a documented divergence
(INTEGRATION.md section 4): a new RSTn marker in the scan, which the
reference reads as data, or a scan that ends inside the last MCU."""
import os
import sys

import pytest

import oracle_py as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "fuzz"))


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
def test_mutants_agree_with_reference_or_documented():
    import ref_diff
    srcs = [(n, open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read()) for n in ref_diff.FILES]
    cnt, why, examples = ref_diff.classify(srcs, 210, seed=7)
    assert cnt["both_accept_differ"] == 0, examples.get("both_accept_differ")
    assert cnt["host_accepts_only"] == 0, examples.get("host_accepts_only")
    assert why.get("unexplained", 0) == 0, examples.get("ref_accepts_only")
    assert cnt["both_accept_equal"] >= 40 and cnt["both_reject"] >= 60, dict(cnt)
