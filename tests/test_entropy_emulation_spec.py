"""CPU: the speculative sync of latency decoders ("Single-image
latency": ent_spec_kernel / ent_cand_kernel / ent_chain_kernel, run on the
host by hjd_debug_entropy_emulate with HJD_SYNC_SPEC=1) must reproduce the
host Huffman decoder's coefficients exactly, like the round-based sync.  Every
test of test_entropy_emulation.py runs again in this mode (imported below),
and the spec runs' lead-in is swept, down to 0 bits, where the chain leaves
the candidate slots often and the chain kernel's repair path is exercised."""
import os

import numpy as np
import pytest

import test_entropy_emulation as E
from test_entropy_emulation import *  # noqa: F401,F403  (re-run the whole module in speculative mode)


@pytest.fixture(autouse=True)
def _spec_sync(monkeypatch):
    monkeypatch.setenv("HJD_SYNC_SPEC", "1")
    yield


@pytest.mark.parametrize("lead", [0, 64, 512, 2048])
@pytest.mark.parametrize("sub_bits", [32, 256, 512])
def test_lead_in_sweep(hjd, monkeypatch, lead, sub_bits):
    monkeypatch.setenv("HJD_SPEC_LEAD", str(lead))
    for i, (name, kw) in enumerate(E.CASES[:11]):
        kw = dict(kw)
        data = E._pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=900 + i, **kw)
        ref, _ = hjd.decode_coefs(data)
        got, status = hjd.emulate_entropy(data, sub_bits)
        np.testing.assert_array_equal(got, ref, err_msg=f"{name} S={sub_bits} lead={lead}")
        assert status & ~1 == 0


def test_reference_sample_all_leads(hjd, monkeypatch):
    for lead in (0, 1, 300, 4096):
        monkeypatch.setenv("HJD_SPEC_LEAD", str(lead))
        for name in E.O.golden_cases():
            data = open(os.path.join(E.O.GOLDEN, name + ".jpg"), "rb").read()
            ref, _ = hjd.decode_coefs(data)
            got, status = hjd.emulate_entropy(data, 64)
            np.testing.assert_array_equal(got, ref, err_msg=f"{name} lead={lead}")


def test_repair_sets_status_bit_and_long_leads_avoid_it(hjd, monkeypatch):
    """The premise of the decoder's lead-in ladder (spec_lead_bits): status bit
    0 reports that the chain needed a repair; this q90 4:4:4 FHD frame breaks
    9 times at the short lead-in (512 bits) and never at the ladder's next
    step (1536).  The GPU test of the ladder relies on exactly this."""
    data = E._pil(1920, 1080, 90, 0, seed=5)
    ref, _ = hjd.decode_coefs(data)
    for lead, bit in ((512, 1), (1536, 0)):
        monkeypatch.setenv("HJD_SPEC_LEAD", str(lead))
        got, status = hjd.emulate_entropy(data, 512)
        np.testing.assert_array_equal(got, ref, err_msg=f"lead={lead}")
        assert status == bit, (lead, status)
