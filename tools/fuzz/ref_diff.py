"""Differential fuzzing of the host decoder against the compiled reference
(oracle/_ref/libref.so, this container only): damaged copies of the golden
JPEGs (byte flips in the scan, 0xFF / RSTn insertions, truncation) decoded by
the reference's own load_jpg (in a forked child: it may abort) and by
hjd_jpeg_decode_coefs.  Every mutant is classified:

  both_reject, both_accept_equal         agreement
  both_accept_differ                     a divergence to explain
  ref_accepts_only, host_accepts_only    a divergence to explain

    python tools/fuzz/ref_diff.py [--mutants 2000] [--seed 1] [--json out.json]

Divergent mutants are written to --keep DIR for a closer look.
"""
import argparse
import collections
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

FILES = ["JPEG_example_JPG_RIP_050", "syn444_64x40_q90", "syn420_160x48_q95_dri", "syn444_odd_41x23_q75",
         "syn420_80x80_q50_opt", "syn420_96x64_q90", "syn444_48x32_q100"]


def mutate(data: bytes, so: int, rng) -> bytes:
    d = bytearray(data)
    kind = int(rng.integers(0, 5))
    end = len(d) - 2
    if kind == 0:      # byte flips inside the scan
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(so, end))
            d[p] = int(rng.integers(0, 256))
    elif kind == 1:    # a bit flip inside the scan
        p = int(rng.integers(so, end))
        d[p] ^= 1 << int(rng.integers(0, 8))
    elif kind == 2:    # insert 0xFF or an RSTn marker
        p = int(rng.integers(so, end))
        ins = bytes([0xFF]) if rng.random() < 0.5 else bytes([0xFF, 0xD0 + int(rng.integers(0, 8))])
        d[p:p] = ins
    elif kind == 3:    # delete a byte of the scan
        p = int(rng.integers(so, end))
        del d[p]
    else:              # truncation, EOI kept or not
        p = int(rng.integers(so, end))
        d = d[:p] + (b"\xff\xd9" if rng.random() < 0.5 else b"")
    return bytes(d)


def _rst_count(d: bytes) -> int:
    return sum(d.count(bytes([0xFF, 0xD0 + n])) for n in range(8))


def explain(orig: bytes, d: bytes, host_err: str, info) -> str:
    """The documented reasons the reference accepts a mutant the host rejects
    (INTEGRATION.md section 4): an RSTn marker that was not there before (an
    inserted one, or one made by an inserted 0xFF / a deleted stuffing 0x00),
    which the reference reads as two data bytes; or a shortened scan that ends
    in the last MCU, which the reference completes from past its data."""
    if _rst_count(d) > _rst_count(orig):
        return "new_rst_marker_read_as_data"
    nmcu = info.mcu_w * info.mcu_h
    if f"(MCU {nmcu - 1} of {nmcu})" in host_err:
        return "last_mcu_read_past_data"
    return "unexplained"


def classify(data_list, mutants, seed, keep=None):
    """Mutate and classify; returns (counts, explanations of ref_accepts_only,
    examples per divergent class)."""
    import ocljpegdecoder_amd as hjd
    import oracle_py as O
    from test_truncation import _ref_decode
    rng = np.random.default_rng(seed)
    cnt = collections.Counter()
    why = collections.Counter()
    examples = collections.defaultdict(list)
    for i in range(mutants):
        k = i % len(data_list)
        name, data = data_list[k]
        so = hjd.parse(data).scan_offset
        d = mutate(data, so, rng)
        ref_ok, cap = _ref_decode(d)
        try:
            coefs, info = hjd.decode_coefs(d)
            host_ok, err = True, ""
        except Exception as e:   # noqa: BLE001 -- the decoder's error is the classification
            host_ok, err = False, str(e)
        if ref_ok and host_ok:
            nat = O.dequant_natural(coefs, np.array(info.qt), info.sampling)
            cls = "both_accept_equal" if cap is not None and np.array_equal(nat, cap) else "both_accept_differ"
        elif ref_ok:
            cls = "ref_accepts_only"
        elif host_ok:
            cls = "host_accepts_only"
        else:
            cls = "both_reject"
        cnt[cls] += 1
        if cls == "ref_accepts_only":
            why[explain(data, d, err, hjd.parse(data))] += 1
        if cls not in ("both_reject", "both_accept_equal"):
            examples[cls].append({"mutant": i, "file": name, "host_error": err[-120:]})
            if keep:
                os.makedirs(keep, exist_ok=True)
                with open(os.path.join(keep, f"{cls}_{i}.jpg"), "wb") as f:
                    f.write(d)
    return cnt, why, examples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mutants", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--json")
    ap.add_argument("--keep")
    a = ap.parse_args()
    import oracle_py as O
    srcs = [(n, open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read()) for n in FILES]
    cnt, why, examples = classify(srcs, a.mutants, a.seed, a.keep)
    out = {"mutants": a.mutants, "seed": a.seed, "counts": dict(cnt),
           "ref_accepts_only_explained": dict(why),
           "examples": {k: v[:20] for k, v in examples.items()}}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
