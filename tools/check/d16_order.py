#!/usr/bin/env python3
"""Static check of the 4:4:4 d16 gather in the BUILT library.

    python tools/check/d16_order.py [path/to/libhjd.so]

load_round_pk_d16 (csrc/hjd_kernels.hpp) issues ds_read_u16_d16_hi as inline
asm whose result the compiler believes is ready at once; the data really
lands only when the LDS counter says so.  The kernel is correct only if the
first instruction touching each d16 destination VGPR comes after an
`s_waitcnt lgkmcnt(k)` that covers that load.  LDS operations of a wave
complete in order, so once the d16 load was issued, lgkmcnt <= k guarantees
it is done when k <= the number of DS instructions issued after it (every
younger DS op is still counted while the d16 op is pending).  SMEM ops share
the counter but may complete out of order, so they are not counted as cover.

This script extracts the code objects of the build's architecture (HJD_ARCH,
default gfx950, as tools/build_native.py) from the library (llvm-objdump
--offloading, in a temporary directory), disassembles them and checks every
ds_read_u16_d16_hi in program order: the destination register must not
appear in any operand (read, copy or overwrite) before a covering wait, and
no branch may come between the load and that wait.  Exit status 1 and a list
of violations if any load is not covered.
"""
from __future__ import annotations

import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM_OBJDUMP = os.environ.get("LLVM_OBJDUMP", "/opt/rocm/lib/llvm/bin/llvm-objdump")
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_LIB = os.path.join(REPO, "ocljpegdecoder_amd", "lib", "libhjd.so")
# the architecture the library was built for (tools/build_native.py ARCH)
ARCH = os.environ.get("HJD_ARCH", "gfx950")

_FUNC = re.compile(r"^[0-9a-f]+ <([^>]+)>:")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_BRANCH = ("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_endpgm")


def disassemble(lib_path: str, arch: str = ARCH) -> str:
    """Disassembly text of every `arch` code object bundled in lib_path."""
    tmp = tempfile.mkdtemp(prefix="hjd_d16chk_")
    try:
        dst = os.path.join(tmp, os.path.basename(lib_path))
        shutil.copy(lib_path, dst)
        subprocess.run([LLVM_OBJDUMP, "--offloading", dst], cwd=tmp, check=True, capture_output=True)
        texts = []
        for co in sorted(glob.glob(os.path.join(tmp, f"*{arch}*"))):
            r = subprocess.run([LLVM_OBJDUMP, "-d", f"--mcpu={arch}", co], check=True, capture_output=True, text=True)
            texts.append(r.stdout)
        return "\n".join(texts)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _regs(operands: str):
    out = set()
    for m in _VREG.finditer(operands):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _parse(text: str):
    """[(function, mnemonic, operand text)] in program order."""
    insts, func = [], None
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            func = m.group(1)
            continue
        body = line.split("//", 1)[0].strip()
        if not body or func is None or body.endswith(":"):
            continue
        parts = body.split(None, 1)
        insts.append((func, parts[0], parts[1] if len(parts) > 1 else ""))
    return insts


def check_text(text: str):
    """(number of d16 loads checked, [violation strings])."""
    insts = _parse(text)
    errors, n = [], 0
    for i, (func, mn, ops) in enumerate(insts):
        if mn != "ds_read_u16_d16_hi":
            continue
        n += 1
        dst = int(ops.split(",")[0].strip()[1:])
        younger_ds, covered = 0, False
        for j in range(i + 1, len(insts)):
            f2, mn2, ops2 = insts[j]
            if f2 != func:
                errors.append(f"{func}: d16 load #{i} into v{dst}: function ends before a covering wait")
                break
            if mn2 == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", ops2)
                if m and int(m.group(1)) <= younger_ds:
                    covered = True
                    break
                continue
            if mn2.startswith(_BRANCH):
                errors.append(f"{func}: d16 load #{i} into v{dst}: {mn2} before a covering wait")
                break
            if dst in _regs(ops2):
                errors.append(f"{func}: d16 load #{i} into v{dst}: `{mn2} {ops2}` touches it before a covering "
                              f"wait ({younger_ds} younger DS ops)")
                break
            if mn2.startswith("ds_"):
                younger_ds += 1
        else:
            if not covered:
                errors.append(f"{func}: d16 load #{i} into v{dst}: no covering wait")
    return n, errors


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    n, errors = check_text(disassemble(lib))
    for e in errors:
        print(e)
    print(f"{n} ds_read_u16_d16_hi checked, {len(errors)} not covered by an s_waitcnt lgkmcnt")
    sys.exit(1 if errors or n == 0 else 0)


if __name__ == "__main__":
    main()
