"""Build the native library in-tree: ocljpegdecoder_amd/lib/libhjd.so (gfx950).

    python tools/build_native.py [--force]

One shared library holds the HIP kernels + C-ABI runtime (include/hjd.h), the
idct.h compatibility shim (include/idct.h) and the host JPEG front end
(include/hjd_host.h).  hipcc cross-compiles for gfx950 without a GPU.
"""
from __future__ import annotations

import json
import os
import subprocess
import time
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ocljpegdecoder_amd")
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libhjd.so")
OBJDIR = os.path.join(REPO, "build", "obj")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HJD_ARCH", "gfx950")

HIP_SOURCES = ["hjd_runtime.hip", "idct_compat.hip", "stream_pipeline.hip", "hjd_entropy.hip", "numa_affinity.hip",
               "hjd_probe.hip"]
CXX_SOURCES = ["jpeg_host.cpp"]

COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}"]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _needs(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return hs


def build(verbose: bool = False, force: bool = False, variant: str = "",
          defines=(), record: bool = False) -> str:
    """variant="name", defines=("FLAG", ...) builds an A/B library
    build/variants/<name>/libhjd.so with -DFLAG (tuning only; load it with
    HJD_LIB=build/variants/<name>/libhjd.so)."""
    global LIBDIR, LIB, OBJDIR
    if variant:
        LIBDIR = os.path.join(REPO, "build", "variants", variant)
        LIB = os.path.join(LIBDIR, "libhjd.so")
        OBJDIR = os.path.join(REPO, "build", "obj_variants", variant)
        COMMON.extend(f"-D{d}" for d in defines)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    headers = _headers()
    jobs = []
    objs = []
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        if not os.path.exists(s):
            continue
        o = os.path.join(OBJDIR, src + ".o")
        objs.append(o)
        if force or _needs(o, [s] + headers):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-c", s, "-o", o])
    for src in CXX_SOURCES:
        s = os.path.join(CSRC, src)
        if not os.path.exists(s):
            continue
        o = os.path.join(OBJDIR, src + ".o")
        objs.append(o)
        if force or _needs(o, [s] + headers):
            # host-only C++ (no device code): compiled by hipcc's clang as plain C++
            extra = os.environ.get("HJD_HOST_CXXFLAGS", "").split()   # tuning A/Bs of the host decoder
            jobs.append([HIPCC, *COMMON, *extra, "-x", "c++", "-pthread", "-c", s, "-o", o])
    t0 = time.time()
    if force:   # a forced build starts from an empty object directory
        for f in os.listdir(OBJDIR):
            if f.endswith(".o"):
                os.remove(os.path.join(OBJDIR, f))
    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    if force or jobs or _needs(LIB, objs):
        out = _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", LIB, *objs])
        if verbose and out.strip():
            print(out)
    if record:
        rec = {"build_mode": "full" if force else "incremental", "objects_compiled": len(jobs),
               "objects_linked": len(objs), "sources": [os.path.relpath(j[-3], REPO) for j in jobs], "arch": ARCH,
               "library": os.path.relpath(LIB, REPO), "library_bytes": os.path.getsize(LIB),
               "seconds": round(time.time() - t0, 1), "utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        with open(os.path.join(REPO, "build", "build_record.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print("build_record:", json.dumps(rec))
    return LIB


if __name__ == "__main__":
    var, defs = "", []
    if "--variant" in sys.argv:
        var = sys.argv[sys.argv.index("--variant") + 1]
        defs = [a[2:] for a in sys.argv if a.startswith("-D")]
    print(build(verbose=True, force="--force" in sys.argv, variant=var, defines=defs))
