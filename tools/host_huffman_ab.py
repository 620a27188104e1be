"""Interleaved A/B of the host Huffman decoder (jpeg_host.cpp) across library
builds: each round runs every library in its own process on the same pool of
synthetic 4K q90 JPEGs (bench.encode_pool), 1 thread and N threads.

    python tools/host_huffman_ab.py product+build/variants/x/libhjd.so [--rounds 3] [--threads 16] [--sampling 1]

("product" = the in-tree library; libraries separated by '+'; a "#bytewise"
suffix runs that library with the byte-wise reader, hjd_debug_host_reader(1)).
Outputs are preallocated and touched once, so no page faults are timed.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, json, sys, time
import numpy as np
sys.path.insert(0, REPO)
import bench
from ocljpegdecoder_amd import _lib
lib = _lib.load()
s, nt, reader = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
lib.hjd_debug_host_reader(reader)
pool = bench.encode_pool(3840, 2160, s, 8, seed0=99)
u8p, i16p = ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int16)
bufs = [(ctypes.c_uint8 * len(d)).from_buffer_copy(d) for d in pool]
cap = 3840 * 2160 * 3 // 128 + 4096        # blocks of a 4K 4:4:4 frame and then some
outs = [np.ones((cap, 64), np.int16) for _ in range(2 * nt)]   # touched once: no page faults timed

def run(n, reps):
    arr_d = (u8p * reps)(*[ctypes.cast(bufs[i % len(bufs)], u8p) for i in range(reps)])
    arr_s = (ctypes.c_size_t * reps)(*[len(pool[i % len(pool)]) for i in range(reps)])
    arr_o = (i16p * reps)(*[outs[i % len(outs)].ctypes.data_as(i16p) for i in range(reps)])
    st = (ctypes.c_int32 * reps)()
    t0 = time.perf_counter()
    rc = lib.hjd_jpeg_decode_batch(arr_d, arr_s, reps, arr_o, cap, n, st)
    dt = time.perf_counter() - t0
    assert rc == 0 and not any(st)
    return reps * 3840 * 2160 / dt / 1e6

run(1, 2)
res = {}
for key, n, reps in (("one_thread", 1, 8), ("threads", nt, 8 * nt)):
    res[key] = round(max(run(n, reps) for _ in range(3)), 1)
print(json.dumps(res))
""".replace("REPO", repr(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--sampling", type=int, default=1)
    a = ap.parse_args()
    rows = []
    for r in range(a.rounds):
        for lib in a.libs.split("+"):
            env = dict(os.environ)
            path, _, reader = lib.partition("#")
            if path != "product":
                env["HJD_LIB"] = os.path.join(REPO, path)
            out = subprocess.run([sys.executable, "-c", CHILD, str(a.sampling), str(a.threads),
                                  "1" if reader == "bytewise" else "0"], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode:
                raise SystemExit(out.stderr[-2000:])
            d = json.loads(out.stdout.strip().splitlines()[-1])
            rows.append({"round": r, "lib": lib, **d})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    summary = {}
    for lib in a.libs.split("+"):
        mine = [x for x in rows if x["lib"] == lib]
        summary[lib] = {k: [x[k] for x in mine] for k in ("one_thread", "threads")}
    print(json.dumps({"what": "host Huffman Mpx/s (4K q90 synthetic, bench.encode_pool)", "threads": a.threads,
                      "sampling": a.sampling, "rows": rows, "summary": summary}))


if __name__ == "__main__":
    main()
