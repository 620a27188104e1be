"""One worker process of bench.py's multi-core timing of the REFERENCE CPU path
(cpu_reference): the reference's own decode_mcu_data (src/decoder.cpp:397-523,
USE_CPU_ONLY: Fast_IDCT + upsample + fp64 colour + its BMP fwrite), compiled
from its sources into oracle/_ref/libref.so.  TEST INFRASTRUCTURE ONLY: started
by bench.py's cpu_baseline leg, never on the product path.

    python tests/ref_cpu_worker.py <frame.npy> <width> <height> <sampling> <reps> <workdir>

The reference keeps global state and writes "m:\\output.bmp" into its cwd
(src/decoder.cpp:420), so each worker is its own process in its own workdir.
Protocol: prints "ready" once the frame copies are made, waits for one line
on stdin ("go"), decodes `reps` copies of the frame (the reference transforms
mcu_data in place, so every rep gets a fresh copy, made before "ready"), then
prints one JSON line {"frames", "seconds"}.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_py as O  # noqa: E402


def main():
    path, w, h, s, reps, workdir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5]), sys.argv[6]
    nat = np.load(path)
    bufs = [np.ascontiguousarray(nat, dtype=np.int32).copy() for _ in range(reps)]
    lib = O.ref()
    lib.ref_decode_mcu_data.argtypes = [O.i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    os.chdir(workdir)
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    for b in bufs:
        rc = lib.ref_decode_mcu_data(b.ctypes.data_as(O.i32p), w, h, s)
        if rc != 0:
            print(json.dumps({"error": f"decode_mcu_data rc {rc}"}), flush=True)
            sys.exit(1)
    print(json.dumps({"frames": reps, "seconds": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
