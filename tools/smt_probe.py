"""SMT yield of the host Huffman decoder: the same
16-thread hjd_jpeg_decode_batch over synthetic 4K q90 4:2:0 files
(bench.encode_pool) pinned to
  * "cores":    16 logical CPUs on 16 different physical cores,
  * "siblings": 16 logical CPUs that are the two SMT threads of 8 cores,
  * "node":     every logical CPU of one NUMA node (threads = that count),
all on one NUMA node.  Under the one-GPU box's 16-CPU cgroup quota "cores"
and "siblings" get the same CPU time; siblings / (cores / 2) is what one
physical core gains from its second hardware thread.

    python tools/smt_probe.py [--rounds 3] [--files 8]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def topology():
    """{core key: [logical cpus]} and {cpu: numa node} for the allowed CPUs."""
    allowed = sorted(os.sched_getaffinity(0))
    cores, node_of = {}, {}
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}"
        try:
            pkg = open(f"{base}/topology/physical_package_id").read().strip()
            core = open(f"{base}/topology/core_id").read().strip()
        except OSError:
            pkg, core = "0", str(c)
        cores.setdefault((pkg, core), []).append(c)
        node = 0
        for e in os.listdir(base):
            if e.startswith("node") and e[4:].isdigit():
                node = int(e[4:])
        node_of[c] = node
    return cores, node_of


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import bench
    from ocljpegdecoder_amd import _lib
    lib = _lib.load()
    cores, node_of = topology()
    node0 = node_of[min(node_of)]
    mine = [v for v in cores.values() if node_of[v[0]] == node0]
    pairs = [v for v in mine if len(v) >= 2]
    n = a.threads
    sets = {"cores": [v[0] for v in mine[:n]]}
    if len(pairs) >= n // 2:
        sets["siblings"] = [c for v in pairs[: n // 2] for c in v[:2]]
    sets["node"] = sorted(c for v in mine for c in v)
    pool = bench.encode_pool(3840, 2160, 1, a.files, seed0=99)
    u8p, i16p = ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int16)
    bufs = [(ctypes.c_uint8 * len(d)).from_buffer_copy(d) for d in pool]
    cap = 3840 * 2160 * 3 // 128 + 4096
    nmax = max(len(s) for s in sets.values())
    outs = [np.ones((cap, 64), np.int16) for _ in range(2 * nmax)]

    def run(nthreads, reps):
        arr_d = (u8p * reps)(*[ctypes.cast(bufs[i % len(bufs)], u8p) for i in range(reps)])
        arr_s = (ctypes.c_size_t * reps)(*[len(pool[i % len(pool)]) for i in range(reps)])
        arr_o = (i16p * reps)(*[outs[i % len(outs)].ctypes.data_as(i16p) for i in range(reps)])
        st = (ctypes.c_int32 * reps)()
        t0 = time.perf_counter()
        rc = lib.hjd_jpeg_decode_batch(arr_d, arr_s, reps, arr_o, cap, nthreads, st)
        dt = time.perf_counter() - t0
        assert rc == 0 and not any(st)
        return reps * 3840 * 2160 / dt / 1e6

    full = os.sched_getaffinity(0)
    res = {k: [] for k in sets}
    try:
        for r in range(a.rounds):
            for k, cpus in sets.items():
                os.sched_setaffinity(0, cpus)   # the pool's threads inherit the caller's mask
                run(len(cpus), len(cpus))       # warm
                res[k].append(round(run(len(cpus), 6 * len(cpus)), 1))
                print(json.dumps({"round": r, "set": k, "cpus": len(cpus), "mpx_s": res[k][-1]}), file=sys.stderr,
                      flush=True)
    finally:
        os.sched_setaffinity(0, full)
    best = {k: max(v) for k, v in res.items()}
    out = {"what": "host Huffman Mpx/s, 4K q90 4:2:0 (bench.encode_pool), pinned CPU sets on NUMA node %d" % node0,
           "sets": {k: v for k, v in sets.items()}, "threads": {k: len(v) for k, v in sets.items()},
           "rounds": res, "best": best, "node_logical_cpus": len(sets["node"]), "node_cores": len(mine),
           "affinity_cpus": len(full), "cpu_share": lib.hjd_host_cpu_share()}
    if "siblings" in best:
        out["smt_core_yield"] = round(best["siblings"] / (best["cores"] / 2), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
