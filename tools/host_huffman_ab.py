"""Interleaved A/B of the host Huffman decoder (jpeg_host.cpp) across library
builds: each round runs every library in its own process on the same pool of
synthetic 4K q90 JPEGs (bench.encode_pool), 1 thread and N threads.

    python tools/host_huffman_ab.py product+build/variants/x/libhjd.so [--rounds 3] [--threads 16] [--sampling 1]

("product" = the in-tree library; libraries separated by '+').
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, REPO)
import bench
import ocljpegdecoder_amd as hjd
s, nt = int(sys.argv[1]), int(sys.argv[2])
pool = bench.encode_pool(3840, 2160, s, 8, seed0=99)
hjd.decode_coefs_batch(pool[:2], nthreads=1)
res = {}
for key, n, reps in (("one_thread", 1, 8), ("threads", nt, 8 * nt)):
    best = 0.0
    for _ in range(3):
        datas = [pool[i % len(pool)] for i in range(reps)]
        t0 = time.perf_counter()
        hjd.decode_coefs_batch(datas, nthreads=n)
        best = max(best, reps * 3840 * 2160 / (time.perf_counter() - t0) / 1e6)
    res[key] = round(best, 1)
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
            if lib != "product":
                env["HJD_LIB"] = os.path.join(REPO, lib)
            out = subprocess.run([sys.executable, "-c", CHILD, str(a.sampling), str(a.threads)], env=env,
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
