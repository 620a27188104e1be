#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite (.db) output: per-kernel count / total / mean
duration and memory copies by direction.   python tools/rocpd_summary.py run_results.db"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start) from kernels group by {name} "
                     f"order by sum(end-start) desc").fetchall()
    print(f"{'kernel':60s} {'n':>6s} {'total ms':>10s} {'mean us':>9s}")
    for n, k, tot, avg in rows:
        print(f"{n[:60]:60s} {k:6d} {tot / 1e6:10.3f} {avg / 1e3:9.1f}")
    mc = [r[1] for r in c.execute("pragma table_info(memory_copies)")]
    kind = next((k for k in ("name", "direction", "kind") if k in mc), None)
    size = next((k for k in ("size", "bytes") if k in mc), None)
    if kind and size:
        print()
        for d, k, b, tot in c.execute(f"select {kind}, count(*), sum({size}), sum(end-start) from memory_copies "
                                      f"group by {kind}"):
            print(f"copy {d}: n={k} bytes={b} busy_ms={tot / 1e6:.3f} GB/s_while_busy={b / max(tot, 1):.2f}")
    t0, t1 = c.execute("select min(start), max(end) from kernels").fetchone()
    print(f"\nkernel span {(t1 - t0) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
