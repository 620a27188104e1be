#!/usr/bin/env python3
"""Tabulate the per-box measurements of round-4 bench lines (one row per
bench JSON): GPU serial, 4:2:0 / 4:4:4 fraction of 8 TB/s, fraction of the
box's own ceiling, in-kernel clock under load, the memory-only variant's
time, and the box's read-only / write-only streaming rates.

    python tools/box_table.py gpurun_out/r04*/bench*.json > profiles/r04_box_table.json
"""
import json
import sys


def row(path):
    d = json.load(open(path))
    out = {"source": path, "box": d.get("box")}
    for key, x in (("4k420", d), ("4k444", d.get("config4_444") or {})):
        r = x.get("roofline") or {}
        bc = x.get("box_ceiling") or {}
        st = x.get("stages") or {}
        out[key] = {"frac": r.get("frac"), "frac_of_box_ceiling": r.get("frac_of_box_ceiling"),
                    "box_ceiling_GBps": r.get("box_ceiling_GBps"), "ceiling_from": bc.get("ceiling_from"),
                    "kernel_ms": r.get("kernel_ms_per_launch"), "memory_only_ms": st.get("memory_only_ms"),
                    "sclk_GHz": (x.get("clock_under_load") or {}).get("sclk_GHz_median"),
                    "read_only_GBps": bc.get("read_only_GBps"), "write_only_GBps": bc.get("write_only_GBps"),
                    "launch": {k: (x.get("launch") or {}).get(k) for k in ("tasks_per_wave", "stores")}}
    return out


if __name__ == "__main__":
    print(json.dumps({"what": "round-4 bench lines per MI355X box (tools/box_table.py)",
                      "rows": [row(p) for p in sys.argv[1:]]}, indent=1))
