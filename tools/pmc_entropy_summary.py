#!/usr/bin/env python3
"""Summarise the SQ counter passes of tools/pmc_entropy.txt per entropy kernel."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(os.path.join(root, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            k = "sync" if "ent_sync" in k else "write" if "ent_write" in k else None
            if k:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in sorted(agg.items()):
        wc = d["SQ_WAVE_CYCLES"] or 1
        w = d["SQ_WAVES"] or 1
        print(f"{k}: parked {d['SQ_WAIT_ANY'] / wc * 100:.0f}%  issue-stall {d['SQ_WAIT_INST_ANY'] / wc * 100:.0f}%  "
              f"active {d['SQ_ACTIVE_INST_ANY'] / wc * 100:.0f}% (valu {d['SQ_ACTIVE_INST_VALU'] / wc * 100:.0f}%)  | per wave: "
              f"valu {d['SQ_INSTS_VALU'] / w:.0f} salu {d['SQ_INSTS_SALU'] / w:.0f} lds {d['SQ_INSTS_LDS'] / w:.0f} "
              f"branch {d['SQ_INSTS_BRANCH'] / w:.0f} vmem_rd {d['SQ_INSTS_VMEM_RD'] / w:.0f}")


if __name__ == "__main__":
    main()
