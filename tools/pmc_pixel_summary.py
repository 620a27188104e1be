#!/usr/bin/env python3
"""Summarise tools/pmc_pixel.txt passes for the fused kernel (decode_kernel)."""
import collections
import csv
import glob
import os
import sys


def main():
    d = collections.defaultdict(float)
    for p in glob.glob(os.path.join(sys.argv[1], "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            if "decode_kernel" in r["Kernel_Name"]:
                d[r["Counter_Name"]] += float(r["Counter_Value"])
    wc = d["SQ_WAVE_CYCLES"] or 1
    w = d["SQ_WAVES"] or 1
    print(f"parked {d['SQ_WAIT_ANY'] / wc * 100:.0f}%  issue-stall {d['SQ_WAIT_INST_ANY'] / wc * 100:.0f}%  "
          f"active {d['SQ_ACTIVE_INST_ANY'] / wc * 100:.0f}% (valu {d['SQ_ACTIVE_INST_VALU'] / wc * 100:.0f}%, "
          f"lds {d['SQ_ACTIVE_INST_LDS'] / wc * 100:.0f}%)  lds_stall {d['SQ_WAIT_INST_LDS'] / wc * 100:.0f}%  "
          f"bank_conflict_cycles/lds_inst {d['SQ_LDS_BANK_CONFLICT'] / max(1, d['SQ_INSTS_LDS']):.2f}")
    print(f"per wave: valu {d['SQ_INSTS_VALU'] / w:.0f} salu {d['SQ_INSTS_SALU'] / w:.0f} lds {d['SQ_INSTS_LDS'] / w:.0f} "
          f"vmem_rd {d['SQ_INSTS_VMEM_RD'] / w:.0f} vmem_wr {d['SQ_INSTS_VMEM_WR'] / w:.0f}")


if __name__ == "__main__":
    main()
