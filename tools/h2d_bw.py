#!/usr/bin/env python3
"""Pinned host -> device copy bandwidth (the PCIe ceiling of the JPEG stream)."""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for mb in (4, 64, 256):
        n = mb << 20
        h = torch.empty(n, dtype=torch.uint8).pin_memory()
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        reps = max(4, 2048 // mb)
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            for _ in range(reps):
                d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        res[f"{mb}MiB"] = round(n * reps / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps({"h2d_pinned_GBps": res}))


if __name__ == "__main__":
    main()
