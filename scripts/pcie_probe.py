"""PCIe rates between page-locked host memory and HBM on this box (torch as plumbing:
pinned tensors, copies on side streams): host->device alone, device->host alone, both
directions at once, and 4 device->host streams at once -- the bounds of the drop-in
caller's end-to-end path (bench.py pcie_inclusive: a C2 request uploads 52.9 MB of
compressed blocks and downloads 90.3 MB of 16-bit PCM or 180.6 MB of int32).

usage: python3 scripts/pcie_probe.py [--mb 90] [--reps 10]"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=90)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = a.mb << 20
    hs = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    ds = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
    st = [torch.cuda.Stream() for _ in range(4)]

    def run(jobs):
        # jobs: list of (stream index, direction); each job copies n bytes reps times
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            for i, dirn in jobs:
                with torch.cuda.stream(st[i]):
                    if dirn == "h2d":
                        ds[i].copy_(hs[i], non_blocking=True)
                    else:
                        hs[i].copy_(ds[i], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return round(n * a.reps * len(jobs) / dt / 1e9, 2)

    run([(0, "h2d"), (1, "d2h")])  # warm
    out = {"MB": a.mb, "reps": a.reps,
           "h2d_GBs": run([(0, "h2d")]),
           "d2h_GBs": run([(0, "d2h")]),
           "both_GBs_total": run([(0, "h2d"), (1, "d2h")]),
           "d2h_x4_GBs_total": run([(i, "d2h") for i in range(4)]),
           "h2d_x4_GBs_total": run([(i, "h2d") for i in range(4)]),
           "mixed_2h2d_2d2h_GBs_total": run([(0, "h2d"), (1, "h2d"), (2, "d2h"), (3, "d2h")])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
