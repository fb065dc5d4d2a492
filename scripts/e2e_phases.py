"""Where a warm end-to-end request's time goes (bench.py's `pcie_inclusive`): reset,
add_files (host framing into the page-locked blob) or add_files_device, upload, decode
(+ sync), download into page-locked memory -- each phase timed on its own, median of 7,
for C2 (one file of 1,024 blocks) and the first 400 files of C5.

usage: python3 scripts/e2e_phases.py [--kernel two_wave|lane|auto]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def phases(b, files, device: bool, reps: int = 7):
    rows = []
    for _ in range(reps):
        t = [time.perf_counter()]
        b.reset()
        t.append(time.perf_counter())
        if device:
            b.add_files_device(files)
        else:
            b.add_files(files)
        t.append(time.perf_counter())
        b.upload()
        b.sync()
        t.append(time.perf_counter())
        b.decode()
        b.sync()
        t.append(time.perf_counter())
        b.download(pinned=True)
        t.append(time.perf_counter())
        rows.append(np.diff(t) * 1e3)
    med = np.median(np.array(rows), axis=0)
    return {k: round(float(v), 3) for k, v in zip(("reset", "add_files", "upload", "decode", "download"), med)} | {
        "total": round(float(med.sum()), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="two_wave")
    a = ap.parse_args()
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    _, c2 = corpora.c2(return_pcm=True)
    cfgs = {"c2": [c2], "c5_400": corpora.c5(400)}
    for name, files in cfgs.items():
        b = DecodeBatch(4096)
        b.set_kernel(a.kernel)
        for device in (False, True):
            phases(b, files, device, reps=1)  # warm: buffers grown, page-locked landing area allocated
            r = phases(b, files, device)
            print(json.dumps({"config": name, "framing": "device" if device else "host", "kernel": a.kernel,
                              "ms": r}), flush=True)
        b.close()


if __name__ == "__main__":
    main()
