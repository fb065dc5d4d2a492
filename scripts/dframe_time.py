#!/usr/bin/env python3
"""Framing cost: host framing (wvg_batch_add_files on 16 threads) + upload vs
device framing (wvg_batch_add_files_device, framed inside the upload), on a warm
batch (reset between runs), for C2 (one 1,024-block file) and a C5 slice.
Prints one JSON line per workload."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from synth import corpora  # noqa: E402
from wavpackdecoder_amd import api  # noqa: E402


def run(name, files, reps=5):
    res = {"workload": name, "files": len(files)}
    for mode in ("host", "device"):
        b = api.DecodeBatch(4096)
        ts, tf = [], []
        for r in range(reps + 1):
            b.reset()
            t = time.perf_counter()
            if mode == "host":
                b.add_files(files, threads=16)
            else:
                b.add_files_device(files)
            t1 = time.perf_counter()
            b.upload()
            ts.append(time.perf_counter() - t)
            tf.append(t1 - t)
        res[f"{mode}_add_ms"] = round(sorted(tf[1:])[len(tf[1:]) // 2] * 1e3, 3)
        b.decode()
        b.sync()
        if mode == "device":
            res["framed_device_host"] = b.framing_stats()
        res[f"{mode}_ms"] = round(sorted(ts[1:])[len(ts[1:]) // 2] * 1e3, 3)
        res["blocks"] = b.num_blocks
        b.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    run("C2 1 file x 1024 blocks", [corpora.c2()])
    run("C5 files 0..1999", corpora.c5(2000))
