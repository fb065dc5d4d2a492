"""Per-phase host timings of the end-to-end request path (frame, upload,
decode, download) for 1 and 3 concurrent host threads, one batch each, on the
C2 batch.  Diagnostic for bench.py's pcie_inclusive / pipelined numbers.

    python scripts/e2e_probe.py [--rounds 4] [--threads 1 3]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from synth import corpora  # noqa: E402
import wavpackdecoder_amd.api as api  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 3])
    ap.add_argument("--frame-threads", type=int, default=0)
    a = ap.parse_args()
    data = corpora.c2(nblocks=1024, block=22050)
    batches = []
    for _ in range(max(a.threads)):
        b = DecodeBatch(4096)
        b.add_files([data])
        b.upload()
        b.decode()
        b.download(pinned=True)
        batches.append(b)
    frames = batches[0].frames
    for nt in a.threads:
        ph = {k: [] for k in ("frame", "upload", "decode", "download")}
        lock = threading.Lock()

        def serve(b):
            for _ in range(a.rounds):
                t0 = time.perf_counter()
                b.reset()
                b.add_files([data], threads=a.frame_threads)
                t1 = time.perf_counter()
                b.upload()
                t2 = time.perf_counter()
                b.decode()
                b.sync()
                t3 = time.perf_counter()
                b.download(pinned=True)
                t4 = time.perf_counter()
                with lock:
                    ph["frame"].append(t1 - t0)
                    ph["upload"].append(t2 - t1)
                    ph["decode"].append(t3 - t2)
                    ph["download"].append(t4 - t3)

        th = [threading.Thread(target=serve, args=(batches[i],)) for i in range(nt)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        t = time.perf_counter() - t
        print(json.dumps({"threads": nt, "Msamples_per_s": round(frames * a.rounds * nt / t / 1e6, 1),
                          "ms_per_request_wall": round(t / (a.rounds * nt) * 1e3, 2),
                          **{k + "_ms": round(float(np.median(v)) * 1e3, 2) for k, v in ph.items()}}), flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
