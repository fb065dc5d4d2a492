"""bench.py's `pipelined_pcm` request stream with 1, 2 and 4 request threads, each
phase of each request timed in its thread (reset, add_files, upload, decode + sync,
format + download_pcm): which phase stops the threads from overlapping.

usage: python3 scripts/pipe_probe.py [--kernel lane|two_wave|auto] [--rounds 4]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PHASES = ("reset", "add_files", "upload", "decode", "pcm_down")


def serve(b, files, rounds, rec):
    for _ in range(rounds):
        t = [time.perf_counter()]
        b.reset()
        t.append(time.perf_counter())
        b.add_files(files)
        t.append(time.perf_counter())
        b.upload()
        t.append(time.perf_counter())
        b.decode()
        b.sync()
        t.append(time.perf_counter())
        b.format()
        b.download_pcm(pinned=True)
        t.append(time.perf_counter())
        rec.append(np.diff(t) * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="lane")
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    _, c2 = corpora.c2(return_pcm=True)
    files = [c2]
    frames = None
    batches = []
    for _ in range(4):
        b = DecodeBatch(4096)
        b.set_kernel(a.kernel)
        serve(b, files, 1, [])  # warm: buffers and page-locked landing areas
        frames = b.frames
        batches.append(b)
    for nt in (1, 2, 4):
        recs = [[] for _ in range(nt)]
        th = [threading.Thread(target=serve, args=(batches[i], files, a.rounds, recs[i])) for i in range(nt)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        allr = np.array([r for rr in recs for r in rr])
        print(json.dumps({"threads": nt, "kernel": a.kernel, "Msamples_per_s": round(frames * a.rounds * nt / dt / 1e6, 1),
                          "wall_ms": round(dt * 1e3, 2),
                          "phase_ms_mean": {k: round(float(v), 3) for k, v in zip(PHASES, allr.mean(axis=0))}}),
              flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
