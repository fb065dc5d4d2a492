"""bench.py's pipelined PCM request stream (T request threads, a ring of D batches
each: the next D-1 requests framed, uploaded and decoding before the current one's
format + PCM download) with every call of every request timed in its thread, so the
phase that keeps the stream below the PCIe bound shows.

usage: python3 scripts/pipe2_probe.py [--threads 1,2,4,6] [--depth 2,3] [--rounds 6]
       [--kernel auto] [--device-framing]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PHASES = ("reset", "add_files", "upload", "decode_issue", "format_issue", "download_pcm")


def serve_ring(bb, files, rounds, rec, dev):
    """Requests 0..rounds-1 on the ring bb (request k on bb[k % D]): requests k+1..k+D-1
    are started before request k's format + download."""
    D = len(bb)

    def start(x, t):
        t.append(time.perf_counter())
        x.reset()
        t.append(time.perf_counter())
        if dev:
            x.add_files_device(files)
        else:
            x.add_files(files)
        t.append(time.perf_counter())
        x.upload()
        t.append(time.perf_counter())
        x.decode()
        t.append(time.perf_counter())

    ts = [[] for _ in range(rounds)]
    for k in range(min(D - 1, rounds)):
        start(bb[k % D], ts[k])
    for k in range(rounds):
        if k + D - 1 < rounds:
            start(bb[(k + D - 1) % D], ts[k + D - 1])
        t = ts[k]
        t0 = time.perf_counter()
        bb[k % D].format()
        t1 = time.perf_counter()
        bb[k % D].download_pcm(pinned=True)
        t2 = time.perf_counter()
        rec.append(list(np.diff(t)) + [t1 - t0, t2 - t1])


def serve_async(bb, files, rounds, rec, dev):
    """bench.py's ring: every call of request k issued back to back (the PCM download
    queued, wvg_batch_download_pcm_async); the thread waits only for request k - D."""
    D = len(bb)
    for k in range(rounds):
        x = bb[k % D]
        t = [time.perf_counter()]
        if k >= D:
            x.sync()
        t.append(time.perf_counter())
        x.reset()
        (x.add_files_device if dev else x.add_files)(files)
        t.append(time.perf_counter())
        x.upload()
        t.append(time.perf_counter())
        x.decode()
        t.append(time.perf_counter())
        x.format()
        t.append(time.perf_counter())
        x.download_pcm_async()
        t.append(time.perf_counter())
        rec.append(list(np.diff(t)))
    for k in range(max(0, rounds - D), rounds):
        bb[k % D].sync()


def serve_pc(pool, files, total, producers, consumers, add_threads=0):
    """Producer/consumer server: `producers` threads take a free batch, frame, upload, decode
    and format a request on it (no call waits for the device) and queue it; `consumers`
    threads take the queued batches in order and download their PCM (page-locked, blocking),
    then free the batch.  Returns (wall seconds, requests)."""
    import queue
    free, ready = queue.Queue(), queue.Queue()
    for b in pool:
        free.put(b)
    left = [total]
    lock = threading.Lock()

    def produce():
        while True:
            with lock:
                if left[0] == 0:
                    return
                left[0] -= 1
            x = free.get()
            x.reset()
            x.add_files(files, threads=add_threads)
            x.upload()
            x.decode()
            x.format()
            ready.put(x)

    done = [0]

    def consume():
        while True:
            x = ready.get()
            if x is None:
                return
            x.download_pcm(pinned=True)
            with lock:
                done[0] += 1
            free.put(x)

    ps = [threading.Thread(target=produce) for _ in range(producers)]
    cs = [threading.Thread(target=consume) for _ in range(consumers)]
    t0 = time.perf_counter()
    for t in ps + cs:
        t.start()
    for t in ps:
        t.join()
    for _ in cs:
        ready.put(None)
    for t in cs:
        t.join()
    return time.perf_counter() - t0, done[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4,6")
    ap.add_argument("--depth", default="2")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--device-framing", action="store_true")
    ap.add_argument("--async-download", action="store_true", help="every call back to back (serve_async)")
    ap.add_argument("--pc", default="", help="producer/consumer server: comma list of P:C:pool configs")
    ap.add_argument("--switch", type=float, default=0.0, help="sys.setswitchinterval (0: Python's default)")
    a = ap.parse_args()
    if a.switch > 0:
        sys.setswitchinterval(a.switch)
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    _, c2 = corpora.c2(return_pcm=True)
    files = [c2]
    nts = [int(x) for x in a.threads.split(",")]
    depths = [int(x) for x in a.depth.split(",")]
    batches = []
    for _ in range(max(depths) * max(nts)):
        b = DecodeBatch(4096)
        b.set_kernel(a.kernel)
        batches.append(b)
    frames = None
    for i in range(0, len(batches), 2):  # warm: buffers and page-locked landing areas
        serve_ring(batches[i:i + 2], files, 2, [], a.device_framing)
        frames = batches[i].frames
    for cfg in [x for x in a.pc.split(",") if x]:
        P, C, N, *T = (int(v) for v in cfg.split(":"))  # (P:C:pool[:add_files threads, 0: the library's])
        while len(batches) < N:
            b = DecodeBatch(4096)
            b.set_kernel(a.kernel)
            serve_ring([b], files, 1, [], a.device_framing)
            batches.append(b)
        dt, nreq = serve_pc(batches[:N], files, a.rounds * N, P, C, T[0] if T else 0)
        print(json.dumps({"producers": P, "consumers": C, "pool": N, "add_threads": T[0] if T else 0,
                          "kernel": a.kernel, "requests": nreq,
                          "Msamples_per_s": round(frames * nreq / dt / 1e6, 1),
                          "ms_per_request": round(dt * 1e3 / nreq, 3)}), flush=True)
    if a.pc:
        return
    for D in depths:
        for nt in nts:
            recs = [[] for _ in range(nt)]
            fn = serve_async if a.async_download else serve_ring
            th = [threading.Thread(target=fn, args=(batches[D * i:D * i + D], files, a.rounds, recs[i],
                                                    a.device_framing)) for i in range(nt)]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = time.perf_counter() - t0
            allr = np.array([r for rr in recs for r in rr]) * 1e3
            names = ("wait", "reset+add_files", "upload", "decode", "format", "download_issue") if a.async_download \
                else PHASES
            print(json.dumps({"threads": nt, "depth": D, "kernel": a.kernel, "device_framing": a.device_framing,
                              "async_download": a.async_download,
                              "Msamples_per_s": round(frames * a.rounds * nt / dt / 1e6, 1),
                              "ms_per_request": round(dt * 1e3 / (a.rounds * nt), 3),
                              "phase_ms_mean": {k: round(float(v), 3) for k, v in zip(names, allr.mean(axis=0))}}),
                  flush=True)
    for b in batches:
        b.close()


if __name__ == "__main__":
    main()
