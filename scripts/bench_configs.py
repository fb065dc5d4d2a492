#!/usr/bin/env python3
"""Device-resident decode rate of the BASELINE.json configurations other than the
headline one (bench.py runs config 2).  Not part of the driver contract: the
numbers go into DESIGN.md.

  C1  WvDemo file (20 s 16-bit stereo, default terms): decode + the
      WavpackFormatSamples epilogue, one file
  C3  4,096 x 44,100-frame 24-bit stereo high-mode blocks (16 terms)
  C4  1,024 x 22,050-frame float32 hybrid (FloatUtils.float_values path)
  C5  mixed corpus sample (NFILES files of the 100k corpus; mono/stereo,
      16/24-bit, DSD modes 0/1/3)

Each line: kernel ms (hipEvents, mean of K decodes with input resident in HBM),
Mframes/s, CRC errors, and a lossless round-trip check where one exists.
usage: python scripts/bench_configs.py [c1 c3 c4 c5] [--c3-blocks N] [--c5-files N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# as bench.py: more hardware queues than the boxes' exported 4 (set before HIP starts)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("WVG_BENCH_HW_QUEUES", "24")
sys.path.insert(0, ROOT)

from synth import corpora  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402


def run(name, files, pcm=None, iters=5, fmt=False):
    t0 = time.perf_counter()
    b = DecodeBatch(4096)
    b.set_kernel(KERNEL)
    b.add_files(files)  # host framing on worker threads
    t_frame = time.perf_counter() - t0
    b.upload()
    b.decode()
    b.sync()
    ms = b.time(iters)
    # per launch group: end time of each group's kernels from the decode's start
    # (each group on its own stream), median of 3 single decodes
    group_ms = None
    if hasattr(b._L, "wvg_batch_group_times"):  # (absent from older A/B builds)
        b.set_timing(True)
        gts = []
        for _ in range(3):
            b.decode()
            b.sync()
            gts.append(b.group_times())
        b.set_timing(False)
        group_ms = {g: round(float(np.median([t[g] for t in gts])), 3) for g in gts[0]}
    out = b.download()
    crc = sum(b.result(i).crc_errors for i in range(len(files)) if b.infos[i].open_ok)
    from wavpackdecoder_amd import _lib as _LL
    redone = int(np.count_nonzero(b.block_status() & _LL.WVG_ST_REDONE))
    ok = None
    if pcm is not None:
        ok = bool(np.array_equal(out, pcm.reshape(-1)))
    fmt_ms = None
    if fmt:
        t = time.perf_counter()
        for _ in range(iters):
            b.format()
        b.sync()
        fmt_ms = (time.perf_counter() - t) / iters * 1e3
    line = {"config": name, "files": len(files), "blocks": b.num_blocks, "frames": b.frames,
            "compressed_bytes": b.bytes_in, "kernel_ms": round(ms, 3),
            "Mframes_per_s": round(b.frames / ms / 1e3, 1), "crc_errors": int(crc), "redone_blocks": redone,
            "lossless_roundtrip": ok, "host_framing_s": round(t_frame, 3), "group_end_ms": group_ms}
    if INFLIGHT > 1:
        # the same batch as INFLIGHT copies on their own streams, decodes issued
        # round-robin (bench.py's --inflight): throughput with launches overlapping
        copies = [b]
        for _ in range(INFLIGHT - 1):
            c = DecodeBatch(4096)
            c.set_kernel(KERNEL)
            c.add_files(files)
            c.upload()
            copies.append(c)
        steps = 4 * INFLIGHT
        for c in copies:
            c.decode()
        for c in copies:
            c.sync()
        t = time.perf_counter()
        for k in range(steps):
            copies[k % INFLIGHT].decode()
        for c in copies:
            c.sync()
        dt = time.perf_counter() - t
        line["inflight"] = INFLIGHT
        line["Mframes_per_s_inflight"] = round(b.frames * steps / dt / 1e6, 1)
        for c in copies[1:]:
            c.close()
    if fmt_ms is not None:
        line["format_epilogue_ms_wall"] = round(fmt_ms, 3)
    if CPU_THREADS:
        line["cpu_baseline_Mframes_per_s"] = round(cpu_rate(files), 1)
        line["cpu_threads"] = CPU_THREADS
    print(json.dumps(line), flush=True)
    b.close()


def run_wvc(name, wv, wvc, iters=5, exact=None):
    """A hybrid file with its .wvc: device time of the exact decode (one batch; and
    INFLIGHT copies in flight), the output checked against `exact` when given."""
    def mk():
        c = DecodeBatch(4096)
        c.set_kernel(KERNEL)
        c.add_file(wv, wvc=wvc)
        c.upload()
        return c
    b = mk()
    b.decode()
    b.sync()
    ms = b.time(iters)
    out = b.download()
    r = b.result(0)
    st = b.block_status()
    line = {"config": name, "files": 1, "blocks": b.num_blocks, "frames": b.frames,
            "compressed_bytes": b.bytes_in, "kernel": KERNEL, "kernel_ms": round(ms, 3),
            "Mframes_per_s": round(b.frames / ms / 1e3, 1), "crc_errors": int(r.crc_errors),
            "redone_blocks": int(((st & 0x200) != 0).sum()),
            "exact": None if exact is None else bool(np.array_equal(out[: exact.size], exact))}
    if INFLIGHT > 1:
        copies = [b] + [mk() for _ in range(INFLIGHT - 1)]
        steps = 4 * INFLIGHT
        for c in copies:
            c.decode()
        for c in copies:
            c.sync()
        t = time.perf_counter()
        for k in range(steps):
            copies[k % INFLIGHT].decode()
        for c in copies:
            c.sync()
        line["inflight"] = INFLIGHT
        line["Mframes_per_s_inflight"] = round(b.frames * steps / (time.perf_counter() - t) / 1e6, 1)
        for c in copies[1:]:
            c.close()
    print(json.dumps(line), flush=True)
    b.close()


CPU_THREADS = 0
INFLIGHT = 1
KERNEL = "two_wave"


def cpu_rate(files):
    """The oracle (C restatement of the reference path, 4096-frame calls) over the
    same files on CPU_THREADS host threads (multi-block files split at block
    boundaries so every thread has work); test infrastructure used as the
    CPU baseline only."""
    from concurrent.futures import ThreadPoolExecutor

    import bench
    from oracle import oracle as O
    parts = []
    for f in files:
        parts += bench.split_blocks(f, max(1, CPU_THREADS // max(len(files), 1)))
    with ThreadPoolExecutor(max_workers=CPU_THREADS) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(lambda p: O.decode_file(p, chunk=4096, max_frames=len(p) * 8), parts))
        dt = time.perf_counter() - t0
    return sum(r.frames for r in res) / dt / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c1", "c3", "c4", "c5"])
    ap.add_argument("--c3-blocks", type=int, default=4096)
    ap.add_argument("--c3-copies", type=int, default=1)
    ap.add_argument("--c5-files", type=int, default=4000)
    ap.add_argument("--list-blocks", type=int, default=1024, help="blocks per batch of the 'lists' config")
    ap.add_argument("--lists", default="", help="'lists' config: comma-separated name prefixes (default all)")
    ap.add_argument("--dsd-files", type=int, default=64, help="files per DSD mode batch (one block each)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="also time the oracle on this many host threads")
    ap.add_argument("--inflight", type=int, default=1, help="also time this many copies of each batch in flight")
    ap.add_argument("--kernel", choices=("two_wave", "lane", "auto"), default="two_wave",
                    help="PCM kernel for the term-set groups (wvg_batch_set_kernel)")
    a = ap.parse_args()
    global CPU_THREADS, INFLIGHT, KERNEL
    CPU_THREADS = a.cpu_threads
    INFLIGHT = a.inflight
    KERNEL = a.kernel
    from wavpackdecoder_amd import _lib
    import wavpackdecoder_amd.api as api
    api._ctx = _lib.lib().wvg_open(0)
    for c in a.configs:
        if c == "c1":
            pcm, data = corpora.c1()
            run("C1 WvDemo file 20 s 16-bit stereo default", [data], pcm, fmt=True)
        elif c == "c3":
            # BASELINE config 3 at full size: 4,096 distinct 44,100-frame blocks (encoded on
            # every host core; --c3-copies > 1 repeats a smaller set instead)
            pcm, data = corpora.c3(nblocks=a.c3_blocks, return_pcm=True)
            run(f"C3 {a.c3_copies} x {a.c3_blocks} x 44100 24-bit stereo high (16 terms)", [data] * a.c3_copies,
                np.concatenate([pcm.reshape(-1)] * a.c3_copies))
            del pcm, data
        elif c == "c4":
            run("C4 1024 x 22050 float32 hybrid+bitrate", [corpora.c4()])
        elif c == "c4wvc":  # C4 with its .wvc correction files: the exact decode (generic kernel)
            wv, wvc, ll = corpora.c4_wvc()
            # (the exactness check: the same mantissas encoded losslessly, decoded here too)
            r = DecodeBatch(4096)
            r.add_file(ll)
            r.decode()
            ref = r.download().copy()
            r.close()
            run_wvc("C4 1024 x 22050 float32 hybrid+bitrate + .wvc (exact)", wv, wvc, exact=ref)
        elif c == "c5":
            run(f"C5 mixed corpus, files 0..{a.c5_files - 1}", corpora.c5(a.c5_files))
        elif c == "lists":
            # C2's shape (1,024 x 22,050-frame 16-bit stereo blocks) under term lists with and
            # without a lane instantiation: the run-time list kernel (wv_pcm_lane_rt) against
            # the compile-time ones on the same PCM
            from synth import wvsynth as S
            pcm = corpora.c2_pcm(a.list_blocks)
            lists = {"default (instantiated)": S.TERMS_DEFAULT, "alt5 (run-time)": [18, 18, 2, 3, -1],
                     "high16 (instantiated)": S.TERMS_HIGH,
                     "alt16 (run-time)": [18, 18, 2, 3, -1, 18, 2, 4, 7, 5, 3, 6, 8, -2, 17, 2],
                     "high10 (run-time)": S.TERMS_HIGH10}
            for nm, t in lists.items():
                if a.lists and not any(nm.startswith(x) for x in a.lists.split(",")):
                    continue
                data = S.encode_pcm_parallel(pcm, S.EncParams(terms=t, block_samples=22050, joint_stereo=True))
                run(f"C2-shape {a.list_blocks} x 22050 16-bit stereo, list {nm}", [data], pcm)
        elif c == "hykinds":
            # C2's PCM (--list-blocks x 22,050 frames, 16-bit stereo, default terms) as the PCM kinds
            # the round-6 lanes added, beside their neighbours: lossless (C2), hybrid with and without
            # HYBRID_BITRATE, INT32 hybrid (zeros) and INT32 lossless with a shift-only fixup
            from synth import wvsynth as S
            pcm = corpora.c2_pcm(a.list_blocks)
            base = dict(terms=S.TERMS_DEFAULT, block_samples=22050, joint_stereo=True)
            kinds = {"lossless (C2)": (pcm, dict()),
                     "hybrid + bitrate": (pcm, dict(hybrid=True, hybrid_bitrate=True, bitrate_x256=896)),
                     "hybrid, no bitrate": (pcm, dict(hybrid=True, hybrid_bitrate=False, bitrate_x256=896)),
                     "int32 hybrid zeros=3": (S.int32_layout(pcm, zeros=3, seed=5),
                                              dict(bytes_per_sample=4, hybrid=True, hybrid_bitrate=True,
                                                   bitrate_x256=896, int32_zeros=3)),
                     "int32 lossless shift=4": (S.int32_layout(pcm, zeros=4, seed=6),
                                                dict(bytes_per_sample=4, int32_zeros=4))}
            for nm, (x, kw) in kinds.items():
                if a.lists and not any(nm.startswith(y) for y in a.lists.split(",")):
                    continue
                data = S.encode_pcm_parallel(x, S.EncParams(**base, **kw))
                run(f"{a.list_blocks} x 22050 16-bit stereo as {nm}", [data], x if not kw.get("hybrid") else None)
        elif c.startswith("dsd"):  # dsd0 / dsd1 / dsd3: N stereo files of one 22,050-frame block in one mode
            from synth import wvsynth as S
            mode = int(c[3:])
            # 64 distinct files repeated: a DSD block's cost does not depend on its content's identity
            base = [S.encode_dsd(S.dsd_random_like(22050, 2, seed=i, density=0.5),
                                 S.DsdParams(nch=2, mode=mode, block_samples=22050)) for i in range(min(64, a.dsd_files))]
            files = [base[i % len(base)] for i in range(a.dsd_files)]
            run(f"DSD mode {mode}: {a.dsd_files} files x 22050 frames stereo", files)


if __name__ == "__main__":
    main()
