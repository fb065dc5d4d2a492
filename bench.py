#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X.

metric : Msamples/sec decoded (node) + HBM GB/s, batched 44.1 kHz/16-bit stereo blocks
step   : one decode of the config-2 batch (1,024 independent WavPack blocks x
         22,050 frames, 16-bit stereo, fast terms {17,17}) already resident in
         HBM -> int32 PCM in HBM (the WavpackUnpackSamples output contract)
N GPUs : one process per GPU.  Under torch.distributed.run the ranks come from
         the environment (WORLD_SIZE must equal --gpus); `python bench.py --gpus N`
         alone spawns the N rank processes itself (the parent never touches a GPU).
         --workload c2 (default, weak scaling): every rank decodes its own copy of
         the C2 batch, so per-GPU work is identical at every N.
         --workload c5 (strong scaling): a fixed slice of the mixed corpus (C5) is
         file-partitioned across the ranks (LPT on estimated device cost).
         No data-path collective: only a CPU (gloo) barrier and max/sum reduces.
value  : frames decoded by all ranks / max-over-ranks wall time of the K steps.
         Steps are issued round-robin over --inflight copies of the batch, each
         with its own device buffers and HIP stream, so consecutive steps overlap
         on the device as in a decode server with several batches in flight:
         every step is still one complete decode of the whole batch into its own
         output.  The measured kernel is the lane-per-block one (--kernel lane,
         wv_lane.h; the library's default WVG_KERNEL_AUTO picks it once batches
         overlap): a block is one serial entropy chain, one lane decodes it, a
         batch of 1,024 blocks is 9 workgroups of 4 waves (two parser/reconstruction
         pairs of 64 lane slots each, the lane order's gap slots included: SQ_WAVES
         36; one workgroup per CU), so the chip holds many batches at once -- the
         default keeps min(K, 20) in flight.  --kernel two_wave is the
         one-workgroup-per-block kernel (lowest latency for a batch alone; best at
         3 in flight), measured beside it in "two_wave".  The line also reports
         the same K steps run one batch at a time ("value_one_batch_at_a_time")
         and the per-launch device times (launch_ms).

Before the timed region every copy's output is overwritten with 0x7F bytes and its
block statuses marked unwritten (wvg_batch_poison); right after it every in-flight
copy -- whose last decode is a timed one -- is downloaded and checked (C2): its int32
output must equal the generator's PCM bit for bit, every block's status must have
been stored by a decode, every block's CRC must match (crc_errors == 0), and the
blocks handed back by the lane kernel to its fallback (WVG_ST_REDONE) are counted
("redo_blocks").

Also printed in the same JSON line:
  roofline     : algorithmic bytes per launch (compressed bytes in + int32
                 out) / mean device time per launch measured
                 with hipEvents on the decode stream, vs 8 TB/s HBM peak.
  cpu_baseline : the oracle (C restatement of the reference algorithm, kind
                 "port") on rank 0 only: one decoder context per thread on the
                 physical cores of one socket that this process may use
                 (BASELINE.md:35-38), plus a single-thread figure.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# one stream per launch group and several batches in flight: more hardware
# queues than HIP's default 4, which the GPU boxes export -- a stream beyond the
# process's queues shares one, and kernels of one queue run one after another, so
# the batches in flight would serialise to 4.  Set before anything initialises HIP
# (wvg_open only fills it in when the host left it unset).  WVG_BENCH_HW_QUEUES
# overrides; at most 32.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("WVG_BENCH_HW_QUEUES", "24")

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "Msamples/sec decoded (node) + HBM GB/s, batched 44.1kHz/16-bit stereo blocks"


# ---------------------------------------------------------------------------
# process layout
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (children,
    never an exec; this parent initialises nothing on the GPU) and return the
    worst exit code.  Rank 0 prints the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def _dist(gpus: int):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}")
    pg = None
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=ws)  # CPU barrier + timing reduces only
        pg = dist
    return ws, rank, local, pg


def _barrier(pg):
    if pg is not None:
        pg.barrier()


def _reduce(pg, v: float, op: str) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX if op == "max" else pg.ReduceOp.SUM)
    return float(t.item())


def _gather(pg, v: float, ws: int) -> list[float]:
    if pg is None:
        return [v]
    import torch
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(ws)]
    pg.all_gather(out, torch.tensor([v], dtype=torch.float64))
    return [float(t.item()) for t in out]


# ---------------------------------------------------------------------------
# workload helpers
# ---------------------------------------------------------------------------
def split_blocks(data: bytes, parts: int):
    """Split a multi-block .wv file at block boundaries into `parts` files."""
    offs = []
    i = 0
    n = len(data)
    while i + 32 <= n:
        if data[i:i + 4] != b"wvpk":
            break
        ck = int.from_bytes(data[i + 4:i + 8], "little")
        offs.append(i)
        i += ck + 8
    offs.append(n)
    nb = len(offs) - 1
    per = (nb + parts - 1) // parts
    return [data[offs[k]:offs[min(k + per, nb)]] for k in range(0, nb, per)]


def algorithmic_bytes(data: bytes) -> int:
    """sum(ckSize + 8) + sum(block_samples * nch_out * 4) over the
    decoded blocks (INITIAL blocks; nch_out from the MONO_FLAG)."""
    i, tot = 0, 0
    while i + 32 <= len(data) and data[i:i + 4] == b"wvpk":
        ck = int.from_bytes(data[i + 4:i + 8], "little")
        bs = int.from_bytes(data[i + 20:i + 24], "little")
        flags = int.from_bytes(data[i + 24:i + 28], "little")
        nch = 1 if flags & 4 else 2
        tot += ck + 8 + bs * nch * 4
        i += ck + 8
    return tot


def pmc_traffic(kernel_substr: str = "wv_pcm_2wave<17, 17>"):
    """Per-launch HBM bytes of the bench kernel from the newest profiles/<tag>_pmc.json
    (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, scripts/profile.sh + scripts/pmc_to_profile.py)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json"))):
        with open(path) as f:
            d = json.load(f)
        if kernel_substr in d.get("kernel", ""):
            best = (path, d)
    if best is None:
        return None, None
    return float(best[1]["traffic_bytes_per_launch"]), os.path.relpath(best[0], ROOT)


# the bench kernel's name as rocprofv3 reports it (profiles/<tag>_pmc.json "kernel")
KERNEL_NAMES = {"lane": "wv_pcm_lane<false, 0, 17, 17>", "two_wave": "wv_pcm_2wave<17, 17>"}


def c5_end_to_end(sets, slices) -> dict:
    """C5 end to end on warm batches: per slice, host framing into the page-locked blob
    (wvg_batch_add_files, the library's framing threads), the upload, the decode,
    WavpackFormatSamples on the device and the PCM download into page-locked memory.
    `serial`: one slice at a time, each phase timed (synchronised after each).
    `pipelined`: one host thread per slice batch of the first copy set, two batches each
    when a second copy exists (the next slice framed, uploaded and decoding before the
    current one's format + download), every slice of the rank once; the wall time of
    the whole pass.  Reported beside `value` (device-resident), never as it."""
    import threading
    bats = sets[0]
    for bb in bats:  # (the PCM image and its page-locked landing buffer: allocated untimed)
        bb.format()
        bb.download_pcm(pinned=True)
    ph = {"framing": 0.0, "upload": 0.0, "decode": 0.0, "format_download": 0.0}
    frames = 0
    t_all = time.perf_counter()
    for bb, sl in zip(bats, slices):
        t0 = time.perf_counter()
        bb.reset()
        bb.add_files(sl)
        t1 = time.perf_counter()
        bb.upload()
        t2 = time.perf_counter()
        bb.decode()
        bb.sync()
        t3 = time.perf_counter()
        bb.format()
        bb.download_pcm(pinned=True)
        t4 = time.perf_counter()
        for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            ph[k] += v
        frames += bb.frames
    t_serial = time.perf_counter() - t_all
    pcm_bytes = sum(int(bb._L.wvg_batch_pcm_bytes(bb._b)) for bb in bats)
    in_bytes = sum(bb.bytes_in for bb in bats)
    # pipelined: thread i serves slices i, i + T, ... with its one or two batches
    T = len(bats)
    spare = sets[1] if len(sets) > 1 else [None] * T

    def serve(i, dev=False):
        mine = list(range(i, len(slices), T))
        pair = (bats[i], spare[i]) if spare[i] is not None else (bats[i],)

        def start(b, j):
            b.reset()
            (b.add_files_device if dev else b.add_files)(slices[j])
            b.upload()
            b.decode()
        start(pair[0], mine[0])
        for k, j in enumerate(mine):
            if k + 1 < len(mine) and len(pair) > 1:
                start(pair[(k + 1) % 2], mine[k + 1])
            cur = pair[k % len(pair)]
            cur.format()
            cur.download_pcm(pinned=True)
            if k + 1 < len(mine) and len(pair) == 1:
                start(pair[0], mine[k + 1])
    def pipelined(dev):
        th = [threading.Thread(target=serve, args=(i, dev)) for i in range(T)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0
    t_pipe = pipelined(False)
    t_pipe_dev = pipelined(True)  # the header / sub-block walk in kernels (wvg_batch_add_files_device)
    return {"frames": int(frames), "compressed_bytes": int(in_bytes), "pcm_bytes": int(pcm_bytes),
            "serial": {"Msamples_s": round(frames / t_serial / 1e6, 1), "ms": round(t_serial * 1e3, 2),
                       "phase_ms": {k: round(v * 1e3, 2) for k, v in ph.items()}},
            "pipelined": {"Msamples_s": round(frames / t_pipe / 1e6, 1), "ms": round(t_pipe * 1e3, 2),
                          "threads": T, "batches_per_thread": 2 if len(sets) > 1 else 1},
            "pipelined_device_framing": {"Msamples_s": round(frames / t_pipe_dev / 1e6, 1),
                                         "ms": round(t_pipe_dev * 1e3, 2)},
            "what": "warm batches: host framing (wvg_batch_add_files) + upload + decode + device "
                    "WavpackFormatSamples + PCM download into page-locked memory, every slice once"}


# C5: batches in flight the copies aim at (each batch takes up to 3 streams while others
# run, within the process's hardware queues: wv_api.cpp wvg_batch_decode)
C5_BATCHES_IN_FLIGHT = 8


def c5_copies(args, nslices: int) -> int:
    """Copies of a rank's C5 batches: --c5-copies, else enough that about
    C5_BATCHES_IN_FLIGHT batches are in flight (at least 1, at most --steps)."""
    c = args.c5_copies if args.c5_copies else max(1, C5_BATCHES_IN_FLIGHT // max(1, nslices))
    return max(1, min(c, args.steps))


def verify(batches, pcm) -> dict:
    """Download every batch copy and check what its last decode produced: C2's
    int32 output equals the generator's PCM, no CRC error in any file
    (WavPackUtils.cs:273-275), and no block went through the lane kernel's
    fallback (WVG_ST_REDONE).  Raises on any failure."""
    from wavpackdecoder_amd import _lib
    crc = redo = blocks = unwritten = 0
    for bb in batches:
        out = bb.download()
        if pcm is not None:
            assert np.array_equal(out, pcm.reshape(-1)), "decoded PCM differs from the generator's"
        st = bb.block_status()
        unwritten += int(np.count_nonzero(st & _lib.WVG_ST_UNWRITTEN))
        crc += sum(bb.result(i).crc_errors for i in range(len(bb.infos)) if bb.infos[i].open_ok)
        redo += int(np.count_nonzero(st & _lib.WVG_ST_REDONE))
        blocks += int(st.size)
    assert unwritten == 0, f"{unwritten} blocks whose status no decode stored"
    assert crc == 0, f"{crc} CRC errors in a synthetic corpus"
    return {"copies": len(batches), "blocks": blocks, "crc_errors": crc, "redo_blocks": redo,
            "unwritten_blocks": unwritten,
            # (C5 has no generator PCM beside it: its check is every block's CRC over the decoded samples)
            "pcm_equal": True if pcm is not None else None}


# ---------------------------------------------------------------------------
# CPU baseline (BASELINE.md:35-38)
# ---------------------------------------------------------------------------
def cpu_topology() -> dict:
    """Physical cores per socket and sockets (lscpu), CPUs this process may run on
    (sched_getaffinity) and the lease's worker-thread share (OMP_NUM_THREADS)."""
    topo = {"model": None, "sockets": None, "cores_per_socket": None, "threads_per_core": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "Model name":
                topo["model"] = v
            elif k == "Socket(s)":
                topo["sockets"] = int(v)
            elif k == "Core(s) per socket":
                topo["cores_per_socket"] = int(v)
            elif k == "Thread(s) per core":
                topo["threads_per_core"] = int(v)
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    topo["affinity_cpus"] = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    topo["lease_threads"] = int(share) if share and share.isdigit() else None
    return topo


def cpu_decode_rate(data: bytes, threads: int, reps: int):
    """Oracle (C port of the reference path) on `threads` host threads, one decoder
    context per thread over its share of the blocks; ctypes drops the GIL."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    parts = split_blocks(data, threads)
    frames = 0
    times = []
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for _ in range(reps):
            t0 = time.perf_counter()
            res = list(ex.map(lambda p: O.decode_file(p, chunk=4096, max_frames=len(p) * 2), parts))
            times.append(time.perf_counter() - t0)
            frames = sum(r.frames for r in res)
            assert all(r.crc_errors == 0 for r in res)
    t = float(np.median(times))
    return frames / t / 1e6, t, frames


def cpu_baseline_c5(files, force_threads: int | None, sample: int = 400):
    """C5's CPU baseline: the oracle over a bounded sample of the rank's files (the
    first `sample`) on the lease's threads, one decoder context per file."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    topo = cpu_topology()
    cps = topo["cores_per_socket"] or topo["affinity_cpus"]
    usable = min(topo["affinity_cpus"], topo["lease_threads"] or topo["affinity_cpus"])
    threads = force_threads or max(1, min(cps, usable))
    part = files[:sample]
    with ThreadPoolExecutor(max_workers=threads) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(lambda f: O.decode_file(f, chunk=4096, max_frames=len(f) * 8), part))
        dt = time.perf_counter() - t0
    fr = sum(r.frames for r in res)
    v = fr / dt / 1e6
    return {"value": round(v, 2), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle over the rank's first {len(part)} C5 files ({fr} frames) on {threads} threads, "
                      "4096-frame calls",
            "socket_scaled": round(v / threads * cps, 2), "cores_per_socket": cps}


def cpu_baseline(data: bytes, reps: int, force_threads: int | None):
    topo = cpu_topology()
    cps = topo["cores_per_socket"] or topo["affinity_cpus"]
    usable = min(topo["affinity_cpus"], topo["lease_threads"] or topo["affinity_cpus"])
    threads = force_threads or max(1, min(cps, usable))
    capped = threads < cps
    v, t, fr = cpu_decode_rate(data, threads, reps)
    # single thread on a bounded sample (~1/8 of the batch's blocks)
    sample = split_blocks(data, 8)[0]
    v1, t1, fr1 = cpu_decode_rate(sample, 1, max(1, min(reps, 3)))
    per_core = v1
    socket_est = per_core * cps  # linear per-core scaling to one socket (an upper bound for the CPU)
    return {
        "value": round(v, 2), "unit": "Msamples/s", "cores": threads, "kind": "port",
        "sample": (f"oracle (C restatement of the C# path, -O2) decoding the full C2 file ({fr} frames) split at "
                   f"block boundaries over {threads} threads, 4096-frame calls, median of {reps} runs; single "
                   f"thread on {fr1} frames"),
        "single_thread": round(v1, 2),
        "socket": {"model": topo["model"], "sockets": topo["sockets"], "cores_per_socket": cps,
                   "threads_per_core": topo["threads_per_core"], "affinity_cpus": topo["affinity_cpus"],
                   "lease_threads": topo["lease_threads"],
                   "capped_by_lease": capped,
                   "per_core_scaled_to_socket": round(socket_est, 2)},
    }


# ---------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------
def run_selftest(args) -> None:
    """--selftest-dist: the process layout and the host reductions alone (no GPU):
    what tests/test_bench_spawn.py checks on CPU with gloo."""
    ws, rank, local, pg = _dist(args.gpus)
    _barrier(pg)
    tot = _reduce(pg, float(rank + 1), "sum")
    mx = _reduce(pg, float(rank), "max")
    allv = _gather(pg, float(10 * rank + local), ws)
    if rank == 0:
        print(json.dumps({"n_gpus": ws, "sum": tot, "max": mx, "gathered": allv}), flush=True)
    if pg is not None:
        pg.destroy_process_group()


def run_rank(args) -> None:
    if args.selftest_dist:
        return run_selftest(args)
    ws, rank, local, pg = _dist(args.gpus)

    from synth import corpora
    from wavpackdecoder_amd import _lib
    import wavpackdecoder_amd.api as api
    from wavpackdecoder_amd.api import DecodeBatch

    pcm = None
    if args.workload == "c2":
        # every rank decodes its own copy of the C2 batch (identical per-GPU work at every N)
        pcm, data = corpora.c2(nblocks=args.blocks, block=args.block_frames, return_pcm=True)
        files = [data]
        workload = "C2: 1024-block batch, 16-bit stereo 'fast' {17,17}, joint stereo, 44.1 kHz"
        scaling = "weak"
    else:
        from wavpackdecoder_amd import shard
        costs = [corpora.c5_cost(i) for i in range(args.c5_files)]
        # (--c5-share N:r: decode rank r's share of an N-way split in this one process --
        # the per-rank times of an N-GPU run measured one share at a time on one GPU,
        # scripts/c5_scaling.py)
        pw, pr = (int(x) for x in args.c5_share.split(":")) if args.c5_share else (ws, rank)
        mine = shard.partition(costs, pw)[pr]
        t_gen = time.perf_counter()
        files = corpora.c5_files(mine, progress=rank == 0)
        print(f"bench: C5 rank {rank}: {len(files)} files generated in {time.perf_counter() - t_gen:.1f} s",
              file=sys.stderr, flush=True)
        workload = f"C5: files 0..{args.c5_files - 1} of the mixed corpus, LPT file partition over {ws} GPU(s)"
        if args.c5_share:
            workload += f"; share {pr} of an {pw}-way split (--c5-share)"
        scaling = "strong"
    # C5: the rank's files in slices of at most --c5-batch files (one batch each), and
    # --c5-copies copies of that set of batches; step k decodes every slice of copy
    # k % copies, so consecutive steps overlap on the device (each step is still one
    # complete decode of the rank's files).  C2: --inflight copies of the one batch.
    multi = args.workload == "c5"
    slices = [files[k:k + args.c5_batch] for k in range(0, len(files), args.c5_batch)] if multi else [files]

    L = _lib.lib()
    # (WVG_BENCH_SAME_DEVICE=1: every rank on device 0 -- the multi-rank path rehearsed on a
    # one-GPU box, tests/test_gpu_ranks.py; the driver's N-GPU runs leave it unset)
    api._ctx = L.wvg_open(0 if os.environ.get("WVG_BENCH_SAME_DEVICE") == "1" else local)
    if not api._ctx:
        raise SystemExit("no GPU")

    # `inflight` copies of the batch, each with its own device buffers and stream:
    # step k decodes copy k % inflight, so consecutive steps overlap on the device
    # the way a decode server keeps several batches in flight (every step is still
    # one complete decode of the whole batch into its own output)
    if multi:
        copies = c5_copies(args, len(slices))
    else:
        copies = args.inflight if args.inflight else (20 if args.kernel == "lane" else 3)
        copies = max(1, min(copies, args.steps))
    sets = []
    for _ in range(copies):
        cur = []
        for sl in slices:
            bb = DecodeBatch(4096)
            bb.set_kernel(args.kernel)
            bb.add_files(sl)  # host framing on worker threads
            bb.upload()
            cur.append(bb)
        sets.append(cur)
    batches = [bb for cur in sets for bb in cur]
    b = batches[0]
    frames_rank = sum(bb.frames for bb in sets[0])
    alg_bytes = sum(algorithmic_bytes(f) for f in files)

    def step(k):
        for bb in sets[k % copies]:
            bb.decode()
    extras = not multi and not args.timed_only  # the one-batch legs beside `value`

    # setup, untimed: one decode of every copy binds its stream to a hardware queue
    # (a copy's first decode also pays one-time costs: the queue's creation, the code
    # object's first dispatch on it), then the W warmup steps
    for bb in batches:
        bb.decode()
    for bb in batches:
        bb.sync()
    for k in range(args.warmup):
        step(k)
    for bb in batches:
        bb.sync()
    if args.check:
        verify(batches, pcm)
    # every copy's output and block statuses are overwritten (0x7F bytes, WVG_ST_UNWRITTEN)
    # after the untimed decodes, so the check right after the timed region sees only what
    # the timed launches wrote
    for bb in batches:
        bb.poison(0x7F)

    # device time of every launch in the timed region (an event pair around each
    # decode on the stream it runs on)
    for bb in batches:
        bb.set_timing(True)
    _barrier(pg)
    for bb in batches:
        bb.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    t_issue = time.perf_counter()
    for bb in batches:
        bb.sync()
    t1 = time.perf_counter()
    _barrier(pg)
    # the timed decodes were real: every copy's output (poisoned before the timed region,
    # and each copy's last decode is a timed one), CRCs and kernel routing
    ver = verify(batches, pcm)
    ver["checked"] = "right after the timed region; outputs poisoned (0x7F) before it"
    tsum = tn = 0.0
    for bb in batches:
        ms, n = bb.timed()
        tsum += ms * n
        tn += n
        bb.set_timing(False)
    kernel_ms = tsum / max(tn, 1)
    solo_ms = b.time(3) if len(batches) > 1 and extras else kernel_ms  # nothing else in flight
    # the same K steps one batch at a time (reported beside `value`)
    serial_dt = None
    if len(batches) > 1 and extras:
        _barrier(pg)
        b.sync()
        t2 = time.perf_counter()
        for _ in range(args.steps):
            b.decode()
        b.sync()
        serial_dt = _reduce(pg, time.perf_counter() - t2, "max")
    # the other kernel on the same batches, at its own best depth (reported beside `value`)
    other = None
    if extras and args.kernel == "lane":
        nb = min(3, len(batches))
        for bb in batches[:nb]:
            bb.set_kernel("two_wave")
            bb.sync()
        _barrier(pg)
        t3 = time.perf_counter()
        for k in range(args.steps):
            batches[k % nb].decode()
        for bb in batches[:nb]:
            bb.sync()
        dt_o = _reduce(pg, time.perf_counter() - t3, "max")
        other = {"kernel": "two_wave", "batches_in_flight": nb, "value": None, "dt": dt_o}
        for bb in batches[:nb]:
            bb.set_kernel(args.kernel)
    # one batch alone on the kernel the library's default (WVG_KERNEL_AUTO) picks for a
    # caller that decodes one batch at a time: the two-wave kernel (groups <= 2,048 blocks)
    auto_ms = None
    if extras:
        b.set_kernel("two_wave")
        b.sync()
        auto_ms = b.time(3)
        b.set_kernel(args.kernel)
    dt = _reduce(pg, t1 - t0, "max")
    dt_all = _gather(pg, t1 - t0, ws)
    frames_total = _reduce(pg, float(frames_rank), "sum")
    kms_all = _gather(pg, kernel_ms, ws)
    value = frames_total * args.steps / dt / 1e6

    # PCIe-inclusive rate (host bytes in -> host int32 out, framing included),
    # reported beside `value`, never as it
    if args.timed_only or multi:  # profiling runs: only the timed region's launches reach the profiler
        cpu = None
        if multi and rank == 0 and not args.no_cpu:
            cpu = cpu_baseline_c5(files, args.cpu_threads)
        e2e5 = c5_end_to_end(sets, slices) if multi and args.c5_e2e else None
        if rank == 0:
            line = {"metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": ws,
                    "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
                    "higher_is_better": True, "scaling": scaling, "dtype": "int32",
                    "data": "synthetic (repo encoder; C5 seeds per file index)",
                    "config": {"workload": workload, "files_rank0": len(files), "slices_rank0": len(slices),
                               "blocks_rank0": sum(bb.num_blocks for bb in sets[0]), "frames_rank0": int(frames_rank),
                               "frames_total": int(frames_total),
                               "parallelism": f"file-shard x{ws}, no collectives"},
                    "kernel_ms": round(kernel_ms, 4), "per_rank_kernel_ms": [round(x, 4) for x in kms_all],
                    "per_rank_ms_per_step": [round(x * 1e3 / args.steps, 4) for x in dt_all],
                    "batches_in_flight": len(batches), "c5_copies": copies if multi else None,
                    "kernel": args.kernel, "verified": ver,
                    "cpu_baseline": cpu}
            if multi:
                line["end_to_end"] = e2e5
                line["vs_cpu"] = None if cpu is None else {
                    "measured": round(value / cpu["value"], 2),
                    "per_gpu_vs_socket_scaled": round(value / ws / cpu["socket_scaled"], 2)}
            print(json.dumps(line), flush=True)
        for bb in batches:
            bb.close()
        if pg is not None:
            pg.destroy_process_group()
        return
    if rank != 0:  # (the PCIe-inclusive legs below are rank 0's report: no collective follows, and the
        # other ranks' framing threads and page-locked buffers would only contend with rank 0's host)
        for bb in batches:
            bb.close()
        if pg is not None:
            pg.destroy_process_group()
        return
    # a decode server's request on a warm batch: reset, frame the files on the host,
    # upload (page-locked), decode, download into page-locked memory; median of 3
    be = batches[-1]
    be.set_kernel("two_wave")  # (one request at a time: WVG_KERNEL_AUTO's choice for such a caller)
    t_runs = []
    for _ in range(3):
        t_e2e = time.perf_counter()
        be.reset()
        be.add_files(files)
        be.upload()
        be.decode()
        be.download(pinned=True)
        t_runs.append(time.perf_counter() - t_e2e)
    t_e2e = float(np.median(t_runs))
    e2e = frames_rank / t_e2e / 1e6
    # the same request with the framing on the device (wvg_batch_add_files_device)
    t_runs = []
    for _ in range(3):
        t_d = time.perf_counter()
        be.reset()
        be.add_files_device(files)
        be.upload()
        be.decode()
        be.download(pinned=True)
        t_runs.append(time.perf_counter() - t_d)
    t_e2e_dev = float(np.median(t_runs))
    dev_framed = be.framing_stats()
    be.set_kernel(args.kernel)
    # the same request stream served by one host thread per batch copy, so one
    # batch's framing, upload, decode and download overlap the others' (ctypes
    # drops the GIL inside the library; each batch has its own stream)
    e2e_pipe = e2e_pcm = e2e_pcm2 = pipe_ok = None
    if len(batches) > 1:
        import threading
        rounds = 4

        def serve(bb, pcm, rounds=rounds):
            for _ in range(rounds):
                bb.reset()
                bb.add_files(files)
                bb.upload()
                bb.decode()
                if pcm:  # WavpackFormatSamples on the device, PCM bytes down (half the int32 bytes at 16 bits)
                    bb.format()
                    bb.download_pcm(pinned=True)
                else:
                    bb.download(pinned=True)

        # (at most 4 request threads: the host side -- framing, page-locked copies -- is
        # what this measures, and each batch's landing buffers are page-locked)
        pbatches = batches[:4]

        def pipelined(pcm):
            for bb in pbatches:  # first use allocates each batch's page-locked landing buffers: untimed
                serve(bb, pcm, 1)
            th = [threading.Thread(target=serve, args=(bb, pcm)) for bb in pbatches]
            t_p = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            return frames_rank * rounds * len(pbatches) / (time.perf_counter() - t_p) / 1e6

        e2e_pipe = pipelined(False)
        e2e_pcm = pipelined(True)

        # a decode server: producer threads take a free batch and frame, upload, decode and
        # format a request on it (no call waits for the device), consumer threads download
        # the queued requests' PCM in order (page-locked, blocking) and free the batches --
        # the PCIe download, the request's bound, stays busy while the producers' host work
        # and uploads overlap it (round 6; a thread per request ring measured 7,700-8,800,
        # profiles/r06_pipe_pc.jsonl)
        import queue

        def serve_pc(pool, total, producers, consumers):
            free, ready = queue.Queue(), queue.Queue()
            for x in pool:
                free.put(x)
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
                    x.add_files(files)
                    x.upload()
                    x.decode()
                    x.format()
                    ready.put(x)

            def consume():
                while True:
                    x = ready.get()
                    if x is None:
                        return
                    x.download_pcm(pinned=True)
                    free.put(x)
            ps = [threading.Thread(target=produce) for _ in range(producers)]
            cs = [threading.Thread(target=consume) for _ in range(consumers)]
            t_p = time.perf_counter()
            for t in ps + cs:
                t.start()
            for t in ps:
                t.join()
            for _ in cs:
                ready.put(None)
            for t in cs:
                t.join()
            return time.perf_counter() - t_p

        N = min(args.pipe_pool, len(batches))
        if N >= 2:
            pool = batches[:N]
            serve_pc(pool, N, min(args.pipe_producers, N), args.pipe_consumers)  # (landing buffers: untimed)
            for x in pool:  # the page-locked PCM every timed request lands in, poisoned
                x.host_pcm()[:] = 0x7F
            reqs = 4 * N
            e2e_pcm2 = frames_rank * reqs / serve_pc(pool, reqs, min(args.pipe_producers, N), args.pipe_consumers) / 1e6
            if pcm is not None:  # each batch's last request: WavpackFormatSamples' 16-bit image of the generator's PCM
                want = np.ascontiguousarray(pcm.reshape(-1).astype("<i2")).view(np.uint8)
                pipe_ok = all(np.array_equal(x.host_pcm(), want) for x in pool)
                assert pipe_ok, "a pipelined request's PCM differs from the generator's"

    if kernel_ms <= 0:  # (timing off: the launch time of one batch alone stands in)
        kernel_ms = solo_ms if solo_ms > 0 else b.time(3)
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    node_gbs = alg_bytes * args.steps * ws / dt / 1e9
    kname = KERNEL_NAMES[args.kernel]
    traffic, traffic_src = pmc_traffic(kname) if args.workload == "c2" else (None, None)
    if rank == 0:
        cpu = None
        if not args.no_cpu and args.workload == "c2":
            cpu = cpu_baseline(files[0], args.cpu_reps, args.cpu_threads)
        vs = None
        if cpu is not None:
            vs = {"measured": round(value / cpu["value"], 2),
                  "per_gpu_vs_measured": round(value / ws / cpu["value"], 2),
                  "per_gpu_vs_socket_scaled": round(value / ws / cpu["socket"]["per_core_scaled_to_socket"], 2),
                  "per_gpu_vs_single_thread": round(value / ws / cpu["single_thread"], 2),
                  "note": "ratios against the CPU baseline measured in this run (BASELINE.md has no published "
                          "number); socket_scaled = single-thread rate x physical cores of one socket"}
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": vs["measured"] if vs else None,
            "vs_cpu": vs,
            "dtype": "int32",
            "data": "synthetic (repo encoder; C2 seeds 0xC2+block, C5 seeds per file index)",
            "config": {"workload": workload,
                       "files_per_gpu_rank0": len(files), "blocks_rank0": b.num_blocks,
                       "block_frames": args.block_frames if args.workload == "c2" else None, "chunk_frames": 4096,
                       "frames_rank0": int(frames_rank), "frames_total": int(frames_total),
                       "batches_in_flight": len(batches),
                       "compressed_bytes_rank0": sum(len(f) for f in files),
                       "parallelism": f"file-shard x{ws}, no collectives"},
            "per_rank_kernel_ms": [round(x, 4) for x in kms_all],
            "value_one_batch_at_a_time": round(frames_total * args.steps / serial_dt / 1e6, 2) if serial_dt else None,
            "kernel": args.kernel,
            "two_wave": None if other is None else {
                "value": round(frames_total * args.steps / other["dt"] / 1e6, 2),
                "batches_in_flight": other["batches_in_flight"],
                "what": "the same K steps on the one-workgroup-per-block kernel (wvg_batch_set_kernel "
                        "WVG_KERNEL_TWO_WAVE) at its best depth, 3 batches in flight"},
            "hbm_gbs": round(node_gbs, 2),
            "launch_ms": {"in_flight_mean": round(kernel_ms, 4), "alone": round(solo_ms, 4),
                          "alone_api_default": None if auto_ms is None else round(auto_ms, 4),
                          "host_issue_all_steps": round((t_issue - t0) * 1e3, 3),
                          "host_sync_all_steps": round((t1 - t_issue) * 1e3, 3),
                          "what": "device time of one decode launch (hipEvents on its stream): mean over the timed "
                                  "region's launches, and with no other batch in flight (alone_api_default: the "
                                  "kernel the library's default WVG_KERNEL_AUTO picks for a caller decoding one "
                                  "batch at a time, the two-wave kernel)"},
            "pcie_inclusive": {"value": round(e2e, 2), "unit": "Msamples/s", "ms": round(t_e2e * 1e3, 3),
                               "what": "warm batch on the two-wave kernel (WVG_KERNEL_AUTO's choice one request at a time): host framing + upload of the compressed batch (page-locked) + "
                                       "decode + download of int32 PCM into page-locked memory, rank 0, median of 3",
                               "device_framing": {"value": round(frames_rank / t_e2e_dev / 1e6, 2),
                                                  "ms": round(t_e2e_dev * 1e3, 3),
                                                  "files_device_host": list(dev_framed),
                                                  "what": "the same warm request with the header/sub-block walk "
                                                          "on the GPU (wvg_batch_add_files_device)"},
                               "pipelined": None if e2e_pipe is None else round(e2e_pipe, 2),
                               "pipelined_pcm": None if e2e_pcm is None else round(e2e_pcm, 2),
                               "pipelined_pcm_2buf": None if e2e_pcm2 is None else round(e2e_pcm2, 2),
                               "pipelined_what": "the same request served by one host thread per batch copy (at most 4) "
                                                 "(4 requests each), framing/copies/decode of different batches "
                                                 "overlapping; _pcm: formatted on the device (WavpackFormatSamples) "
                                                 "and downloaded as PCM bytes; _pcm_2buf: a decode server over a "
                                                 "pool of pipe_pool batches -- pipe_producers threads frame, upload, "
                                                 "decode and format requests without waiting, pipe_consumers threads "
                                                 "download the queued PCM in order and free the batches (4 x "
                                                 "pipe_pool requests timed)",
                               "pipelined_pcm_2buf_verified": pipe_ok,
                               "pipe_producers": args.pipe_producers, "pipe_consumers": args.pipe_consumers,
                               "pipe_pool": args.pipe_pool,
                               "link_bound_Msamples_s": "~14,200 (90.3 MB of PCM16 down at the box's 56.7 GB/s D2H, "
                                                        "scripts/micro/pcie_kernel.hip); ~12,000 with each "
                                                        "request's 52.9 MB upload sharing the link (~97 GB/s "
                                                        "both ways)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": None if traffic is None else int(traffic),
                         "traffic_unit": "bytes/launch (PMC FETCH_SIZE + WRITE_SIZE, scale calibrated in the profile)",
                         "traffic_source": traffic_src,
                         "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": alg_bytes,
                         "kernel": kname,
                         "node_achieved": round(node_gbs, 2),
                         "node_frac": round(node_gbs / HBM_PEAK_GBS, 6),
                         "binding_limit": "serial entropy decode per block: one lane's dependent word chain "
                                          "(lane kernel) / one wave's scalar issue (two-wave kernel), not HBM"},
            "cpu_baseline": cpu,
            "verified": ver,
        }
        print(json.dumps(line), flush=True)
    for bb in batches:
        bb.close()
    if pg is not None:
        pg.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c2", "c5"), default="c2")
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--block-frames", type=int, default=22050)
    ap.add_argument("--c5-files", type=int, default=4000)
    ap.add_argument("--c5-batch", type=int, default=12500,
                    help="C5: files per batch; a rank with more files decodes all its batches every step")
    ap.add_argument("--c5-e2e", type=int, default=1,
                    help="C5: also time the end-to-end pass (framing, upload, decode, format, download)")
    ap.add_argument("--c5-share", default=None,
                    help="C5: N:r -- decode rank r's share of an N-way file split (one process)")
    ap.add_argument("--c5-copies", type=int, default=0,
                    help="C5: copies of the rank's batches, step k decoding copy k %% copies (0: as many as "
                         "keep about C5_BATCHES_IN_FLIGHT batches in flight)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batch copies decoding concurrently (own buffers and streams); 1 = one batch at a time "
                         "(default: 20 for the lane kernel, 3 for the two-wave kernel, at most --steps)")
    ap.add_argument("--kernel", choices=("lane", "two_wave"), default="lane",
                    help="PCM kernel (wvg_batch_set_kernel): lane-per-block or one workgroup per block")
    ap.add_argument("--pipe-producers", type=int, default=6,
                    help="pcie_inclusive.pipelined_pcm_2buf: producer threads of the decode server")
    ap.add_argument("--pipe-consumers", type=int, default=2, help="its PCM download threads")
    ap.add_argument("--pipe-pool", type=int, default=20, help="its batches (at most --inflight)")
    ap.add_argument("--cpu-threads", type=int, default=None, help="override the socket/lease-derived thread count")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the decoded PCM against the generator's")
    ap.add_argument("--selftest-dist", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--timed-only", action="store_true",
                    help="warmup + timed region only (rocprofv3 runs: the kernel average is the timed launches')")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    run_rank(args)


if __name__ == "__main__":
    main()
