#!/usr/bin/env python3
"""Why the lane kernel hands blocks back: decode a config with WVG_LANE_KERNEL=2
(the lane kernel alone, ST_REDO left in the status) and count the reason bits
(status bits 16-23, wv_lane.h; bits 24-31: the parser's reasons in the first group that
set any), then the lane kernel's time alone and, with the
fallback on (WVG_LANE_KERNEL=1), the same batch's time.

usage: lane_diag.py [c2|c3|c1|c5|c4|dsd3s|dsd3m|dsd3mix|hymix] ...  (default c2) -> one JSON line per config

Reason bits: 1 outside the lane's scope (lane_ok), 2 medians >= 2^26, 4 a weight
that could leave int16, 8 a mute, 16 a bits error / count too long, 32 a word past
the window, 64 a ring underrun, 128 the partner wave stopped."""
import collections
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the per-wave counters need the diagnostics build (make -C wavpackdecoder_amd counters)
_CNT = os.path.join(ROOT, "wavpackdecoder_amd", "build_cnt", "libwvgpu.so")
if os.path.exists(_CNT) and "WVG_LIB" not in os.environ:
    os.environ["WVG_LIB"] = _CNT
REASONS = {1: "scope", 2: "median_bound", 4: "weight_int16", 8: "mute", 16: "bits_error", 32: "past_window",
           64: "ring_underrun", 128: "partner_stopped"}


def files_of(cfg):
    from synth import corpora
    if cfg == "c2":
        return [corpora.c2()]
    if cfg == "c3":
        return [corpora.c3()]
    if cfg == "c1":
        return [corpora.c1()]
    if cfg == "c4":
        return [corpora.c4()]
    if cfg == "c5":
        return corpora.c5(4000)
    if cfg == "hymix":  # the hybrid lane GPU test's mixed batch
        sys.path.insert(0, ROOT)
        from tests.test_gpu_hybrid_lane import _hy
        rng = np.random.default_rng(7)
        out = []
        for k in range(140):
            kind = ("music", "music", "noise", "zeros")[k % 4] if k % 7 else "music"
            frames = int(rng.integers(1, 12000))
            out.append(_hy(frames, 300 + k, bits=24 if k % 3 == 1 else 16, flt=k % 3 == 0,
                           bitrate=int(rng.integers(512, 2048)), block=int(rng.choice([1000, 4410, 7000])), kind=kind,
                           silence=(frames // 4, frames // 2) if k % 5 == 0 else None))
        return out
    if cfg == "dsd3mix":  # the DSD lane GPU test's mixed batch
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from synth import wvsynth as S
        rng = np.random.default_rng(5)
        out = []
        for k in range(150):
            nch, fs = ((2, False), (1, False), (2, True))[k % 3]
            frames, block = int(rng.integers(1, 9000)), int(rng.choice([777, 2000, 5000]))
            dd = S.dsd_random_like(frames, 1 if fs else nch, seed=100 + k, density=float(rng.uniform(0.05, 0.6)))
            dd = np.repeat(dd, 2, axis=1) if fs else dd
            out.append(S.encode_dsd(dd, S.DsdParams(nch=nch, false_stereo=fs, mode=3, block_samples=block,
                                                    rate_i=int(rng.integers(0, 40)))))
        return out
    if cfg in ("dsd3s", "dsd3m"):  # DSD mode 3 stereo / mono files (the DSD lane kernel)
        from synth import wvsynth as S
        nch = 2 if cfg == "dsd3s" else 1
        return [S.encode_dsd(S.dsd_random_like(fr, nch, seed=101 + k, density=0.3),
                             S.DsdParams(nch=nch, mode=3, block_samples=2000, rate_i=7))
                for k, fr in enumerate((4638, 700, 22050, 22050))]
    raise SystemExit(f"unknown config {cfg}")


def one(cfg):
    from wavpackdecoder_amd.api import DecodeBatch
    files = files_of(cfg)
    b = DecodeBatch(4096)  # (WVG_LANE_KERNEL=2 from the environment: no set_kernel, which would set 1)
    b.add_files(files)
    b.upload()
    b.decode()
    b.sync()
    b.download()
    st = b.block_status()
    redo = (st & (1 << 15)) != 0
    why, first = collections.Counter(), collections.Counter()
    for s in st[redo]:
        r, r0 = (int(s) >> 16) & 0xFF, int(s) >> 24
        for bit, name in REASONS.items():
            if r & bit:
                why[name] += 1
            if r0 & bit:
                first[name] += 1
    ms = b.time(3)
    waves = {}
    for ts in range(8):  # per term set: the slowest parser waves and their group paths
        try:
            c = b.lane_counters(ts)
        except RuntimeError:
            continue
        if c.size == 0 or c[:, 1].sum() == 0:
            continue
        order = np.argsort(-c[:, 0].astype(np.int64))
        waves[f"ts{ts}"] = {"waves": int(c.shape[0]), "cycles_max": int(c[order[0], 0]),
                            "cycles_median": int(np.median(c[:, 0])),
                            "slowest": [dict(zip(("wave", "cycles", "groups", "bulk", "norun", "split", "fast",
                                                  "checked", "replay", "wait_consumed", "wait_loads", "words", "stage"),
                                                 [int(i)] + [int(v) for v in c[i][:12]]))
                                        for i in order[:4]],
                            "totals": dict(zip(("groups", "bulk", "norun", "split", "fast", "checked", "replay"),
                                               [int(v) for v in c[:, 1:8].sum(axis=0)]))}
    b.close()
    return {"config": cfg, "lane_waves": waves, "blocks": int(st.size), "redo_blocks": int(redo.sum()),
            "redo_fraction": round(float(redo.mean()) if st.size else 0.0, 5), "reasons": dict(why), "first_reasons": dict(first),
            "redo_first": np.nonzero(redo)[0][:16].tolist(), "lane_kernel_alone_ms": round(ms, 3)}


def with_fallback(cfg):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(4096)
    b.set_kernel("lane")
    b.add_files(files_of(cfg))
    b.upload()
    b.decode()
    b.sync()
    ms = b.time(3)
    b.download()
    st = b.block_status()
    b.close()
    return {"with_fallback_ms": round(ms, 3), "redone": int(np.count_nonzero(st & 0x200))}


if __name__ == "__main__":
    cfgs = sys.argv[1:] or ["c2"]
    if os.environ.get("WVG_LANE_KERNEL") == "1":  # (child: the fallback run)
        print(json.dumps(with_fallback(cfgs[0])), flush=True)
        sys.exit(0)
    os.environ["WVG_LANE_KERNEL"] = "2"
    os.environ["WVG_LANE_COUNTERS"] = "1"
    for cfg in cfgs:
        d = one(cfg)
        # the fallback run in a child (the kernel mode is read when a batch is created)
        env = dict(os.environ, WVG_LANE_KERNEL="1")
        out = subprocess.run([sys.executable, os.path.abspath(__file__), cfg], env=env, capture_output=True,
                             text=True, timeout=600)
        if out.returncode == 0:
            d.update(json.loads(out.stdout.strip().splitlines()[-1]))
        print(json.dumps(d), flush=True)
