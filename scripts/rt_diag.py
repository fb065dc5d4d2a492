#!/usr/bin/env python3
"""Why the run-time list lanes hand blocks back, per test case: decode each case of
tests/test_gpu_lane_rt.py's hybrid sets with WVG_LANE_KERNEL=2 (the lane kernels alone:
ST_REDO and its reason bits stay in the block status) and print the hand-backs'
reasons (status bits 16-23, wv_lane.h: 1 out of scope, 2 bounds, 4 weight, 8 mute, 16
count, 32 window, 64 ring, 128 wait) and the first group's (bits 24-31)."""
import collections
import os
import sys

os.environ["WVG_LANE_KERNEL"] = "2"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import tests.test_gpu_lane_rt as T  # noqa: E402
from synth import wvsynth as S  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

REDO = 1 << 15


def cases():
    lists = {"fast": S.TERMS_FAST, "alt5": T.STEREO_LISTS["alt5"], "high10": S.TERMS_HIGH10,
             "high16": S.TERMS_HIGH, "alt16": T.STEREO_LISTS["alt16"], "default": S.TERMS_DEFAULT}
    for k, (n, t) in enumerate(lists.items()):
        for bal in (False, True):
            yield f"hy_{n}{'_bal' if bal else ''}", T._hyb(12000, t, 700 + 2 * k + bal, balance=bal,
                                                         bits=16 + 8 * (k % 2))
        yield f"hy_{n}_float", T._hyb(9000, t, 720 + k, flt=True, balance=k % 2 == 0, bitrate=1200)
    for k, t in enumerate((T.MONO_LISTS["m4"], S.TERMS_MONO_HIGH[:5], T.MONO_LISTS["m10"], T.MONO_LISTS["m16alt"])):
        yield f"hym{k}", T._hyb(12000, t, 800 + k, nch=1)
        yield f"hym{k}_fs", T._hyb(9000, t, 810 + k, fs=True, bitrate=1200)
        yield f"hym{k}_24_ragged", T._hyb(7000, t, 820 + k, nch=1, bits=24, block=997)
        yield f"hym{k}_float", T._hyb(6000, t, 830 + k, nch=1, flt=True)


def main():
    for name, data in cases():
        b = DecodeBatch(4096)
        b.add_file(data)
        b.decode()
        b.download()
        st = b.block_status()
        red = st[(st & REDO) != 0]
        why = collections.Counter(int((x >> 16) & 0xFF) for x in red)
        first = collections.Counter(int((x >> 24) & 0xFF) for x in red)
        print(f"{name:22s} blocks {st.size:3d} handed back {red.size:3d}  reasons {dict(why)}  first {dict(first)}  "
              f"groups {b.lane_groups():#x}", flush=True)
        b.close()


if __name__ == "__main__":
    main()
