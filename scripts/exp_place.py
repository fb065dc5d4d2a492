#!/usr/bin/env python3
"""Wave placement + timeline probe for the two-wave kernel (not part of the product).

Needs a WV2_EXP=5 build (`make -C wavpackdecoder_amd build/exp5/libwvgpu.so`):
every block writes {HW_ID, XCC_ID, t_begin, t_end} (s_memrealtime, 100 MHz) of
its parser wave into output ints 12-15 and of its reconstruction wave into
ints 16-19.

Usage: WVG_LIB=<exp5 libwvgpu.so> python scripts/exp_place.py [nblocks]
Prints: blocks per CU, parser waves per SIMD, parser/recon durations, and the
parser duration grouped by how many parsers share the SIMD.
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from synth import corpora  # noqa: E402
from wavpackdecoder_amd import _lib  # noqa: E402
import wavpackdecoder_amd.api as api  # noqa: E402


def fields(hw):
    # gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]
    return (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    L = _lib.lib()
    api._ctx = L.wvg_open(0)
    data = corpora.c2(nblocks=n)
    b = api.DecodeBatch(4096)
    b.add_file(data)
    b.upload()
    b.decode()
    b.sync()
    ms = b.time(3)
    b.decode()
    o = b.download().view(np.uint32)
    per = o.size // n
    blk = o[: per * n].reshape(n, per)
    p = blk[:, 12:16].astype(np.int64)
    r = blk[:, 16:20].astype(np.int64)
    keys_p = []
    simd_par = collections.Counter()
    simd_all = collections.Counter()
    cu_blocks = collections.Counter()
    for role, arr in (("P", p), ("R", r)):
        for hw, xcc, _, _ in arr:
            simd, cu, sh, se = fields(int(hw))
            key = (int(xcc), se, sh, cu, simd)
            simd_all[key] += 1
            if role == "P":
                simd_par[key] += 1
                cu_blocks[key[:4]] += 1
                keys_p.append(key)
    base = p[:, 2].min()
    start = ((p[:, 2] - base) % (1 << 32)) / 100.0  # us
    dur_p = ((p[:, 3] - p[:, 2]) % (1 << 32)) / 100.0
    dur_r = ((r[:, 3] - r[:, 2]) % (1 << 32)) / 100.0
    end = start + dur_p
    print(f"blocks={n} kernel_ms={ms:.3f}")
    print(f"CUs used={len(cu_blocks)} blocks/CU histogram: {dict(collections.Counter(cu_blocks.values()))}")
    print(f"SIMDs with parsers={len(simd_par)} parsers/SIMD histogram: {dict(collections.Counter(simd_par.values()))}")
    print(f"waves/SIMD histogram: {dict(collections.Counter(simd_all.values()))}")
    print(f"parser us: min={dur_p.min():.1f} med={np.median(dur_p):.1f} max={dur_p.max():.1f} "
          f"slowest blocks={list(np.argsort(dur_p)[::-1][:8])}")
    print(f"recon  us: min={dur_r.min():.1f} med={np.median(dur_r):.1f} max={dur_r.max():.1f}")
    print(f"start  us: max={start.max():.1f}; last parser end {end.max():.1f}")
    dp = np.array([simd_par[k] for k in keys_p])
    for k in sorted(set(dp.tolist())):
        sel = dp == k
        print(f"  parsers sharing a SIMD={k}: n={int(sel.sum())} parser us med={np.median(dur_p[sel]):.1f} "
              f"max={dur_p[sel].max():.1f}")
    # per-kind (music / zeros / noise as corpora.c2 draws them)
    kinds = []
    for i in range(n):
        rr = ((0xC2 + i) * 2654435761) % 100
        kinds.append("zeros" if rr < 2 else ("noise" if rr < 3 else "music"))
    kinds = np.array(kinds)
    for k in ("music", "zeros", "noise"):
        sel = kinds == k
        if sel.any():
            print(f"  {k}: n={int(sel.sum())} parser us med={np.median(dur_p[sel]):.1f} max={dur_p[sel].max():.1f}")
    b.close()


if __name__ == "__main__":
    main()
