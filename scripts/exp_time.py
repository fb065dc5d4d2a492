#!/usr/bin/env python3
"""Kernel-time probe for performance experiments (not part of the product).

Usage: WVG_LIB=<path to a libwvgpu.so build> python scripts/exp_time.py [nblocks ...]
Prints one line per batch size: blocks, kernel ms (hipEvents, mean of 10), Mframes/s.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from synth import corpora  # noqa: E402
from wavpackdecoder_amd import _lib  # noqa: E402
import wavpackdecoder_amd.api as api  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [1024]
    L = _lib.lib()
    api._ctx = L.wvg_open(0)
    tag = os.environ.get("WVG_LIB", "default")
    for n in sizes:
        data = corpora.c2(nblocks=n)
        b = api.DecodeBatch(4096)
        b.add_file(data)
        b.upload()
        b.decode()
        b.sync()
        ms = b.time(10)
        if os.environ.get("WVG_PROF") == "4":
            import numpy as np
            o = b.download().view("uint32").astype("uint64")
            per = o.size // n
            blk = o[: per * n].reshape(n, per)
            tp = blk[:, 4] | (blk[:, 5] << 32)
            tr = blk[:, 8] | (blk[:, 9] << 32)
            trw = blk[:, 10] | (blk[:, 11] << 32)
            for name, arr in (("parser", tp), ("recon", tr)):
                idx = np.argsort(arr)[::-1][:6]
                print(f"  {name}: median={np.median(arr):.0f} max={arr.max()} slowest="
                      + ", ".join(f"{i}:{arr[i]}(fast={blk[i,0]},zr={blk[i,1]},slow={blk[i,2]},rwait={trw[i]})" for i in idx),
                      flush=True)
        elif os.environ.get("WVG_PROF"):
            c = b.download()[:8].view("uint32").astype("uint64")
            words = 2 * b.frames // n
            t = int(c[4] | (c[5] << 32))
            tw = int(c[6] | (c[7] << 32))
            print(f"  block0: fast={c[0]} zr={c[1]} slow={c[2]} refill={c[3]} words={words} "
                  f"cycles={t} ({t / words:.1f}/word) wait={tw}", flush=True)
        print(f"{tag} blocks={n} kernel_ms={ms:.3f} Mframes/s={b.frames / ms / 1e3:.1f}", flush=True)
        b.close()


if __name__ == "__main__":
    main()
