#!/usr/bin/env python3
"""Diagnostics: decode a lane_diag config with the lane kernel alone (WVG_LANE_KERNEL=2:
no fallback, the lane's own output stays) and print, per file whose output differs
from the oracle's, the first differing value and the status of its blocks.
usage: lane_firstdiff.py CONFIG [max_files]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ["WVG_LANE_KERNEL"] = "2"


def main():
    import lane_diag as L
    from oracle import oracle as O
    from wavpackdecoder_amd.api import DecodeBatch
    cfg = sys.argv[1]
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    files = L.files_of(cfg)
    b = DecodeBatch(4096)
    idx = [b.add_file(f) for f in files]
    b.decode()
    out = b.download()
    st = b.block_status()
    infos = list(b.infos)
    b.close()
    shown = 0
    for k, (f, i, info) in enumerate(zip(files, idx, infos)):
        ref = O.decode_file(f, chunk=4096)
        if i < 0 or ref.status < 0:
            continue
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        bad = np.nonzero(got != ref.samples)[0]
        if bad.size:
            j = int(bad[0])
            print(f"file {k}: {bad.size} values differ, first at {j} (frame {j // ref.nch}): "
                  f"got {got[j:j + 6].tolist()} ref {ref.samples[j:j + 6].tolist()}", flush=True)
            shown += 1
            if shown >= cap:
                break
    print("redo reasons of the first blocks:", [hex(int(s)) for s in st[(st & (1 << 15)) != 0][:12]])


if __name__ == "__main__":
    main()
