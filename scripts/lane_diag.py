#!/usr/bin/env python3
"""Why the lane kernel hands C2 blocks back: decode C2 with WVG_LANE_KERNEL=2 (the
lane kernel alone, ST_REDO left in the status) and count the reason bits."""
import collections
import ctypes
import os
import sys

import numpy as np

os.environ.setdefault("WVG_LANE_KERNEL", "2")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from synth import corpora  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

data = corpora.c2()
b = DecodeBatch(4096)
b.add_file(data)
b.upload()
b.decode()
b.sync()
b.download()
n = b.num_blocks
st = np.zeros(n, dtype=np.uint32)
b._L.wvg_batch_block_status(b._b, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n)
redo = (st & (1 << 15)) != 0
why = collections.Counter()
for s in st[redo]:
    why[int(s) >> 16] += 1
print("blocks", n, "redo", int(redo.sum()), "reasons", dict(why))
print("redo block indices", np.nonzero(redo)[0][:40].tolist())
ms = b.time(5)
print("lane kernel alone ms", ms)
