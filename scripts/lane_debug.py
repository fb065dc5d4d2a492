#!/usr/bin/env python3
"""Debug aid: one corrupted file through the lane kernel (WVG_LANE_KERNEL as set)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vectors as V  # noqa: E402
from synth import wvsynth as S  # noqa: E402
from oracle import oracle as O  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

base = S.encode_pcm(S.audio_like(20000, 2, 16, seed=11), S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4000))
for k in range(3):
    d = V.corrupt(base, k)
    b = DecodeBatch(4096)
    b.add_file(d)
    b.upload()
    b.decode()
    out = b.download()
    n = b.num_blocks
    st = np.zeros(n, dtype=np.uint32)
    b._L.wvg_batch_block_status(b._b, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), n)
    r = O.decode_file(d)
    print(k, "lane", os.environ.get("WVG_LANE_KERNEL"), "status", [hex(x) for x in st], "out", out[:4], "oracle",
          r.samples[:4], "equal", np.array_equal(out, r.samples), "crc", b.result(0).crc_errors, r.crc_errors)
    b.close()
