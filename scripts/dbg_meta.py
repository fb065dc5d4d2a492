"""GPU debug: which files/blocks of the fuzzed-metadata batch differ from the host core."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.emu import emu as E
from tests.test_meta_defer import _bases, meta_fuzz
from tests.test_gpu_parity import _gpu_decode
from wavpackdecoder_amd.api import DecodeBatch

files = [meta_fuzz(d, 9000 + 100 * b + s) for b, d in enumerate(_bases()) for s in range(12)]
files.append(meta_fuzz(_bases()[3], 5312))
exp = [E.decode(f) for f in files]

def report(tag, fl, lane=False, host_meta=False):
    os.environ["WVG_HOST_META"] = "1" if host_meta else "0"
    out, res, infos = _gpu_decode(fl, 4096, DecodeBatch, force_lane=lane)
    bad = []
    for k, (f, r, info) in enumerate(zip(fl, res, infos)):
        n, eout, crc, st = exp[files.index(f)]
        if n < 0 or r is None:
            continue
        got = out[info.out_offset: info.out_offset + len(eout)]
        if not np.array_equal(got, eout):
            d = np.nonzero(got != eout)[0]
            bad.append((files.index(f), len(d), int(d[0]), int(d[-1]), r.frames, r.crc_errors, crc))
    print(tag, "bad:", bad, flush=True)

report("batch", files)
report("batch-lane", files, lane=True)
report("batch-hostmeta", files, host_meta=True)
report("alone2", [files[2]])
report("alone2-lane", [files[2]], lane=True)
report("alone2-hostmeta", [files[2]], host_meta=True)
