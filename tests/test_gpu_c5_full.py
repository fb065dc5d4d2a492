"""GPU: BASELINE config 5 at its own size -- the 100,000-file mixed corpus on one GPU
(VERDICT r05 "Next round" #3: in the driver's run by default; WVG_C5_FULL=<files> picks
another size, 0 skips it).

The files are decoded as bench.py's C5 workload decodes them at N = 1: slices of 12,500
files, one batch each, every batch issued before any finishes (WVG_KERNEL_AUTO: the lane
kernels once batches overlap; each batch's launch groups on streams of its own within the
hardware-queue budget).  Every file must decode with no CRC error and no exception, and
an evenly spaced sample of files (WVG_C5_SAMPLE, default 3,000, plus every DSD mode-1 and
mode-3 file among the first 20,000) must equal the oracle bit for bit.  Reference:
WavPackUtils.cs:200-282 per file."""
import json
import os
import time

import numpy as np
import pytest

from oracle import oracle as O
from wavpackdecoder_amd._lib import WVG_ST_REDONE, WVG_ST_TIMEOUT, WVG_ST_UNWRITTEN

N_FILES = int(os.environ.get("WVG_C5_FULL", "100000"))
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(N_FILES <= 0, reason="WVG_C5_FULL=0")]


@pytest.mark.timeout(1500)
def test_c5_full_corpus_one_gpu():
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    n = N_FILES
    per = int(os.environ.get("WVG_C5_BATCH", "12500"))
    t0 = time.perf_counter()
    files = corpora.c5_files(range(n), progress=True)
    t_gen = time.perf_counter() - t0
    batches = []
    t0 = time.perf_counter()
    for k in range(0, n, per):
        b = DecodeBatch(4096)
        b.set_kernel("auto")
        b.add_files(files[k:k + per])
        b.upload()
        batches.append(b)
    t_frame = time.perf_counter() - t0
    t0 = time.perf_counter()
    for b in batches:
        b.decode()
    for b in batches:
        b.sync()
    t_dec = time.perf_counter() - t0
    # the oracle sample: evenly spaced files, and the DSD mode-1 / mode-3 files of the first 20,000
    ns = int(os.environ.get("WVG_C5_SAMPLE", "3000"))
    sample = set(range(0, n, max(1, n // ns)))
    sample |= {i for i in range(min(n, 20000)) if corpora.c5_meta(i)[0] in ("dsd1", "dsd3")}
    sample = sorted(sample)
    t0 = time.perf_counter()
    refs = dict(zip(sample, O.decode_many([files[i] for i in sample])))
    t_cpu = time.perf_counter() - t0
    frames = blocks = redone = compared = 0
    for k, b in enumerate(batches):
        out = b.download()
        st = b.block_status()
        assert not np.any(st & WVG_ST_UNWRITTEN)
        redone += int(np.count_nonzero(st & WVG_ST_REDONE))
        blocks += int(st.size)
        for i in range(len(b.infos)):
            g = k * per + i
            r = b.result(i)
            assert b.infos[i].open_ok and not (r.status_or & WVG_ST_TIMEOUT), g
            assert r.exception == 0 and r.crc_errors == 0, g
            frames += r.frames
            if g in refs:
                ref = refs[g]
                assert ref.status == 0 and r.frames == ref.frames, g
                info = b.infos[i]
                got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
                np.testing.assert_array_equal(got, ref.samples, err_msg=f"file {g}")
                compared += 1
        b.close()
    assert compared == len(sample)
    rec = {"test": "c5_full_corpus_one_gpu", "files": n, "blocks": blocks, "frames": frames, "batches": len(batches),
           "redone": redone, "oracle_files": compared, "gen_s": round(t_gen, 1), "host_framing_s": round(t_frame, 1),
           "decode_s_wall": round(t_dec, 3), "Mframes_per_s_wall": round(frames / t_dec / 1e6, 1),
           "oracle_s": round(t_cpu, 1)}
    print("PARITY " + json.dumps(rec), flush=True)
    path = os.environ.get("WVG_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
