"""GPU parity at the BASELINE configurations' own sizes, on the routes the library
ships (VERDICT r04 "Next round" #1).

* C3: 4,096 x 44,100-frame 24-bit stereo blocks, WavPack's 16-term 'high' list,
  on the lane kernel (wvg_batch_set_kernel(WVG_KERNEL_LANE));
* C4: 1,024 x 22,050-frame float32 hybrid + bitrate blocks on the hybrid lanes;
* C5: files 0..3,999 of the mixed corpus in four batches decoded in flight on the
  default kernel choice (WVG_KERNEL_AUTO: lanes once batches overlap);
* the ranked product path (shard.run_rank) at world size 1 with DecodeBatch as the
  decode function.

The oracle (oracle/, the C restatement of the C# path) decodes the same inputs on
the host's threads: C3 and C4 are split at block boundaries into parts, which the
GPU decodes as the files of one batch (identical inputs on both sides), and the
whole file is decoded on the GPU too -- it must equal the parts' concatenation
(C3: also the generator's PCM, a lossless round trip).  Every test prints the
number of blocks the lane kernels handed back (WVG_ST_REDONE) and appends a record
to $WVG_PARITY_LOG when it is set.  Reference: WavPackUtils.cs:200-282 per file,
UnpackUtils.cs:510-686, WordsUtils.cs:272-511, FloatUtils.cs:32-56."""
import json
import os
import time

import numpy as np
import pytest

from oracle import oracle as O
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_REDONE, WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


def _log(rec: dict):
    print("PARITY " + json.dumps(rec), flush=True)
    path = os.environ.get("WVG_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _parts(data: bytes, nparts: int) -> list:
    """The file split at block boundaries into nparts runs of whole blocks."""
    spans = V.block_spans(data)
    per = (len(spans) + nparts - 1) // nparts
    out = []
    for k in range(0, len(spans), per):
        lo = spans[k][0]
        last = spans[min(k + per, len(spans)) - 1]
        out.append(data[lo:last[0] + last[1]])
    return out


def _gpu(files, kernel):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(4096)
    b.set_kernel(kernel)
    idx = b.add_files(files)
    t0 = time.perf_counter()
    b.decode()
    b.sync()
    ms = (time.perf_counter() - t0) * 1e3
    out = b.download()
    res = [b.result(i) for i in idx]
    infos = list(b.infos)
    st = b.block_status()
    b.close()
    return out, res, infos, st, ms


def _compare(refs, out, res, infos, tag):
    """Every file bit-exact with its oracle decode; returns the concatenated output."""
    got_all = []
    for k, (ref, r, info) in enumerate(zip(refs, res, infos)):
        assert ref.status == 0, (tag, k, ref.status)
        assert not (r.status_or & WVG_ST_TIMEOUT), (tag, k)
        assert r.exception == 0 and r.frames == ref.frames and r.crc_errors == ref.crc_errors, \
            (tag, k, r.frames, ref.frames, r.crc_errors, ref.crc_errors)
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        bad = np.flatnonzero(got != ref.samples)
        assert bad.size == 0, f"{tag} file {k}: {bad.size} values differ, first at {bad[:1].tolist()}"
        got_all.append(got)
    return np.concatenate(got_all) if got_all else np.zeros(0, np.int32)


@pytest.mark.timeout(900)
def test_c3_full_size_lane_vs_oracle():
    from synth import corpora
    t0 = time.perf_counter()
    pcm, data = corpora.c3(return_pcm=True)
    t_gen = time.perf_counter() - t0
    parts = _parts(data, 64)
    t0 = time.perf_counter()
    refs = O.decode_many(parts)
    t_cpu = time.perf_counter() - t0
    out, res, infos, st, ms = _gpu(parts, "lane")
    cat = _compare(refs, out, res, infos, "c3")
    assert st.size == 4096
    redone = int(np.count_nonzero(st & WVG_ST_REDONE))
    del out, refs
    # the whole file, one descriptor chain per block as a caller's file: lossless, and the
    # same values as its parts (the call seams fall elsewhere; well-formed weights never
    # reach the (short) store's range)
    out2, res2, infos2, st2, ms2 = _gpu([data], "lane")
    assert res2[0].crc_errors == 0 and res2[0].frames == 4096 * 44100
    np.testing.assert_array_equal(out2, pcm.reshape(-1))
    np.testing.assert_array_equal(out2, cat)
    redone2 = int(np.count_nonzero(st2 & WVG_ST_REDONE))
    _log({"test": "c3_full_size_lane", "blocks": int(st.size), "frames": int(pcm.shape[0]), "parts": len(parts),
          "redone_parts_batch": redone, "redone_whole_file": redone2, "gpu_ms_parts": round(ms, 2),
          "gpu_ms_whole": round(ms2, 2), "oracle_s": round(t_cpu, 2), "gen_s": round(t_gen, 1)})
    assert redone == 0 and redone2 == 0, "C3's blocks all stay on the lanes (profiles/r04_c3_lane_diag.json)"


@pytest.mark.timeout(600)
def test_c4_full_size_hybrid_lanes_vs_oracle():
    from synth import corpora
    data = corpora.c4()
    parts = _parts(data, 64)
    t0 = time.perf_counter()
    refs = O.decode_many(parts)
    t_cpu = time.perf_counter() - t0
    out, res, infos, st, ms = _gpu(parts, "lane")
    cat = _compare(refs, out, res, infos, "c4")
    assert st.size == 1024
    redone = int(np.count_nonzero(st & WVG_ST_REDONE))
    out2, res2, infos2, st2, ms2 = _gpu([data], "lane")
    assert res2[0].crc_errors == 0 and res2[0].frames == 1024 * 22050
    np.testing.assert_array_equal(out2, cat)
    _log({"test": "c4_full_size_hybrid_lanes", "blocks": int(st.size), "parts": len(parts),
          "redone_parts_batch": redone, "redone_whole_file": int(np.count_nonzero(st2 & WVG_ST_REDONE)),
          "gpu_ms_parts": round(ms, 2), "gpu_ms_whole": round(ms2, 2), "oracle_s": round(t_cpu, 2)})


@pytest.mark.timeout(900)
def test_c5_4000_files_in_flight_auto_vs_oracle():
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    n = 4000
    t0 = time.perf_counter()
    files = corpora.c5(n)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    refs = O.decode_many(files)
    t_cpu = time.perf_counter() - t0
    nb = 4
    per = n // nb
    batches = []
    for k in range(nb):
        b = DecodeBatch(4096)
        b.set_kernel("auto")
        b.add_files(files[k * per:(k + 1) * per])
        b.upload()
        batches.append(b)
    t0 = time.perf_counter()
    for b in batches:  # issued back to back: each decode starts while the earlier ones run
        b.decode()
    for b in batches:
        b.sync()
    ms = (time.perf_counter() - t0) * 1e3
    redone = blocks = 0
    for k, b in enumerate(batches):
        out = b.download()
        res = [b.result(i) for i in range(per)]
        _compare(refs[k * per:(k + 1) * per], out, res, list(b.infos), f"c5 batch {k}")
        st = b.block_status()
        redone += int(np.count_nonzero(st & WVG_ST_REDONE))
        blocks += int(st.size)
        b.close()
    frames = sum(r.frames for r in refs)
    _log({"test": "c5_4000_files_in_flight_auto", "files": n, "blocks": blocks, "frames": int(frames),
          "batches_in_flight": nb, "redone": redone, "gpu_ms_all": round(ms, 2), "oracle_s": round(t_cpu, 2),
          "gen_s": round(t_gen, 1)})


@pytest.mark.timeout(600)
def test_shard_run_rank_ws1_with_decode_batch():
    """bench.py's ranked path with the product decode: shard.run_rank at world size 1
    (the partition, the per-rank DecodeBatch, the totals) on a C5 slice; frames and
    CRC errors equal the oracle's sums."""
    from synth import corpora
    from wavpackdecoder_amd import shard
    from wavpackdecoder_amd.api import DecodeBatch
    files = corpora.c5(400)
    refs = O.decode_many(files)

    def decode(mine):
        b = DecodeBatch(4096)
        idx = b.add_files(mine)
        t0 = time.perf_counter()
        b.decode()
        b.sync()
        sec = time.perf_counter() - t0
        b.download()
        frames = crc = 0
        for i in idx:
            r = b.result(i)
            assert r.exception == 0 and not (r.status_or & WVG_ST_TIMEOUT)
            frames += r.frames
            crc += r.crc_errors
        b.close()
        return frames, crc, sec

    frames, crc, sec = shard.run_rank(files, 0, 1, decode, None)
    assert frames == sum(r.frames for r in refs) and crc == 0 and sec > 0
