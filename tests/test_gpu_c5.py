"""GPU: BASELINE config 5 (the mixed corpus) decoded in one batch, host-framed and
device-framed, every file against the oracle (WavPackUtils.cs:200-282 per file;
DSD through DsdUtils.cs:56-136).

The slice is large enough that every kind of the corpus appears (stereo16, mono16,
FALSE_STEREO, stereo24, mono24, DSD modes 0/1/3); each file's samples, frame count
and crc_errors must equal the oracle's, with no CRC error and no exception."""
import struct

import numpy as np
import pytest

from oracle import oracle as O
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu

N_FILES = 240
FALSE_STEREO = 0x40000000


def _kinds(files):
    from synth import corpora
    kinds = []
    for i, f in enumerate(files):
        kind, _ = corpora.c5_meta(i)
        flags = struct.unpack_from("<I", f, 24)[0]
        if kind == "mono16" and flags & FALSE_STEREO:
            kind = "false_stereo"
        kinds.append(kind)
    return kinds


@pytest.fixture(scope="module")
def c5_corpus():
    from synth import corpora
    files = corpora.c5(N_FILES)
    refs = [O.decode_file(f, chunk=4096) for f in files]
    return files, refs


@pytest.mark.parametrize("framing,kernel", [("host", "two_wave"), ("device", "two_wave"), ("host", "lane")])
def test_c5_batch_matches_oracle(gpu_batch_cls, c5_corpus, framing, kernel):
    """kernel 'lane': every PCM kind of the corpus has a lane instantiation (stereo16 {17,17} and
    default lists, mono16 / false stereo on the mono default list, 24-bit stereo and mono on the
    16-term lists)."""
    files, refs = c5_corpus
    kinds = _kinds(files)
    assert set(kinds) == {"stereo16", "mono16", "false_stereo", "stereo24", "mono24", "dsd0", "dsd1", "dsd3"}
    b = gpu_batch_cls(4096)
    b.set_kernel(kernel)
    if framing == "host":
        idx = b.add_files(files, threads=8)
    else:
        idx = b.add_files_device(files)
    assert idx == list(range(N_FILES))
    b.decode()
    out = b.download()
    if framing == "device":
        dev, host = b.framing_stats()
        assert dev + host == N_FILES and dev > N_FILES // 2, (dev, host)
    for k, (ref, kind) in enumerate(zip(refs, kinds)):
        assert ref.status == 0 and ref.crc_errors == 0, (k, kind)
        info = b.infos[k]
        assert info.open_ok, (k, kind)
        r = b.result(k)
        assert not (r.status_or & WVG_ST_TIMEOUT), (k, kind)
        assert r.exception == 0 and r.crc_errors == 0, (k, kind)
        assert r.frames == ref.frames, (k, kind)
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        np.testing.assert_array_equal(got, ref.samples, err_msg=f"file {k} ({kind}, {framing}-framed)")
    b.close()


def test_c5_batches_in_flight_match_oracle(gpu_batch_cls, c5_corpus):
    """Two mixed batches decoded back to back: the second is issued while the first
    runs, so it keeps all its launch groups (DSD modes 1/3, the PCM term sets) on one
    stream (wv_api.cpp wvg_batch_decode); both must still equal the oracle."""
    files, refs = c5_corpus
    halves = [(0, N_FILES // 2), (N_FILES // 2, N_FILES)]
    batches = []
    for lo, hi in halves:
        b = gpu_batch_cls(4096)
        b.add_files(files[lo:hi], threads=8)
        b.upload()
        batches.append(b)
    for b in batches:
        b.decode()
    for (lo, hi), b in zip(halves, batches):
        out = b.download()
        for k in range(hi - lo):
            ref, info, r = refs[lo + k], b.infos[k], b.result(k)
            assert not (r.status_or & WVG_ST_TIMEOUT), lo + k
            assert r.exception == 0 and r.crc_errors == 0 and r.frames == ref.frames, lo + k
            got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
            np.testing.assert_array_equal(got, ref.samples, err_msg=f"file {lo + k}")
        b.close()
