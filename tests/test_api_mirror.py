"""The host mirror of the reference API (wavpackdecoder_amd/api.py) call by call
against the oracle's context API (the same WavpackUnpackSamples loop,
WavPackUtils.cs:200-282): the frames each call returns, the samples, and the
getters that follow the calls -- GetSampleIndex (:355-358), GetNumErrors
(:363-366, counted at block ends :273-275), Lossy -- plus the call on which the
reference throws (earlier calls still return their frames)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import vectors as V

pytestmark = pytest.mark.gpu


def _oracle_calls(data, samples, seek=None):
    L = O.lib()
    L.wvo_set_sample.restype = ctypes.c_int
    L.wvo_set_sample.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    ctx = L.wvo_open(data, len(data), 0)
    calls = []
    try:
        if seek is not None:
            calls.append(("seek", L.wvo_set_sample(ctx, seek), L.wvo_get_sample_index(ctx), L.wvo_get_num_errors(ctx)))
        nch = max(L.wvo_get_reduced_channels(ctx), 1)
        buf = np.zeros(samples * nch, dtype=np.int32)
        for _ in range(100000):
            n = L.wvo_unpack_samples(ctx, buf.ctypes.data, buf.size, samples)
            if n < 0:
                calls.append(("exc",))
                break
            calls.append((int(n), buf[: n * nch].copy(), L.wvo_get_sample_index(ctx), L.wvo_get_num_errors(ctx)))
            if n == 0:
                break
    finally:
        L.wvo_close(ctx)
    return calls


def _mirror_calls(data, samples, seek=None, window=0):
    from wavpackdecoder_amd import api
    wpc = api.WavpackOpenFileInput(data, window_frames=window)
    calls = []
    if seek is not None:
        calls.append(("seek", int(api.SetSample(wpc, seek)), api.WavpackGetSampleIndex(wpc),
                      api.WavpackGetNumErrors(wpc)))
    nch = max(api.WavpackGetReducedChannels(wpc), 1)
    buf = np.zeros(samples * nch, dtype=np.int32)
    for _ in range(100000):
        try:
            n = api.WavpackUnpackSamples(wpc, buf, samples)
        except api.WavpackException:
            calls.append(("exc",))
            break
        calls.append((int(n), buf[: n * nch].copy(), api.WavpackGetSampleIndex(wpc), api.WavpackGetNumErrors(wpc)))
        if n == 0:
            break
    wpc.close()
    return calls


def _same(a, b, name):
    assert len(a) == len(b), name
    for k, (x, y) in enumerate(zip(a, b)):
        assert x[0] == y[0], (name, k)
        if x[0] in ("exc",):
            continue
        if x[0] == "seek":
            assert x[1:] == y[1:], (name, k)
            continue
        np.testing.assert_array_equal(x[1], y[1], err_msg=f"{name} call {k}")
        assert x[2:] == y[2:], (name, k, x[2:], y[2:])


def _files():
    from synth import wvsynth as S
    base = S.encode_pcm(S.audio_like(20000, 2, 16, seed=11), S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4000))
    fs = [("corrupt#%d" % k, V.corrupt(base, k)) for k in range(10)]
    fs += [(n, d) for n, d, c in V.pcm_cases() if n in ("stereo16_default", "int32_wvx_short", "int32_wvxnew_short",
                                                        "hybrid_bitrate", "mono16_high")]
    fs.append(("block_index_7", S.encode_pcm(S.audio_like(9000, 2, 16, seed=5), S.EncParams(
        terms=S.TERMS_FAST, block_samples=3000, block_index_start=7))))
    return fs


@pytest.mark.parametrize("samples", [4096, 1000])
def test_unpack_calls_match_oracle(samples):
    for name, data in _files():
        _same(_oracle_calls(data, samples), _mirror_calls(data, samples), name)


def test_seek_then_calls_match_oracle():
    for name, data in _files()[:4] + _files()[-3:]:
        for target in (0, 5000, 12345):
            _same(_oracle_calls(data, 4096, seek=target), _mirror_calls(data, 4096, seek=target), f"{name}@{target}")


@pytest.mark.parametrize("window", [1, 999, 4096, 10007])
def test_stream_windows_match_oracle(window):
    """The stream serves the calls from staged windows of `window` frames (wvg_stream,
    host memory bounded by two windows): window edges inside calls, at call edges,
    a window of one frame, over C1 (20 s, 40 blocks), a corrupted file and a file
    whose reference decode throws."""
    from synth import corpora
    cases = [("config1", corpora.c1()[1])] + [f for f in _files() if f[0] in ("corrupt#3", "int32_wvx_short")]
    for name, data in cases:
        if window == 1 and name == "config1":
            continue  # 882,000 one-frame DMAs: covered by the shorter files
        for samples in (4096, 777):
            _same(_oracle_calls(data, samples), _mirror_calls(data, samples, window=window), f"{name}/{window}/{samples}")


def test_dsd_calls_and_seeks_match_oracle():
    """DSD modes 0/1/3 (stereo, mono, false stereo, RLE tables) and corrupted mode-3
    streams (the final chunk's CRC mute) through the call sequence: caller chunks that
    cut the decoders' 64-value output runs (37, 1000), and seeks whose discarded
    values start mid-run (DsdUtils.cs:56-136, WavPackUtils.cs:200-282).  (A corrupted
    mode-1 stream can stop decoding mid-chunk, leaving the rest of the caller's
    buffer as it was -- ST_NONDET, not comparable call by call.)"""
    files = [(n, d) for n, d, c in V.dsd_cases()]
    for n, d in list(files):
        if n == "dsd_m3_ch2_fs0":
            files += [(f"{n}_corrupt#{k}", V.corrupt(d, k, start=200)) for k in range(3)]
    for name, data in files:
        for samples in (37, 1000):
            _same(_oracle_calls(data, samples), _mirror_calls(data, samples), f"{name}/{samples}")
        for target in (3, 5001, 9999):
            _same(_oracle_calls(data, 4096, seek=target), _mirror_calls(data, 4096, seek=target), f"{name}@{target}")


def test_overrun_layouts_calls_match_oracle():
    """a block that writes 2 ints a frame into a 1-int file throws
    in the call whose store runs past the caller's buffer (WavPackUtils.cs:261); that
    call returns nothing, the calls before it their frames -- call by call against the
    oracle, PCM (FALSE_STEREO + MONO_FLAG, a stereo block in a mono file) and DSD
    (FALSE_STEREO in a mono file)."""
    from tests.test_layout_quirks import dsd_fs_mono_cases, quirk_cases
    names = ("fs_monoflag", "fs_monoflag_chunk500", "fs_monoflag_overrun", "mono_file_stereo_block",
             "mono_file_stereo_block_chunk300")
    cases = [(n, d, c) for n, d, c in quirk_cases() if n in names]
    cases += [(n, d, c) for n, d, c in dsd_fs_mono_cases() if O.decode_file(d, chunk=c).status == -3]
    for name, data, chunk in cases:
        for samples in sorted({chunk, 4096, 1000}):
            _same(_oracle_calls(data, samples), _mirror_calls(data, samples), f"{name}/{samples}")
