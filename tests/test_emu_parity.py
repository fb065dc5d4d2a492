"""Host build of the device decode core (tests/emu) vs the oracle.

wv_framing.cpp + wv_decode_core.h are the exact sources the HIP kernels and
the host framing use; compiling them for the CPU lets the decode semantics
(chunk seams, muting, CRC verdicts, fixup, DSD) be checked bit-exactly against
the oracle without a GPU.  The GPU kernels are checked against the same oracle
in test_gpu_parity.py.  Blocks the framing marks NONDET (the reference reads
uninitialised caller memory there) are compared on frame count and CRC verdict
only.
"""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from tests.emu import emu as E

ST_NONDET = 0x80


def check(data: bytes, chunk: int = 4096):
    r = O.decode_file(data, chunk=chunk)
    n, out, crc_errors, st = E.decode(data, chunk)
    if r.status != 0:
        assert n == r.status
        return r, st
    assert n == r.frames
    assert crc_errors == r.crc_errors
    if not (st & ST_NONDET):
        assert np.array_equal(out, r.samples)
    return r, st


PCM = V.pcm_cases()
DSD = V.dsd_cases()


@pytest.mark.parametrize("name,data,chunk", PCM, ids=[c[0] for c in PCM])
def test_pcm_modes(name, data, chunk):
    r, st = check(data, chunk)
    if name.endswith("_short"):  # truncated wvx stream: the reference over-reads it and throws (B-10)
        assert r.status == -3
    else:
        assert r.status == 0 and r.crc_errors == 0


@pytest.mark.parametrize("name,data,chunk", DSD, ids=[c[0] for c in DSD])
def test_dsd_modes(name, data, chunk):
    r, st = check(data, chunk)
    assert r.status == 0 and r.crc_errors == 0


@pytest.mark.parametrize("chunk", [13, 1000, 4096])
def test_chunk_schedules(chunk):
    x = S.audio_like(15000, 2, 16, seed=21)
    for terms in (S.TERMS_FAST, S.TERMS_DEFAULT, S.TERMS_HIGH):
        check(S.encode_pcm(x, S.EncParams(terms=terms, block_samples=6000)), chunk)


@pytest.mark.parametrize("seed", range(12))
def test_corrupt_stereo(seed):
    x = S.audio_like(20000, 2, 16, seed=1)
    base = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=7000))
    check(V.corrupt(base, seed, start=200))


@pytest.mark.parametrize("seed", range(12))
def test_corrupt_mono(seed):
    m = S.audio_like(12000, 1, 16, seed=3)
    base = S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=3001))
    check(V.corrupt(base, 100 + seed, start=100), chunk=1000)


@pytest.mark.parametrize("seed", range(6))
def test_corrupt_hybrid_and_dsd(seed):
    x = S.audio_like(12000, 2, 16, seed=5)
    h = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, hybrid_bitrate=True, bitrate_x256=768,
                                    block_samples=5000))
    check(V.corrupt(h, 200 + seed, start=150))
    dd = S.dsd_random_like(9000, 2, seed=6, density=0.35)
    d = S.encode_dsd(dd, S.DsdParams(nch=2, mode=(1, 3)[seed % 2], block_samples=4000))
    check(V.corrupt(d, 300 + seed, start=150))


def test_truncated_and_ff_tail():
    x = S.audio_like(20000, 2, 16, seed=7)
    base = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=7000))
    check(base[: len(base) // 2])
    check(base[: len(base) - 37])
    check(base + b"\xff" * 64)


def test_dsd_mode0_false_stereo_exception():
    """The reference throws on DSD mode 0 + FALSE_STEREO (DsdUtils.cs:81 then :119-131)."""
    dd = np.repeat(S.dsd_random_like(6000, 1, seed=8, density=0.3), 2, axis=1)
    data = S.encode_dsd(dd, S.DsdParams(nch=2, false_stereo=True, mode=0, block_samples=3000))
    r = O.decode_file(data)
    assert r.status == -3
    n, _, _, _ = E.decode(data)
    assert n == -3


def test_file_info_matches_oracle_getters():
    """WavpackOpenFileInput + getters (WavPackUtils.cs:36-120, 346-499) through the product
    API (wvg_probe_file is host-only framing, so this runs without a GPU) vs the oracle."""
    from wavpackdecoder_amd import api
    L = O.lib()
    for name, data, _ in PCM[:8] + DSD:
        ctx = L.wvo_open(data, len(data), 0)
        try:
            wpc = api.WavpackOpenFileInput(data)
            assert api.WavpackGetErrorMessage(wpc) is None, name
            assert api.WavpackGetNumSamples(wpc) == L.wvo_get_num_samples(ctx, 0), name
            assert api.WavpackGetNumSamples(wpc, True) == L.wvo_get_num_samples(ctx, 1), name
            assert api.WavpackGetSampleRate(wpc) == L.wvo_get_sample_rate(ctx), name
            assert api.WavpackGetNumChannels(wpc) == L.wvo_get_num_channels(ctx), name
            assert api.WavpackGetBitsPerSample(wpc) == L.wvo_get_bits_per_sample(ctx), name
            assert api.WavpackGetBytesPerSample(wpc) == L.wvo_get_bytes_per_sample(ctx), name
            assert api.WavpackGetReducedChannels(wpc) == L.wvo_get_reduced_channels(ctx), name
            assert api.WavpackGetMode(wpc) == L.wvo_get_mode(ctx), name
            assert api.WavpackGetVersion(wpc) == L.wvo_get_version(ctx), name
            assert api.WavpackGetIsFloat(wpc) == bool(L.wvo_get_is_float(ctx)), name
            assert api.WavpackGetIsFive(wpc) == bool(L.wvo_get_is_five(ctx)), name
            assert api.WavpackGetFileFormat(wpc) == L.wvo_get_file_format(ctx), name
        finally:
            L.wvo_close(ctx)


def test_not_wavpack():
    from wavpackdecoder_amd import api
    assert E.file_info(b"RIFF" + b"\0" * 200)["open_ok"] == 0
    assert api.WavpackGetErrorMessage(api.WavpackOpenFileInput(b"RIFF" + b"\0" * 200))
    assert O.decode_file(b"RIFF" + b"\0" * 200).status == -2
