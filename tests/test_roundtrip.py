"""Generator -> oracle round trips (SURVEY.md §4 items 1-2, §8c "what pins results").

Lossless modes must give the generator's input PCM back bit-exactly with no
CRC error; this pins the oracle (and the generator) without any reference
fixture.  Lossy modes (hybrid, DSD) are pinned by their embedded block CRCs.
"""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S

F = 12000


def _rt(pcm, params, chunk=4096):
    data = S.encode_pcm(pcm, params)
    r = O.decode_file(data, chunk=chunk)
    assert r.status == 0
    assert r.crc_errors == 0
    return r


@pytest.mark.parametrize("terms", [S.TERMS_FAST, S.TERMS_DEFAULT, S.TERMS_HIGH], ids=["fast", "default", "high"])
@pytest.mark.parametrize("joint", [True, False])
def test_stereo16_lossless(terms, joint):
    x = S.audio_like(F, 2, 16, seed=11)
    r = _rt(x, S.EncParams(terms=terms, joint_stereo=joint, block_samples=5000))
    assert np.array_equal(r.samples, x.reshape(-1))


@pytest.mark.parametrize("bits,bps", [(8, 1), (24, 3)])
def test_other_widths(bits, bps):
    x = S.audio_like(F, 2, bits, seed=12)
    r = _rt(x, S.EncParams(terms=S.TERMS_DEFAULT, bytes_per_sample=bps, block_samples=4000))
    assert np.array_equal(r.samples, x.reshape(-1))


def test_mono_and_false_stereo():
    m = S.audio_like(F, 1, 16, seed=13)
    r = _rt(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=3001), chunk=1000)
    assert np.array_equal(r.samples, m.reshape(-1))
    fs = np.repeat(m, 2, axis=1)
    r = _rt(fs, S.EncParams(nch=2, false_stereo=True, terms=S.TERMS_MONO_HIGH[:5], block_samples=5000))
    assert np.array_equal(r.samples, fs.reshape(-1))


def test_shift_and_int32():
    x = S.audio_like(F, 2, 16, seed=14)
    r = _rt((x >> 4) << 4, S.EncParams(terms=S.TERMS_DEFAULT, shift=4))
    assert np.array_equal(r.samples, ((x >> 4) << 4).reshape(-1))
    x24 = S.audio_like(F, 2, 24, seed=15)
    x32 = (x24.astype(np.int64) << 8).astype(np.int32)
    r = _rt(x32, S.EncParams(terms=S.TERMS_DEFAULT, bytes_per_sample=4, int32_zeros=8))
    assert np.array_equal(r.samples, x32.reshape(-1))


@pytest.mark.parametrize("chunk", [13, 1000, 4096, 22050])
def test_chunk_schedule_invariant_lossless(chunk):
    """The caller's chunk size moves the (short) weight seams; lossless output must not change."""
    x = S.audio_like(F, 2, 16, seed=16)
    r = _rt(x, S.EncParams(terms=S.TERMS_HIGH, block_samples=7000), chunk=chunk)
    assert np.array_equal(r.samples, x.reshape(-1))


def test_zero_runs():
    z = S.audio_like(F, 2, 16, kind="zeros")
    r = _rt(z, S.EncParams(block_samples=5000))
    assert np.array_equal(r.samples, z.reshape(-1))


@pytest.mark.parametrize("hyb", [dict(hybrid_bitrate=True, bitrate_x256=768),
                                 dict(hybrid_bitrate=True, hybrid_balance=True, bitrate_x256=1024),
                                 dict(bitrate_x256=1280)], ids=["bitrate", "balance", "nobitrate"])
def test_hybrid_crc_clean(hyb):
    x = S.audio_like(F, 2, 16, seed=17)
    r = _rt(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, **hyb))
    assert r.lossy
    assert np.abs(r.samples.astype(np.int64) - x.reshape(-1)).max() < 4096


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_dsd_lossless(mode):
    dd = S.dsd_random_like(6000, 2, seed=18, density=0.4)
    data = S.encode_dsd(dd, S.DsdParams(nch=2, mode=mode, block_samples=3000))
    r = O.decode_file(data)
    assert r.status == 0 and r.crc_errors == 0
    assert np.array_equal(r.samples, dd.reshape(-1))
