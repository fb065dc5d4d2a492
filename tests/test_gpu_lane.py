"""GPU parity of the lane-per-block kernel (wv_lane.h, wvg_batch_set_kernel
WVG_KERNEL_LANE) against the oracle, bit-exact: output, per-file crc_errors and
the exception outcome.

The lane kernel decodes the lossless stereo blocks whose term list has a
compile-time specialisation and hands every block it cannot follow exactly back
to the two-wave kernel inside the same decode (ST_REDO), so these cases cover
both sides of that split: plain music, digital silence (zero runs), full-scale
noise (long words, LIMIT_ONES escapes at block starts), corrupted streams
(bits errors, mutes, CRC errors), ragged block lengths in one wave, more blocks
than one workgroup, files the lane kernel does not take at all, and the
C2-sized batch through its lossless round trip."""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


def _decode(files, chunk=4096, kernel="lane"):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(chunk)
    b.set_kernel(kernel)
    idx = [b.add_file(d) for d in files]
    b.decode()
    out = b.download()
    res = [b.result(i) if i >= 0 else None for i in idx]
    infos = list(b.infos)
    b.close()
    return out, res, infos


def _check(files, names, chunk=4096):
    out, res, infos = _decode(files, chunk)
    for data, r, info, name in zip(files, res, infos, names):
        ref = O.decode_file(data, chunk=chunk)
        if ref.status == -2:
            assert not info.open_ok, name
            continue
        assert r is not None and not (r.status_or & WVG_ST_TIMEOUT), name
        if ref.status == -3:
            assert r.exception == 1, name
            continue
        assert r.exception == 0, name
        assert r.frames == ref.frames, name
        assert r.crc_errors == ref.crc_errors, name
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        assert np.array_equal(got, ref.samples), name


def _stereo(frames, kind="music", terms=S.TERMS_FAST, block=4000, seed=0, bits=16):
    x = S.audio_like(frames, 2, bits, seed=seed, kind=kind)
    return S.encode_pcm(x, S.EncParams(terms=terms, block_samples=block, joint_stereo=True,
                                       bytes_per_sample=bits // 8))


def test_lane_music_silence_noise():
    files = [_stereo(20000, "music", seed=1), _stereo(20000, "zeros", seed=2), _stereo(20000, "noise", seed=3),
             _stereo(20000, "music", S.TERMS_DEFAULT, seed=4), _stereo(9000, "music", seed=5, block=1500)]
    _check(files, ["music", "zeros", "noise", "default_terms", "short_blocks"])


def test_lane_ragged_wave_and_tails():
    # block lengths 1..4000 frames in one wave, incl. 1-frame and 8k+1-frame tails
    files = [_stereo(n, "music", seed=10 + k, block=b) for k, (n, b) in
             enumerate([(1, 4000), (9, 4000), (8001, 4000), (4000, 4000), (12345, 997), (777, 50)])]
    _check(files, ["one_frame", "nine", "8k+1", "exact", "ragged", "tiny_blocks"])


def test_lane_many_blocks_and_chunks():
    # more blocks than one workgroup's 128 lanes, and caller chunks that cut blocks
    x = S.audio_like(300 * 1000, 2, 16, seed=21)
    data = S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=1000, joint_stereo=True))
    for chunk in (4096, 1000, 37):
        _check([data], [f"300_blocks_chunk{chunk}"], chunk)


def test_lane_corrupted_streams():
    base = _stereo(20000, "music", S.TERMS_DEFAULT, seed=11)
    files = [V.corrupt(base, k) for k in range(12)]
    _check(files, [f"corrupt#{k}" for k in range(12)])


def test_lane_mixed_batch_with_other_kernels():
    # blocks the lane kernel does not take (mono, 24-bit high lists, hybrid, int32, DSD)
    # share the batch with ones it does
    cases = {n: d for n, d, c in V.pcm_cases()}
    names = [n for n in ("stereo16_default", "stereo16_fast", "shift4", "zeros", "noise", "mono16_high",
                         "hybrid_bitrate", "int32_wvx_short", "stereo24_high", "false_stereo")
             if n in cases]
    files = [cases[n] for n in names] + [_stereo(5000, "music", seed=31)]
    _check(files, names + ["lane_music"])


def test_lane_c2_round_trip():
    from synth import corpora
    pcm, data = corpora.c2(return_pcm=True)
    out_l, res_l, _ = _decode([data], kernel="lane")
    assert res_l[0].crc_errors == 0
    assert np.array_equal(out_l, pcm.reshape(-1))


def test_lane_high16_list():
    # WavPack's 16-term 'high' list (C3's), a lane-only specialisation: 24- and
    # 16-bit, noise (large medians: some blocks go back to the pipelined kernel),
    # digital silence, ragged blocks and corrupted streams
    files = [_stereo(20000, "music", S.TERMS_HIGH, seed=41, bits=24),
             _stereo(20000, "noise", S.TERMS_HIGH, seed=42, bits=24),
             _stereo(12345, "music", S.TERMS_HIGH, seed=43, block=997),
             _stereo(20000, "zeros", S.TERMS_HIGH, seed=44, bits=24)]
    _check(files, ["high24_music", "high24_noise", "high16_ragged", "high24_zeros"])
    base = _stereo(20000, "music", S.TERMS_HIGH, seed=45, bits=24)
    _check([V.corrupt(base, k) for k in range(8)], [f"high_corrupt#{k}" for k in range(8)])


def test_lane_c3_round_trip():
    from synth import corpora
    pcm, data = corpora.c3(nblocks=24, return_pcm=True)
    out_l, res_l, _ = _decode([data], kernel="lane")
    assert res_l[0].crc_errors == 0
    assert np.array_equal(out_l, pcm.reshape(-1))


def _mono(frames, kind="music", terms=S.TERMS_MONO_HIGH[:5], block=4000, seed=0, bits=16, fs=False):
    m = S.audio_like(frames, 1, bits, seed=seed, kind=kind)
    if fs:
        return S.encode_pcm(np.repeat(m, 2, axis=1), S.EncParams(nch=2, false_stereo=True, terms=terms,
                                                                 block_samples=block, bytes_per_sample=bits // 8))
    return S.encode_pcm(m, S.EncParams(nch=1, terms=terms, block_samples=block, bytes_per_sample=bits // 8))


def test_lane_mono_and_false_stereo():
    # the mono lane kernel: WavPack's mono default list (5 terms) and 16-term mono list,
    # 16/24-bit, false stereo (stored twice), silence, noise, ragged and corrupted streams
    files = [_mono(20000, seed=51), _mono(20000, seed=52, fs=True), _mono(20000, "noise", seed=53),
             _mono(20000, "zeros", seed=54), _mono(12345, seed=55, block=997),
             _mono(20000, terms=S.TERMS_MONO_HIGH, seed=56, bits=24),
             _mono(20000, "noise", terms=S.TERMS_MONO_HIGH, seed=57, bits=24),
             _mono(9001, terms=S.TERMS_MONO_HIGH, seed=58, bits=24, fs=True)]
    _check(files, ["m5", "m5_fs", "m5_noise", "m5_zeros", "m5_ragged", "mhigh24", "mhigh24_noise", "mhigh24_fs"])
    base = _mono(20000, seed=59)
    _check([V.corrupt(base, k) for k in range(6)], [f"mono_corrupt#{k}" for k in range(6)])
    for chunk in (1000, 37):
        _check([_mono(9000, seed=60, block=3000), _mono(9000, seed=61, fs=True, block=3000)], ["m_chunk", "fs_chunk"],
               chunk)
