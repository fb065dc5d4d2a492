""".wvc correction files (beyond the reference).

The reference opens ID_WVC_BITSTREAM (UnpackUtils.cs:96-106) but never reads
it, so a hybrid file decodes lossy there.  With its .wvc correction file the
decode here is exact: every word the error limit left inexact reads its exact
magnitude from the correction stream (WavPack 4 get_word: read_code(wvcbits,
high - low) + low), and the difference to the lossy residual is added to the
passes' output (the passes keep the lossy history the encoder decorrelated
against); stereo terms -1/-2, which predict one channel from the other's output
of the same pass, predict the exact value from the other channel's exact output.  No reference behaviour exists, so parity is unpinned and pinned
instead by the round trip to the encoder's input PCM, plus the .wvc headers'
CRC of the exact output; the .wv alone still decodes exactly as the oracle.
For the -1/-2 rule that round trip is circular (synth/wv_encoder.cpp encodes
with the same rule), so it stays unpinned until a WavPack-made .wvc with those
terms can be checked.

CPU: the device core built for the host (tests/emu).  GPU: test_gpu_wvc.py.
"""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests.emu import emu as E


def wvc_cases():
    """(name, wv, wvc, expected exact output, chunk)"""
    x = S.audio_like(20000, 2, 16, seed=71)
    x24 = S.audio_like(15000, 2, 24, seed=72)
    m = S.audio_like(18000, 1, 16, seed=73)
    out = []
    for name, pcm, kw, chunk in (
            ("stereo16_fast_br3", x, dict(terms=S.TERMS_FAST, hybrid_bitrate=True, bitrate_x256=768), 4096),
            ("stereo16_x3_br4_chunk13", x, dict(terms=[18, -3, 1, 17, 2, 3, -3, 18, 1], hybrid_bitrate=True,
                                                bitrate_x256=1024), 13),
            ("stereo16_nobitrate", x, dict(terms=[18, 18, 2, 3], bitrate_x256=1280), 4096),
            ("stereo16_balance", x, dict(terms=S.TERMS_FAST, hybrid_bitrate=True, hybrid_balance=True,
                                         bitrate_x256=896), 4096),
            ("stereo24_br5", x24, dict(terms=[18, 18, 2, 3, 4, 5], bytes_per_sample=3, hybrid_bitrate=True,
                                       bitrate_x256=1280), 4096),
            ("mono16_high_br3", m, dict(nch=1, terms=S.TERMS_MONO_HIGH, hybrid_bitrate=True, bitrate_x256=768), 1000),
            ("nojoint_br2", x, dict(terms=S.TERMS_FAST, joint_stereo=False, hybrid_bitrate=True, bitrate_x256=512),
             4096),
            # stereo terms -1/-2: a pass predicts one channel from the other's output of
            # the same pass (the exact value from the exact output: pass_stereo_wvc)
            ("stereo16_default_br3", x, dict(terms=S.TERMS_DEFAULT, hybrid_bitrate=True, bitrate_x256=768), 4096),
            ("stereo16_neg1_br2_chunk13", x, dict(terms=[18, -1, 2, 17, -1], hybrid_bitrate=True, bitrate_x256=512),
             13),
            ("stereo16_neg12_nobitrate", x, dict(terms=[-2, 18, -1, 3, -3, -2, 2], bitrate_x256=1024), 4096),
            ("stereo24_high_br4", x24, dict(terms=S.TERMS_HIGH, bytes_per_sample=3, hybrid_bitrate=True,
                                            bitrate_x256=1024), 4096),
            ("nojoint_default_balance", x, dict(terms=S.TERMS_DEFAULT, joint_stereo=False, hybrid_bitrate=True,
                                                hybrid_balance=True, bitrate_x256=640), 4096)):
        p = S.EncParams(block_samples=6000, **kw)
        wv, wvc = S.encode_pcm_wvc(pcm, p)
        out.append((name, wv, wvc, pcm.reshape(-1), chunk))
    # float hybrid (config C4's layout): exact ints -> the lossless float decode
    mant = S.float_mantissas(x.astype(np.float32) / 32768.0)
    wv, wvc = S.encode_pcm_wvc(mant, S.EncParams(terms=S.TERMS_FAST, bytes_per_sample=4, float_data=True,
                                                 hybrid_bitrate=True, bitrate_x256=896, block_samples=5000))
    lossless = S.encode_pcm(mant, S.EncParams(terms=S.TERMS_FAST, bytes_per_sample=4, float_data=True,
                                              block_samples=5000))
    out.append(("float_hybrid_br3", wv, wvc, E.decode(lossless)[1], 4096))
    # C4's own layout: float hybrid + bitrate with the default terms (-2 included)
    wv, wvc = S.encode_pcm_wvc(mant, S.EncParams(terms=S.TERMS_DEFAULT, bytes_per_sample=4, float_data=True,
                                                 hybrid_bitrate=True, bitrate_x256=896, block_samples=5000))
    lossless = S.encode_pcm(mant, S.EncParams(terms=S.TERMS_DEFAULT, bytes_per_sample=4, float_data=True,
                                              block_samples=5000))
    out.append(("float_hybrid_default_br3", wv, wvc, E.decode(lossless)[1], 4096))
    return out


CASES = wvc_cases()


@pytest.mark.parametrize("name,wv,wvc,exact,chunk", CASES, ids=[c[0] for c in CASES])
def test_wvc_roundtrip(name, wv, wvc, exact, chunk):
    n, s, crc_errors, status = E.decode_wvc(wv, wvc, chunk)
    assert status & 0x10000, "no block read its correction stream"
    assert crc_errors == 0  # the .wvc headers' CRC of the exact output
    np.testing.assert_array_equal(s, exact, err_msg=name)
    # the .wv alone: lossy, and exactly the reference's decode
    ref = O.decode_file(wv, chunk=chunk)
    n2, s2, ce2, _ = E.decode(wv, chunk)
    assert ce2 == ref.crc_errors == 0
    np.testing.assert_array_equal(s2, ref.samples)
    assert not np.array_equal(s2, exact), "the hybrid stream should be lossy on its own"


def test_wvc_wrong_correction_file_fails_crc():
    """a correction file of another encode: the exact-output CRC check reports every block"""
    _, wv, _, _, _ = CASES[0]
    _, _, wvc_other, _, _ = CASES[3]
    n, s, crc_errors, status = E.decode_wvc(wv, wvc_other, 4096)
    assert crc_errors > 0 or n < 0


def test_wvc_cases_cover_cross_terms():
    """the correction rule for stereo terms -1/-2 (pass_stereo_wvc) is exercised"""
    names = [c[0] for c in CASES]
    assert "stereo16_default_br3" in names and "stereo16_neg1_br2_chunk13" in names
    assert "float_hybrid_default_br3" in names
