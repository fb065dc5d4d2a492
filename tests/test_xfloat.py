"""Exact float output (WVG_OPEN_EXACT_FLOAT; SURVEY.md §8f-4, beyond the reference).

The reference turns a FLOAT_DATA block's integers into 24-bit PCM
(FloatUtils.cs:32-56) and never reads the block's wvx stream, although it opens
it (init_wvx_bitstream, UnpackUtils.cs:115-147) and marks the file lossy for the
float flags that need it (UnpackUtils.cs:62-63).  With the open flag the decode
is WavPack 4's float_values instead: float32 bit patterns, exact when the block
carries its wvx stream (the bits the shift to the block's largest exponent
dropped, the floats it took to 0, -0.0, inf/nan).  No reference behaviour
exists, so parity is unpinned and pinned instead by the round trip to the
encoder's float input, bit for bit, plus the wvx header's crc of the output;
without the flag the same files decode exactly as the oracle.

CPU: the device core built for the host (tests/emu).  GPU: test_gpu_xfloat.py.
"""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests.emu import emu as E

EXACT = 0x40000000  # WVG_OPEN_EXACT_FLOAT
ST_CRC_ERROR, ST_UNSUPPORTED = 0x2, 0x20


def _bits(x):
    return np.ascontiguousarray(x, dtype=np.float32).view(np.int32).reshape(-1)


def _specials(x):
    """-0.0, inf, -inf, nan, denormals and values far below the block's range"""
    x = x.copy()
    n = x.shape[0]
    c = x.shape[1] - 1
    for i, v in enumerate((-0.0, np.inf, -np.inf, np.nan, 1e-40, -3e-39, 1e-30, -2.5e-20, 0.0, 7e-8)):
        x[(97 * i + 13) % n, i % (c + 1)] = v
    return x


def _ones_pattern(x, same=False):
    """floats whose bits below the block's largest exponent are all ones
    (FLOAT_SHIFT_ONES) or, with `same`, all ones or all zeros (FLOAT_SHIFT_SAME)"""
    b = _bits(x).astype(np.uint32).reshape(x.shape)
    e = (b >> 23) & 0xFF
    me = 126  # audio_like / 32768 stays below 1.0 and reaches 0.5
    sc = np.clip(me - e.astype(np.int64), 0, 23).astype(np.uint32)
    mask = ((np.uint64(1) << sc.astype(np.uint64)) - np.uint64(1)).astype(np.uint32)
    nz = e > 0
    sel = np.ones_like(nz) if not same else (np.arange(b.size).reshape(b.shape) % 3 == 0)
    b = np.where(nz & sel, b | mask, np.where(nz, b & ~mask, b))
    return b.astype(np.uint32).view(np.float32)


def xfloat_cases():
    """(name, wv, wvc or None, float input, chunk)"""
    a = S.audio_like(12000, 2, 16, seed=81).astype(np.float32) / 32768.0
    a24 = S.audio_like(9000, 2, 24, seed=82).astype(np.float32) / 8388608.0
    rng = np.random.default_rng(83)
    fine = (a + rng.normal(0, 1e-6, a.shape)).astype(np.float32)  # mantissas below 2^-24: SHIFT_SENT
    m = (S.audio_like(10000, 1, 16, seed=84).astype(np.float32) / 32768.0 * 1.37).astype(np.float32)
    out = []

    def add(name, x, chunk=4096, wvc=False, **kw):
        p = S.EncParams(block_samples=kw.pop("block_samples", 5000), **kw)
        r = S.encode_float_exact(x, p, wvc=wvc)
        wv, c = r if wvc else (r, None)
        out.append((name, wv, c, x, chunk))

    add("ints16_nowvx", a, terms=S.TERMS_FAST)
    add("fine_sent", fine, terms=S.TERMS_DEFAULT)
    add("fine_specials_chunk13", _specials(fine), chunk=13, terms=S.TERMS_FAST, block_samples=4000)
    add("a24_high_nowvx", a24, terms=S.TERMS_HIGH)
    add("shift_ones_nowvx", _ones_pattern(a), terms=S.TERMS_FAST)
    add("shift_same", _ones_pattern(a, same=True), terms=S.TERMS_FAST)
    add("mono_specials", _specials((m + rng.normal(0, 3e-7, m.shape)).astype(np.float32).reshape(-1, 1)), nch=1,
        terms=S.TERMS_MONO_HIGH, chunk=1000)
    lr = np.repeat(fine[:, :1], 2, axis=1)
    add("false_stereo", lr, false_stereo=True, terms=[17, 2, 3])
    add("hybrid_wvc", _specials(fine), wvc=True, terms=S.TERMS_FAST, hybrid_bitrate=True, bitrate_x256=896)
    add("hybrid_wvc_mono", (m + rng.normal(0, 3e-7, m.shape)).astype(np.float32).reshape(-1, 1), wvc=True, nch=1,
        terms=S.TERMS_MONO_HIGH, hybrid_bitrate=True, bitrate_x256=768, chunk=1000)
    return out


CASES = xfloat_cases()


@pytest.mark.parametrize("name,wv,wvc,x,chunk", CASES, ids=[c[0] for c in CASES])
def test_xfloat_roundtrip(name, wv, wvc, x, chunk):
    n, s, crc_errors, status = E.decode_wvc(wv, wvc, chunk, EXACT)
    assert crc_errors == 0 and not (status & ST_UNSUPPORTED), name
    ref_bits = _bits(x)
    if x.shape[1] == 1:
        assert s.size == ref_bits.size
    np.testing.assert_array_equal(s, ref_bits[: s.size] if x.shape[1] > 1 else ref_bits, err_msg=name)
    if "nowvx" not in name:
        assert status & 0x20000, "no block read a wvx stream"
    # without the flag: the reference's 24-bit integers, exactly as the oracle
    n2, s2, ce2, _ = E.decode_wvc(wv, None, chunk, 0)
    ref = O.decode_file(wv, chunk=chunk)
    assert ce2 == ref.crc_errors
    np.testing.assert_array_equal(s2, ref.samples)


def _subblocks(wv):
    """(id, payload offset, payload length) of every sub-block of every block"""
    out, pos = [], 0
    while pos + 32 <= len(wv):
        ck = int.from_bytes(wv[pos + 4: pos + 8], "little")
        end, p = pos + 8 + ck, pos + 32
        while p + 2 <= end:
            i, bl, hl = wv[p], wv[p + 1] * 2, 2
            if i & 0x80:
                bl += (wv[p + 2] << 9) + (wv[p + 3] << 17)
                hl = 4
            out.append((i, p + hl, bl - (1 if i & 0x40 else 0)))
            p += hl + bl
        pos = end
    return out


# FLOAT_INFO flags each case must exercise (OR over its blocks): SHIFT_ONES 1,
# SHIFT_SAME 2, SHIFT_SENT 4, ZEROS_SENT 8, NEG_ZEROS 0x10, EXCEPTIONS 0x20
FLAGS = {"ints16_nowvx": 0, "fine_sent": 4, "fine_specials_chunk13": 0x3C, "a24_high_nowvx": 0,
         "shift_ones_nowvx": 1, "shift_same": 2, "mono_specials": 0x3C, "false_stereo": 4, "hybrid_wvc": 0x3C,
         "hybrid_wvc_mono": 4}


@pytest.mark.parametrize("name,wv,wvc,x,chunk", CASES, ids=[c[0] for c in CASES])
def test_xfloat_cases_cover_float_flags(name, wv, wvc, x, chunk):
    fl = 0
    for i, o, ln in _subblocks(wv):
        if (i & 0x3F) == 0x08:
            fl |= wv[o]
    assert fl == FLAGS[name]


def _wvx_payloads(wv):
    """(offset, length) of each block's classic ID_WVX_BITSTREAM payload"""
    return [(o, ln) for i, o, ln in _subblocks(wv) if (i & 0x3F) == 0x0C and not (i & 0x20)]


def test_xfloat_damaged_wvx_fails_crc():
    """a flipped wvx byte: the wvx crc check reports the block (and only that block)"""
    name, wv, _, x, chunk = CASES[1]
    offs = _wvx_payloads(wv)
    assert len(offs) >= 2
    o, ln = offs[0]
    bad = bytearray(wv)
    bad[o + 4 + ln // 2] ^= 0x5A
    n, s, crc_errors, status = E.decode_wvc(bytes(bad), None, chunk, EXACT)
    assert crc_errors == 1 and (status & ST_CRC_ERROR)


def test_xfloat_zeroed_wvx_tail_fails_crc():
    """a wvx stream whose last bytes are zeroed -> crc error"""
    name, wv, _, x, chunk = CASES[2]
    o, ln = _wvx_payloads(wv)[0]
    bad = bytearray(wv)
    bad[o + ln - 8: o + ln] = b"\0" * 8
    _, _, crc_errors, _ = E.decode_wvc(bytes(bad), None, chunk, EXACT)
    assert crc_errors >= 1


def test_xfloat_flag_ignored_for_integer_files():
    """the flag changes nothing for PCM that is not FLOAT_DATA"""
    x = S.audio_like(6000, 2, 16, seed=85)
    wv = S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=4000))
    a = E.decode_wvc(wv, None, 4096, EXACT)
    b = E.decode_wvc(wv, None, 4096, 0)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[1], x.reshape(-1))
