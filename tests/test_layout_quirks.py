"""Malformed layouts the reference decodes in its own way (formerly ST_UNSUPPORTED here):

* a PCM block whose ints per frame differ from the file's (UnpackUtils.cs:510-686
  writes 1 int a frame for MONO_FLAG without FALSE_STEREO, else 2 -- FALSE_STEREO's
  copy :655-664 included -- from the call's buffer position, while
  WavpackUnpackSamples advances num_channels a frame, WavPackUtils.cs:263-268):
  a 2-int block in a 1-int file shows the first n of its 2n ints, and throws when
  2n pass the caller's buffer; a 1-int block in a 2-int file leaves every other slot
  with the caller's stale buffer (ST_NONDET: the reference output depends on it);
* INT32 sent_bits past 32 with a wvx stream: BitsUtils.getbits on its 32-bit register
  (bytes past 32 bits wrap onto the low ones, C#'s masked shift) and the masked
  `1 << sent_bits` mask (UnpackUtils.cs:1271-1314).

Each case: the oracle (a restatement of the C#) against the host build of the
device decode core (tests/emu) -- frames, crc errors, exception, samples unless
NONDET; tests/test_gpu_layout_quirks.py runs the same files on the GPU."""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from tests.emu import emu as E
from tests.test_meta_defer import block_offsets

ST_UNSUPPORTED, ST_NONDET = 0x20, 0x80
MONO_FLAG, FALSE_STEREO = 0x4, 0x40000000


def set_flags(data: bytes, blocks, set_bits=0, clear_bits=0) -> bytes:
    """Set / clear header flag bits (offset 24 of a block header) in the given blocks."""
    b = bytearray(data)
    for k, o in enumerate(block_offsets(data)):
        if blocks is None or k in blocks:
            f = int.from_bytes(b[o + 24:o + 28], "little")
            f = (f | set_bits) & ~clear_bits
            b[o + 24:o + 28] = f.to_bytes(4, "little")
    return bytes(b)


def set_int32_sent_bits(data: bytes, value: int) -> bytes:
    """Overwrite ID_INT32_INFO's sent_bits byte in every block."""
    b = bytearray(data)
    for o in block_offsets(data):
        end = o + 8 + int.from_bytes(b[o + 4:o + 8], "little")
        p = o + 32
        while p + 2 <= end:
            mid = b[p]
            if mid & 0x80:
                size = (b[p + 1] | (b[p + 2] << 8) | (b[p + 3] << 16)) * 2
                hdr = 4
            else:
                size = b[p + 1] * 2
                hdr = 2
            if (mid & 0x3F) == 0x9:
                b[p + hdr] = value
            p += hdr + size
    return bytes(b)


def quirk_cases():
    x = S.audio_like(3000, 2, 16, seed=41)
    m = S.audio_like(3000, 1, 16, seed=42)
    fs = S.encode_pcm(np.repeat(m, 2, axis=1), S.EncParams(nch=2, false_stereo=True, terms=S.TERMS_MONO_HIGH,
                                                           block_samples=700))
    st = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=700))
    mo = S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=700))
    long_fs = S.encode_pcm(np.repeat(S.audio_like(9000, 1, 16, seed=43), 2, axis=1),
                           S.EncParams(nch=2, false_stereo=True, terms=S.TERMS_MONO_HIGH, block_samples=2000))
    xi = S.audio_like(3000, 2, 24, seed=44)
    out = [
        # FALSE_STEREO + MONO_FLAG everywhere: a 1-int file whose blocks write 2 ints a frame
        ("fs_monoflag", set_flags(fs, None, MONO_FLAG), 4096),
        ("fs_monoflag_chunk500", set_flags(fs, None, MONO_FLAG), 500),
        # ... past the caller's 4096-int buffer: the reference throws
        ("fs_monoflag_overrun", set_flags(long_fs, None, MONO_FLAG), 4096),
        # FALSE_STEREO + MONO_FLAG from the second block on: 2 ints a frame in a 2-int file
        ("fs_monoflag_later", set_flags(fs, {1, 2, 3}, MONO_FLAG), 4096),
        # a stereo block in a mono file (MONO_FLAG cleared after the first block)
        ("mono_file_stereo_block", set_flags(mo, {2}, clear_bits=MONO_FLAG), 4096),
        ("mono_file_stereo_block_chunk300", set_flags(mo, {1, 3}, clear_bits=MONO_FLAG), 300),
        # a mono block in a stereo file: stale slots (NONDET)
        ("stereo_file_mono_block", set_flags(st, {2}, MONO_FLAG), 4096),
    ]
    for nm, wvx, sb in (("int32_wvx_sent40", 1, 40), ("int32_wvx_sent33", 1, 33), ("int32_wvx_sent200", 1, 200),
                        ("int32_wvxnew_sent48", 2, 48), ("int32_nowvx_sent40", 0, 40)):
        base = V.int32_file(xi, sent_bits=8, wvx=wvx, max_width=20 if wvx == 2 else 0, block=1000)
        out.append((nm, set_int32_sent_bits(base, sb), 4096))
    return out


CASES = quirk_cases()


@pytest.mark.parametrize("name,data,chunk", CASES, ids=[c[0] for c in CASES])
def test_quirk_layout_host_core_vs_oracle(name, data, chunk):
    n, out, crc, st = E.decode(data, chunk)
    ref = O.decode_file(data, chunk=chunk)
    assert not (st & ST_UNSUPPORTED), name
    if ref.status == -3:
        assert n == -3, name
        return
    assert n == ref.frames and crc == ref.crc_errors, (name, n, ref.frames, crc, ref.crc_errors)
    if not (st & ST_NONDET):
        np.testing.assert_array_equal(out, ref.samples, err_msg=name)
    else:
        # the slots the block writes agree; the rest is the caller's stale buffer
        assert out.size == ref.samples.size


def test_quirk_cases_cover_each_layout():
    kinds = {nm: O.decode_file(d, chunk=c).status for nm, d, c in CASES}
    assert kinds["fs_monoflag_overrun"] == -3 and kinds["fs_monoflag"] == 0


def dsd_fs_mono_cases():
    """Mono DSD files whose blocks carry FALSE_STEREO (MONO_DATA still set): the unmuted
    call decodes n values and expands them to 2n ints (DsdUtils.cs:119-131) in a 1-int
    file -- past the caller's buffer the C# store throws.  (the lane kernel
    once wrote those 2n ints into the next block's range.)"""
    out = []
    for frames, block in ((9000, 3000), (9000, 5000), (1500, 1500)):
        for mode in (0, 1, 3):
            dd = S.dsd_random_like(frames, 1, seed=5 + mode, density=0.3)
            f = S.encode_dsd(dd, S.DsdParams(nch=1, mode=mode, block_samples=block))
            out.append((f"dsd_m{mode}_mono_fs_{frames}_{block}", set_flags(f, None, FALSE_STEREO), 4096))
    return out


@pytest.mark.parametrize("name,data,chunk", dsd_fs_mono_cases(), ids=[c[0] for c in dsd_fs_mono_cases()])
def test_dsd_false_stereo_in_mono_file(name, data, chunk):
    n, out, crc, st = E.decode(data, chunk)
    ref = O.decode_file(data, chunk=chunk)
    if ref.status == -3:  # the expansion overran the caller's buffer: the same call throws
        assert n == -3, name
        return
    # a layout the device does not decode (the first n of the 2n expanded ints): declined
    assert st & ST_UNSUPPORTED, name
    assert n == ref.frames, name
