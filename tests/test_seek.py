"""Seek: WavPackUtils.SetSample -> seek (WavPackUtils.cs:509-594).

The framing restates the reference's block search (the 25-step bisection by
average_block_size, the forward header walk, the re-open at the found block)
and its decode-and-discard calls of SAMPLE_BUFFER_SIZE / reduced-channels
frames; the device decodes the found block from its start and drops the
discarded frames.  Checked against the oracle's restatement of the same
function on the host build of the device core (CPU) and through the HIP path
(GPU): the frames the following WavpackUnpackSamples calls return, the CRC
error count and SetSample's result.  For lossless files the samples after a
successful seek must also equal the encoder's input from the target on.
"""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from tests.emu import emu as E


def _files():
    x = S.audio_like(50000, 2, 16, seed=41)
    m = S.audio_like(30001, 1, 16, seed=42)
    out = [
        ("stereo_default", S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=7000)), x),
        ("stereo_fast_small_blocks", S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=1000)), x),
        ("mono_high", S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=3001)), m),
        ("riff_header", S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, write_riff=True, block_samples=5000)), x),
    ]
    dd = S.dsd_random_like(12000, 2, seed=43, density=0.4)
    out.append(("dsd_high", S.encode_dsd(dd, S.DsdParams(nch=2, mode=3, block_samples=5000)), None))
    out.append(("dsd_fast", S.encode_dsd(dd, S.DsdParams(nch=2, mode=1, block_samples=5000)), None))
    return out


def _starts(total, block):
    s = {0, 1, block - 1, block, block + 1, 2 * block + 123, total // 2, total - block, total - 1, total, total + 7,
         4095, 4096, 4097}
    return sorted(v for v in s if v >= 0)


def test_seek_emu_matches_oracle():
    for name, data, pcm in _files():
        ref_all = O.decode_file(data)
        total = ref_all.frames
        block = {"stereo_fast_small_blocks": 1000, "mono_high": 3001}.get(name, 5000 if "dsd" in name or "riff" in name
                                                                           else 7000)
        for st in _starts(total, block):
            ref, rc = O.decode_file_from(data, st)
            n, got, crc, _, src = E.decode_from(data, st)
            assert src == rc, (name, st)
            assert n == (ref.frames if ref.status == 0 else ref.status), (name, st)
            assert crc == ref.crc_errors, (name, st)
            np.testing.assert_array_equal(got, ref.samples, err_msg=f"{name} @ {st}")
            if pcm is not None and rc == 1:
                np.testing.assert_array_equal(got, pcm[st:].reshape(-1), err_msg=f"{name} @ {st} lossless")


def test_seek_emu_matches_oracle_corrupted():
    """Corrupted streams: CRC errors and mutes inside the discarded frames and after them."""
    base = S.encode_pcm(S.audio_like(20000, 2, 16, seed=11), S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4000))
    for k in range(8):
        data = V.corrupt(base, 200 + k)
        for st in (0, 3000, 4100, 9999, 15000):
            ref, rc = O.decode_file_from(data, st)
            n, got, crc, _, src = E.decode_from(data, st)
            assert src == rc and crc == ref.crc_errors, (k, st)
            assert n == (ref.frames if ref.status == 0 else ref.status), (k, st)
            np.testing.assert_array_equal(got, ref.samples, err_msg=f"corrupt#{k} @ {st}")


@pytest.mark.gpu
def test_seek_gpu_matches_oracle(gpu_batch_cls):
    """All seeks of all files in one batch through the HIP path."""
    jobs = []
    for name, data, pcm in _files():
        total = O.decode_file(data).frames
        for st in _starts(total, 1000)[::2] + [total // 3]:
            jobs.append((name, data, st))
    b = gpu_batch_cls(4096)
    idx = [b.add_file(d, start_sample=st) for _, d, st in jobs]
    b.decode()
    out = b.download()
    res = [b.result(i) for i in idx]
    infos = list(b.infos)
    b.close()
    for (name, data, st), r, info in zip(jobs, res, infos):
        ref, rc = O.decode_file_from(data, st)
        assert info.seek_result == rc, (name, st)
        assert r.frames == ref.frames and r.crc_errors == ref.crc_errors, (name, st)
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        np.testing.assert_array_equal(got, ref.samples, err_msg=f"{name} @ {st}")
