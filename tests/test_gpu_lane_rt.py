"""GPU parity of the run-time term list lane kernel (wv_pcm_lane_rt: wv_lane.h RChain,
lane_blocks_rt) against the oracle, bit-exact: lossless blocks whose decorr list has no
compile-time instantiation -- any list of up to 16 terms of -3..-1, 1..8, 17, 18
(UnpackUtils.cs:156-187; the passes :688-1154) -- mono, stereo and false stereo, 5-term
lists (the reconstruction computes the word values) and longer ones, several lists in
one batch (the host gives each list waves of its own), silence, noise, ragged blocks and
corrupted streams.  With the lane kernel asked for, these blocks must decode on it: no
block of a clean stream is handed back (ST_REDONE) except full-scale noise's."""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_REDONE, WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu

# encoder order (the decoder reads them reversed); none has a lane instantiation
STEREO_LISTS = {
    "alt5": [18, 18, 2, 3, -1],
    "neg3": [17, -3, 1],
    "one": [1],
    "t1to8": [1, 2, 3, 4, 5, 6, 7, 8],
    "high10": S.TERMS_HIGH10,
    "x3": S.TERMS_X3,
    "alt16": [18, 18, 2, 3, -1, 18, 2, 4, 7, 5, 3, 6, 8, -2, 17, 2],
    "neg_all": [-1, -2, -3, -1, -2, -3],
}
MONO_LISTS = {
    "m17": [17],
    "m4": [18, 2, 3, 8],
    "m10": [18, 18, 2, 3, 17, 4, 5, 6, 7, 1],
    "m16alt": [18, 18, 2, 3, 18, 2, 4, 7, 5, 3, 6, 8, 18, 2, 1, 17],
}


def _stereo(frames, terms, kind="music", block=4000, seed=0, bits=16):
    x = S.audio_like(frames, 2, bits, seed=seed, kind=kind)
    return S.encode_pcm(x, S.EncParams(terms=terms, block_samples=block, joint_stereo=True,
                                       bytes_per_sample=bits // 8))


def _mono(frames, terms, kind="music", block=4000, seed=0, bits=16, fs=False):
    m = S.audio_like(frames, 1, bits, seed=seed, kind=kind)
    if fs:
        return S.encode_pcm(np.repeat(m, 2, axis=1), S.EncParams(nch=2, false_stereo=True, terms=terms,
                                                                 block_samples=block, bytes_per_sample=bits // 8))
    return S.encode_pcm(m, S.EncParams(nch=1, terms=terms, block_samples=block, bytes_per_sample=bits // 8))


def _check(files, names, chunk=4096, clean=False, max_redo=0):
    """Decode on the lane kernels; every file against the oracle; `clean`: at most `max_redo`
    blocks of the batch handed back."""
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(chunk)
    b.set_kernel("lane")
    idx = [b.add_file(d) for d in files]
    b.decode()
    out = b.download()
    st = b.block_status()
    for i, data, name in zip(idx, files, names):
        ref = O.decode_file(data, chunk=chunk)
        info = b.infos[i]
        if ref.status == -2:
            assert not info.open_ok, name
            continue
        r = b.result(i)
        assert not (r.status_or & WVG_ST_TIMEOUT), name
        if ref.status == -3:
            assert r.exception == 1, name
            continue
        assert r.exception == 0 and r.frames == ref.frames and r.crc_errors == ref.crc_errors, name
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        np.testing.assert_array_equal(got, ref.samples, err_msg=name)
    if clean:
        assert int(np.count_nonzero(st & WVG_ST_REDONE)) <= max_redo
    b.close()


def test_rt_stereo_lists():
    names = list(STEREO_LISTS)
    files = [_stereo(20000, STEREO_LISTS[n], seed=100 + k) for k, n in enumerate(names)]
    _check(files, names, clean=True)


def test_rt_stereo_24bit_noise_silence_ragged():
    files, names, noise = [], [], []
    for k, n in enumerate(("alt5", "high10", "alt16")):
        t = STEREO_LISTS[n]
        files += [_stereo(20000, t, seed=200 + k, bits=24), _stereo(20000, t, "zeros", seed=210 + k),
                  _stereo(12345, t, seed=230 + k, block=997)]
        names += [f"{n}_24", f"{n}_zeros", f"{n}_ragged"]
        noise.append(_stereo(20000, t, "noise", seed=220 + k))
    _check(files, names, clean=True)
    _check(noise, ["alt5_noise", "high10_noise", "alt16_noise"])  # (full-scale words: some hand-backs)


def test_rt_mono_and_false_stereo():
    files, names = [], []
    for k, (n, t) in enumerate(MONO_LISTS.items()):
        files += [_mono(20000, t, seed=300 + k), _mono(20000, t, seed=310 + k, fs=True),
                  _mono(9000, t, seed=320 + k, block=777, bits=24)]
        names += [n, f"{n}_fs", f"{n}_ragged24"]
    _check(files, names, clean=True)


def test_rt_mixed_lists_one_batch_and_chunks():
    # every list in one batch, with the instantiated lists and other kernels' blocks beside
    # them; caller chunks that cut blocks
    files = [_stereo(6000, t, seed=400 + k, block=1500) for k, t in enumerate(STEREO_LISTS.values())]
    files += [_mono(6000, t, seed=420 + k, block=1500) for k, t in enumerate(MONO_LISTS.values())]
    files += [_stereo(6000, S.TERMS_DEFAULT, seed=440), _stereo(6000, S.TERMS_FAST, seed=441),
              _stereo(6000, S.TERMS_HIGH, seed=442, bits=24)]
    names = [f"f{k}" for k in range(len(files))]
    for chunk in (4096, 1000):
        _check(files, names, chunk, clean=True)


def test_rt_corrupted_streams():
    for n in ("alt5", "alt16"):
        base = _stereo(20000, STEREO_LISTS[n], seed=500)
        _check([V.corrupt(base, k) for k in range(10)], [f"{n}_corrupt#{k}" for k in range(10)])
    base = _mono(20000, MONO_LISTS["m10"], seed=501)
    _check([V.corrupt(base, k) for k in range(6)], [f"m10_corrupt#{k}" for k in range(6)])


def test_rt_many_blocks_round_trip():
    # more blocks than a workgroup's 128 lanes, two lists interleaved in the file order
    a = S.audio_like(300 * 1000, 2, 16, seed=601)
    d1 = S.encode_pcm(a, S.EncParams(terms=STEREO_LISTS["high10"], block_samples=1000, joint_stereo=True))
    d2 = S.encode_pcm(a, S.EncParams(terms=STEREO_LISTS["alt5"], block_samples=1000, joint_stereo=True))
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(4096)
    b.set_kernel("lane")
    b.add_files([d1, d2])
    b.decode()
    out = b.download()
    st = b.block_status()
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0
    for i in range(2):
        info = b.infos[i]
        assert b.result(i).crc_errors == 0
        np.testing.assert_array_equal(out[info.out_offset: info.out_offset + a.size], a.reshape(-1))
    b.close()


# ---- hybrid blocks (HYBRID_FLAG with HYBRID_BITRATE) on the run-time list lanes ----
def _hyb(frames, terms, seed, nch=2, bits=16, flt=False, balance=False, bitrate=896, block=4000, kind="music",
         fs=False):
    x = S.audio_like(frames, 1 if fs else nch, bits, seed=seed, kind=kind)
    if fs:
        x = np.repeat(x, 2, axis=1)
    p = dict(terms=terms, hybrid=True, hybrid_bitrate=True, hybrid_balance=balance, bitrate_x256=bitrate,
             block_samples=block, nch=2 if fs else nch, false_stereo=fs)
    if flt:
        return S.encode_pcm(S.float_mantissas(x.astype(np.float32) / 32768.0),
                            S.EncParams(bytes_per_sample=4, float_data=True, **p))
    return S.encode_pcm(x, S.EncParams(bytes_per_sample=bits // 8, **p))


def test_rt_hybrid_stereo_lists_and_balance():
    # hybrid stereo on lists without a hybrid lane instantiation (the fast list, 5-term,
    # 10- and 16-term lists), HYBRID_BALANCE (WordsUtils.cs:222-241) on those and on the
    # default list's compile-time hybrid lanes; 16/24-bit integer and float
    cases = {"fast": S.TERMS_FAST, "alt5": STEREO_LISTS["alt5"], "high10": S.TERMS_HIGH10,
             "high16": S.TERMS_HIGH, "alt16": STEREO_LISTS["alt16"], "default": S.TERMS_DEFAULT}
    files, names = [], []
    for k, (n, t) in enumerate(cases.items()):
        for bal in (False, True):
            files.append(_hyb(12000, t, 700 + 2 * k + bal, balance=bal, bits=16 + 8 * (k % 2)))
            names.append(f"hy_{n}{'_bal' if bal else ''}")
        files.append(_hyb(9000, t, 720 + k, flt=True, balance=k % 2 == 0, bitrate=1200))
        names.append(f"hy_{n}_float")
    # (a float block that opens on full-scale words can outrun its lane's ring and go back,
    # as on the compile-time hybrid lanes: tests/test_gpu_hybrid_lane.py)
    _check(files, names, clean=True, max_redo=2)


def test_rt_hybrid_mono_and_false_stereo():
    files, names = [], []
    for k, t in enumerate((MONO_LISTS["m4"], S.TERMS_MONO_HIGH[:5], MONO_LISTS["m10"], MONO_LISTS["m16alt"])):
        files += [_hyb(12000, t, 800 + k, nch=1), _hyb(9000, t, 810 + k, fs=True, bitrate=1200),
                  _hyb(7000, t, 820 + k, nch=1, bits=24, block=997), _hyb(6000, t, 830 + k, nch=1, flt=True)]
        names += [f"hym{k}", f"hym{k}_fs", f"hym{k}_24_ragged", f"hym{k}_float"]
    _check(files, names, clean=True)


def test_rt_hybrid_noise_silence_corrupted():
    files = [_hyb(12000, STEREO_LISTS["alt5"], 900, kind="zeros"), _hyb(12000, S.TERMS_HIGH10, 901, kind="noise"),
             _hyb(12000, MONO_LISTS["m10"], 902, nch=1, kind="noise")]
    _check(files, ["hy_zeros", "hy_noise", "hym_noise"])
    base = _hyb(16000, S.TERMS_HIGH10, 903, balance=True)
    _check([V.corrupt(base, k) for k in range(8)], [f"hy10_corrupt#{k}" for k in range(8)])
    base = _hyb(16000, MONO_LISTS["m4"], 904, nch=1)
    _check([V.corrupt(base, k) for k in range(6)], [f"hym4_corrupt#{k}" for k in range(6)])
