"""GPU parity of the hybrid lane kernel (wv_lane.h with HY: one lane per block,
wvg_batch_set_kernel(WVG_KERNEL_LANE)) against the oracle, bit-exact: output
values, per-file crc_errors and the exception outcome.

Its scope is C4's kind of block: stereo, the default term list, HYBRID_FLAG with
HYBRID_BITRATE and no HYBRID_BALANCE, integer or float (FloatUtils.float_values
after the words).  The words follow get_word's hybrid branch (WordsUtils.cs:
update_error_limit :195-261 once per frame, the bisection :477-492, slow_level
:501-502 and its decay inside zero runs :309-317).  A block outside the scope,
or a lane whose word leaves the bounds it handles exactly, is decoded again by
the two-wave kernel in the same decode (ST_REDO -> ST_REDONE), so the cases
hold both the results and that the lane kernel kept (nearly) every block."""
import numpy as np
import pytest

from oracle import oracle as O
from synth import corpora
from synth import wvsynth as S
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_REDONE, WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


def _hy(frames, seed, bits=16, flt=False, bitrate=896, block=5000, kind="music", silence=None):
    x = S.audio_like(frames, 2, bits, seed=seed, kind=kind)
    if silence is not None:
        x[silence[0]:silence[1]] = 0
    p = dict(terms=S.TERMS_DEFAULT, hybrid=True, hybrid_bitrate=True, bitrate_x256=bitrate, block_samples=block)
    if flt:
        return S.encode_pcm(S.float_mantissas(x.astype(np.float32) / 32768.0),
                            S.EncParams(bytes_per_sample=4, float_data=True, **p))
    return S.encode_pcm(x, S.EncParams(bytes_per_sample=bits // 8, **p))


def _run(files, chunk=4096, kernel="lane"):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(chunk)
    b.set_kernel(kernel)
    idx = [b.add_file(d) for d in files]
    b.decode()
    out = b.download()
    res = [b.result(i) if i >= 0 else None for i in idx]
    infos = list(b.infos)
    st = b.block_status()
    b.close()
    return out, res, infos, st


def _check(files, names, chunk=4096):
    out, res, infos, st = _run(files, chunk)
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
        np.testing.assert_array_equal(got, ref.samples, err_msg=name)
    return st


def test_hybrid_lanes_many_blocks():
    # more hybrid blocks than one wave: integer 16 / 24 bit and float, bitrates from
    # 2 to 8 bits per sample, music / noise / silence, ragged lengths
    rng = np.random.default_rng(7)
    files, names = [], []
    for k in range(140):
        flt = k % 3 == 0
        bits = 24 if k % 3 == 1 else 16
        kind = ("music", "music", "noise", "zeros")[k % 4] if k % 7 else "music"
        frames = int(rng.integers(1, 12000))
        sil = (frames // 4, frames // 2) if k % 5 == 0 else None
        files.append(_hy(frames, 300 + k, bits=bits, flt=flt, bitrate=int(rng.integers(512, 2048)),
                         block=int(rng.choice([1000, 4410, 7000])), kind=kind, silence=sil))
        names.append(f"hy#{k}_{'f' if flt else bits}_{kind}_{frames}")
    st = _check(files, names)
    # the hybrid lane kernel decoded nearly all of them: a file that opens with full-scale
    # noise on zero medians codes its first frames as LIMIT_ONES escapes of ~15 bytes a
    # frame, past the 64 B a group the lane's ring takes in, and that block goes back
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) <= len(st) // 20


def test_hybrid_lanes_c4_blocks():
    # C4's own blocks (float32 hybrid, 22,050 frames, c2-style music / noise / silence mix)
    data = corpora.c4(nblocks=80)
    st = _check([data], ["c4x80"])
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) <= 2


def test_hybrid_lanes_corrupted():
    base = [_hy(15000, 51), _hy(15000, 52, flt=True), _hy(15000, 53, bits=24, bitrate=1500)]
    files = [V.corrupt(b, 700 + k) for k in range(8) for b in base]
    _check(files, [f"corrupt#{k}" for k in range(len(files))])


@pytest.mark.parametrize("chunk", [4096, 1000, 13])
def test_hybrid_lanes_chunks(chunk):
    # the caller's chunk schedule does not change a block's words (crc / mute at the block end)
    files = [_hy(9000, 61, block=4000), _hy(9000, 62, flt=True, block=3000)]
    _check(files, [f"chunk{chunk}#{k}" for k in range(len(files))], chunk)
