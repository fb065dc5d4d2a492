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


def _enc(x, nch=2, **kw):
    p = dict(terms=S.TERMS_DEFAULT if nch == 2 else S.TERMS_MONO_HIGH, block_samples=4000, nch=nch)
    p.update(kw)
    return S.encode_pcm(x, S.EncParams(**p))


def test_hybrid_lanes_without_bitrate():
    """Hybrid blocks without HYBRID_BITRATE (error limit exp2s(bitrate) alone, WordsUtils.cs:209,
    256-258) on the lanes: stereo on the default list (kHyDefault) and on run-time lists, mono;
    16 / 24 bit and float; bitrates 1 to 8 bits per sample."""
    files, names = [], []
    for k in range(24):
        bits = 24 if k % 3 == 1 else 16
        flt = k % 3 == 2
        nch = 1 if k % 4 == 3 else 2
        x = S.audio_like(int(3000 + 700 * k), nch, bits, seed=900 + k, kind="noise" if k % 5 == 4 else "music")
        terms = (S.TERMS_DEFAULT, S.TERMS_HIGH, S.TERMS_FAST)[k % 3] if nch == 2 else S.TERMS_MONO_HIGH[: 5 + k % 3]
        kw = dict(terms=terms, hybrid=True, hybrid_bitrate=False, bitrate_x256=256 + 96 * k)
        if flt:
            files.append(_enc(S.float_mantissas(x.astype(np.float32) / 32768.0), nch, bytes_per_sample=4,
                              float_data=True, **kw))
        else:
            files.append(_enc(x, nch, bytes_per_sample=bits // 8, **kw))
        names.append(f"nobr#{k}_{'f' if flt else bits}_{nch}ch")
    st = _check(files, names)
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) <= max(1, len(st) // 20)


def test_int32_blocks_on_lanes():
    """INT32_DATA blocks without a wvx stream: hybrid (fixup_tail: zeros / ones / dups, or the
    sent_bits shift, then the 4-byte clip; UnpackUtils.cs:1318-1393) on the hybrid lanes, and
    lossless ones whose fixup is a shift (sent_bits) on the lossless lanes."""
    from tests import vectors as V
    x = S.audio_like(9000, 2, 16, seed=77)
    m = S.audio_like(9000, 1, 16, seed=78)
    files, names = [], []
    for k, lay in enumerate((dict(zeros=3), dict(ones=2), dict(dups=4), dict(sent_bits=5), dict(sent_bits=9))):
        y = S.int32_layout(x, seed=80 + k, **lay)
        kw = {("int32_" + a): v for a, v in lay.items()}
        for br in (True, False):
            files.append(_enc(y, bytes_per_sample=4, hybrid=True, hybrid_bitrate=br, bitrate_x256=700, **kw))
            names.append(f"int32_hy_{list(lay)[0]}_br{int(br)}")
        ym = S.int32_layout(m, seed=90 + k, **lay)
        files.append(_enc(ym, nch=1, bytes_per_sample=4, hybrid=True, hybrid_bitrate=True, bitrate_x256=700, **kw))
        names.append(f"int32_hy_mono_{list(lay)[0]}")
    for k, sb in enumerate((4, 11)):  # lossless, the fixup a shift (no wvx: its bits are lost)
        files.append(V.int32_file(x, sent_bits=sb, seed=95 + k))
        names.append(f"int32_ll_sent{sb}")
    for k, z in enumerate((3, 12)):  # lossless, zeros alone: `<<= zeros` ahead of the header shift
        files.append(V.int32_file(x, zeros=z, seed=97 + k))
        names.append(f"int32_ll_zeros{z}")
    st = _check(files, names)
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) <= max(1, len(st) // 20)
