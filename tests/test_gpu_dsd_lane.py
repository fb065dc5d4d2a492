"""GPU parity of the DSD mode-3 lane kernel (wv_dsd_lane.hip: one lane per block,
wvg_batch_set_kernel(WVG_KERNEL_LANE)) against the oracle, bit-exact: output
bytes, per-file crc_errors, mutes (the 0x55 fills of a failed final-call CRC)
and the exception outcome (DsdUtils.cs:321-493).

The kernel takes stereo and mono (and mono false-stereo) mode-3 blocks; a block
outside its scope, or a lane whose payload window runs dry, is decoded again by
the wave-per-block kernel in the same decode (ST_REDO), so the cases cover more
blocks than one wave, mixed channel layouts and lengths in one batch, rates and
densities that move the probability tables differently, corrupted streams, and
mode-3 blocks next to modes 0/1 and PCM."""
import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_NONDET, WVG_ST_REDONE, WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


def _dsd3(frames, nch=2, fs=False, seed=0, block=5000, density=0.3, rate_i=3):
    dd = S.dsd_random_like(frames, 1 if fs else nch, seed=seed, density=density)
    if fs:
        dd = np.repeat(dd, 2, axis=1)
    return S.encode_dsd(dd, S.DsdParams(nch=nch, false_stereo=fs, mode=3, block_samples=block, rate_i=rate_i))


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
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        if r.status_or & WVG_ST_NONDET:  # (the reference reads the caller's stale buffer there)
            assert r.crc_errors == ref.crc_errors, name
            continue
        bad = np.nonzero(got != ref.samples)[0]
        assert bad.size == 0 and r.crc_errors == ref.crc_errors, \
            f"{name}: crc_errors {r.crc_errors} vs {ref.crc_errors}, {bad.size} values differ from index " \
            f"{bad[:1].tolist()}, block status {[hex(int(x)) for x in st[:8]]}"
    return st


@pytest.mark.parametrize("nch,fs", [(1, False), (2, True), (2, False)], ids=["mono", "false_stereo", "stereo"])
def test_dsd3_lanes_one_layout(nch, fs):
    files = [_dsd3(4638, nch, fs, seed=101, block=2000, density=0.3, rate_i=7),
             _dsd3(700, nch, fs, seed=102, block=777, density=0.1, rate_i=30)]
    st = _check(files, [f"ch{nch}_fs{int(fs)}#{k}" for k in range(len(files))])
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0


def test_dsd3_lanes_many_blocks():
    # more mode-3 blocks than one wave, stereo / mono / mono false stereo, varied
    # lengths (ragged waves), rates and densities
    rng = np.random.default_rng(5)
    files, names = [], []
    for k in range(150):
        kind = k % 3
        frames = int(rng.integers(1, 9000))
        block = int(rng.choice([777, 2000, 5000]))
        nch, fs = ((2, False), (1, False), (2, True))[kind]
        files.append(_dsd3(frames, nch, fs, seed=100 + k, block=block, density=float(rng.uniform(0.05, 0.6)),
                           rate_i=int(rng.integers(0, 40))))
        names.append(f"dsd3#{k}_ch{nch}_fs{int(fs)}_{frames}")
    st = _check(files, names)
    # the lane kernel decoded them (nothing handed back to the wave kernel)
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0


def test_dsd3_lanes_corrupted():
    base = [_dsd3(12000, 2, seed=31), _dsd3(12000, 1, seed=32), _dsd3(12000, 2, True, seed=33)]
    files = [V.corrupt(b, 400 + k) for k in range(8) for b in base]
    _check(files, [f"corrupt#{k}" for k in range(len(files))])


def test_dsd3_lanes_with_other_kinds():
    # mode-3 blocks in a batch with modes 0 / 1 and PCM (their own kernels), chunked calls
    files = [d for _, d, _ in V.dsd_cases()] + [d for _, d, _ in V.pcm_cases()[:6]] + \
            [_dsd3(20000, 2, seed=41), _dsd3(7000, 1, seed=42)]
    for chunk in (4096, 1000):
        _check(files, [f"mixed#{k}@{chunk}" for k in range(len(files))], chunk)


@pytest.mark.parametrize("case", V.dsd_cases(), ids=lambda c: c[0])
def test_dsd_cases_lane_route(case):
    name, data, chunk = case
    _check([data], [name], chunk)


def test_dsd3_false_stereo_mono_file_stays_in_range():
    """a mode-3 block flagged FALSE_STEREO inside a mono DSD file once
    reached the mono lane launch, which stored 2 ints a frame into a 1-int range.  The
    framing now declines such blocks (and raises the reference's exception where the
    expansion overruns the caller's buffer), and the lane kernel hands back any block
    whose store width differs from the file's.  The files around it must decode exactly."""
    from tests.test_layout_quirks import FALSE_STEREO, set_flags
    dd = S.dsd_random_like(9000, 1, seed=77, density=0.3)
    flipped = [set_flags(S.encode_dsd(dd, S.DsdParams(nch=1, mode=3, block_samples=b)), None, FALSE_STEREO)
               for b in (1500, 3000)]
    small = set_flags(S.encode_dsd(S.dsd_random_like(1500, 1, seed=78, density=0.3),
                                   S.DsdParams(nch=1, mode=3, block_samples=1500)), None, FALSE_STEREO)
    normal = [_dsd3(7000, 1, seed=79), _dsd3(5000, 2, seed=80), _dsd3(3000, 1, seed=81)]
    files = [normal[0], flipped[0], normal[1], small, flipped[1], normal[2]]
    out, res, infos, st = _run(files)
    for k in (0, 2, 5):
        ref = O.decode_file(files[k], chunk=4096)
        r, info = res[k], infos[k]
        assert r.exception == 0 and r.frames == ref.frames and r.crc_errors == ref.crc_errors, k
        np.testing.assert_array_equal(out[info.out_offset: info.out_offset + ref.frames * ref.nch], ref.samples,
                                      err_msg=str(k))
    for k in (1, 3, 4):
        ref = O.decode_file(files[k], chunk=4096)
        r = res[k]
        assert not (r.status_or & WVG_ST_TIMEOUT), k
        if ref.status == -3:
            assert r.exception == 1, k
        else:
            assert r.status_or & 0x20, k  # declined (WVG_ST_UNSUPPORTED)


@pytest.mark.parametrize("kernel", ["lane", "two_wave"])
def test_dsd_sticky_chains(kernel):
    """DSD blocks continuing the DSD (and crc / mute) state of the block before them,
    one chain per file decoded in order by the wave kernel (decode_dsd_chain; the lane
    kernels hand chain blocks back), against the oracle in one batch."""
    cases = V.dsd_sticky_cases()
    for chunk in (4096, 1000):
        sub = [c for c in cases if c[2] == chunk]
        out, res, infos, st = _run([d for _, d, _ in sub], chunk, kernel)
        for (name, data, _), r, info in zip(sub, res, infos):
            ref = O.decode_file(data, chunk=chunk)
            assert r is not None and not (r.status_or & WVG_ST_TIMEOUT), name
            assert not (r.status_or & 0x20), name  # decoded, not declined
            if ref.status == -3:
                assert r.exception == 1, name
                continue
            assert r.frames == ref.frames and r.crc_errors == ref.crc_errors, name
            if not (r.status_or & WVG_ST_NONDET):
                got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
                np.testing.assert_array_equal(got, ref.samples, err_msg=name)
