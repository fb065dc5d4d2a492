"""GPU parity of the DSD mode-1 row kernel (wv_dsd1_lane.hip: 16 lanes per block, 4
blocks per wave; wvg_batch_set_kernel(WVG_KERNEL_LANE)) against the oracle, bit-exact:
output bytes, per-file crc_errors, mutes and the exception outcome
(DsdUtils.cs:149-304).

The kernel takes stereo and mono (and mono false-stereo) mode-1 blocks; a block
outside its scope, a symbol the reference fails, or a CRC mismatch at the block's
end goes back to the wave-per-block kernel (ST_REDO), so the cases cover every
history size (1..32 bins), run-length coded and raw tables, more blocks than one
wave, ragged lengths, corrupted streams, and mode-1 blocks next to other kinds."""
import numpy as np
import pytest

from synth import wvsynth as S
from tests import vectors as V
from tests.test_gpu_dsd_lane import _check
from wavpackdecoder_amd._lib import WVG_ST_REDONE

pytestmark = pytest.mark.gpu


def _dsd1(frames, nch=2, fs=False, seed=0, block=5000, density=0.3, hbits=5, rle=False):
    dd = S.dsd_random_like(frames, 1 if fs else nch, seed=seed, density=density)
    if fs:
        dd = np.repeat(dd, 2, axis=1)
    return S.encode_dsd(dd, S.DsdParams(nch=nch, false_stereo=fs, mode=1, block_samples=block, history_bits=hbits,
                                        rle_tables=rle))


@pytest.mark.parametrize("nch,fs", [(1, False), (2, True), (2, False)], ids=["mono", "false_stereo", "stereo"])
@pytest.mark.parametrize("rle", [False, True], ids=["raw", "rle"])
def test_dsd1_rows_one_layout(nch, fs, rle):
    files = [_dsd1(4638, nch, fs, seed=201, block=2000, density=0.3, rle=rle),
             _dsd1(700, nch, fs, seed=202, block=777, density=0.1, hbits=2, rle=rle)]
    st = _check(files, [f"ch{nch}_fs{int(fs)}_rle{int(rle)}#{k}" for k in range(len(files))])
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0


def test_dsd1_rows_every_history_size():
    files, names = [], []
    for hb in range(0, 6):
        for rle in (False, True):
            files.append(_dsd1(6000, 2, seed=300 + hb, block=3000, density=0.2 + 0.1 * hb, hbits=hb, rle=rle))
            names.append(f"hb{hb}_rle{int(rle)}")
    st = _check(files, names)
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0


def test_dsd1_rows_many_blocks():
    # more mode-1 blocks than one wave (4 a wave), stereo / mono / mono false stereo,
    # ragged lengths, densities, history sizes and table codings
    rng = np.random.default_rng(7)
    files, names = [], []
    for k in range(90):
        kind = k % 3
        frames = int(rng.integers(1, 9000))
        block = int(rng.choice([777, 2000, 5000]))
        nch, fs = ((2, False), (1, False), (2, True))[kind]
        hb = int(rng.integers(0, 6))
        rle = bool(rng.integers(0, 2))
        files.append(_dsd1(frames, nch, fs, seed=400 + k, block=block, density=float(rng.uniform(0.05, 0.7)), hbits=hb,
                           rle=rle))
        names.append(f"dsd1#{k}_ch{nch}_fs{int(fs)}_{frames}_hb{hb}")
    st = _check(files, names)
    assert int(np.count_nonzero(st & WVG_ST_REDONE)) == 0


def test_dsd1_rows_corrupted():
    base = [_dsd1(12000, 2, seed=31), _dsd1(12000, 1, seed=32), _dsd1(12000, 2, True, seed=33, rle=True)]
    files = [V.corrupt(b, 500 + k, start=120) for k in range(8) for b in base]
    _check(files, [f"corrupt#{k}" for k in range(len(files))])


def test_dsd1_rows_with_other_kinds():
    files = [d for _, d, _ in V.dsd_cases()] + [d for _, d, _ in V.pcm_cases()[:6]] + \
            [_dsd1(20000, 2, seed=41), _dsd1(7000, 1, seed=42, rle=True)]
    for chunk in (4096, 1000):
        _check(files, [f"mixed#{k}@{chunk}" for k in range(len(files))], chunk)
