"""GPU: the default kernel choice (WVG_KERNEL_AUTO) follows what the context does now,
not what it once did.  A batch decoded alone gets the per-block
latency kernels for groups up to kAutoLaneMin blocks; a decode issued while another
batch of the context runs, and every decode for a second after that, gets the lane
kernels; a second later, alone again, the latency kernels again.  Results are the same
either way (the parity tests); this checks the route (wvg_batch_lane_groups)."""
import time

import pytest

from synth import wvsynth as S

pytestmark = pytest.mark.gpu


def _batch(data):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(4096)
    b.set_kernel("auto")
    b.add_file(data)
    b.upload()
    return b


def test_auto_choice_expires():
    x = S.audio_like(256 * 22050, 2, 16, seed=7)
    data = S.encode_pcm_parallel(x, S.EncParams(terms=S.TERMS_FAST, block_samples=22050, joint_stereo=True))
    b1, b2 = _batch(data), _batch(data)
    time.sleep(1.2)  # (earlier tests' overlapping batches are past the hold time)
    b1.decode()
    b1.sync()
    assert b1.lane_groups() == 0  # alone: the two-wave kernel
    b1.decode()
    b2.decode()  # issued while b1 runs (256 blocks: milliseconds)
    assert b2.lane_groups() != 0
    b1.sync()
    b2.sync()
    b1.decode()  # alone, within the hold time: still lanes
    b1.sync()
    assert b1.lane_groups() != 0
    time.sleep(1.2)
    b1.decode()  # alone again after it: the latency kernel
    b1.sync()
    assert b1.lane_groups() == 0
    out1 = b1.download()
    out2 = b2.download()
    assert (out1 == x.reshape(-1)).all() and (out2 == x.reshape(-1)).all()
    b1.close()
    b2.close()
