"""GPU: a decode on a caller's stream followed at once by reset + add + re-upload.

The batch's device buffers are grow-only and reused, so wvg_batch_upload /
wvg_batch_reset must wait for the last decode wherever it ran (its `done`
event), not only for the batch's own stream.  Decoding a long file on a caller
stream and immediately refilling the batch with another file must give the
second file's exact output, and the first decode must have finished intact."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_reset_after_decode_on_caller_stream(gpu_batch_cls):
    import torch

    from synth import corpora
    from synth import wvsynth as S
    big = corpora.c2(nblocks=64)  # ~10 ms of decode: still running when reset() is called
    x = S.audio_like(30000, 2, 16, seed=77)
    small = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=7000))
    s = torch.cuda.Stream()
    b = gpu_batch_cls(4096)
    for rnd in range(3):
        b.add_file(big)
        b.upload()
        b.decode(stream=s.cuda_stream)
        b.reset()  # must wait for the decode on `s` before the buffers are reused
        assert b.add_file(small) == 0
        b.decode(stream=s.cuda_stream)
        out = b.download()
        ref = O.decode_file(small)
        assert b.result(0).crc_errors == 0
        np.testing.assert_array_equal(out[: ref.samples.size], ref.samples, err_msg=f"round {rnd}")
        b.reset()
    b.close()


def test_timing_pairs_bounded(gpu_batch_cls):
    """Timing left on over many decodes keeps a bounded set of events and still
    reports every decode (wvg_batch_timed)."""
    from synth import wvsynth as S
    x = S.audio_like(8000, 2, 16, seed=78)
    data = S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=4000))
    b = gpu_batch_cls(4096)
    b.add_file(data)
    b.upload()
    b.set_timing(True)
    for _ in range(200):
        b.decode()
    ms, n = b.timed()
    assert n == 200 and ms > 0
    b.set_timing(False)
    np.testing.assert_array_equal(b.download()[: x.size], x.reshape(-1))
    b.close()
