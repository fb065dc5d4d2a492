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


def test_decode_server_producers_consumers(gpu_batch_cls):
    """The serving pattern bench.py's pipelined leg uses: producer threads
    take a free batch and call reset / add_files / upload / decode / format, none of which
    waits for the device (round 6), consumer threads download the queued PCM (page-locked)
    and free the batch.  Every request's PCM -- three different file sets, 24 requests over
    5 batches -- must be the oracle's 16-bit image of its files."""
    import queue
    import threading

    from synth import wvsynth as S
    sets = []
    for k in range(3):
        files = [S.encode_pcm(S.audio_like(9000 + 4000 * j + 1000 * k, 2, 16, seed=300 + 10 * k + j),
                              S.EncParams(terms=(S.TERMS_DEFAULT, S.TERMS_FAST, S.TERMS_HIGH)[(j + k) % 3],
                                          block_samples=3000 + 500 * j)) for j in range(4)]
        want = np.concatenate([np.ascontiguousarray(O.decode_file(f).samples.astype("<i2")).view(np.uint8)
                               for f in files])
        sets.append((files, want))
    pool = [gpu_batch_cls(4096) for _ in range(5)]
    free, ready = queue.Queue(), queue.Queue()
    for x in pool:
        free.put(x)
    jobs = list(range(24))
    lock = threading.Lock()
    bad = []

    def produce():
        while True:
            with lock:
                if not jobs:
                    return
                r = jobs.pop(0)
            x = free.get()
            x.reset()
            x.add_files(sets[r % 3][0])
            x.upload()
            x.decode()
            x.format()
            ready.put((r, x))

    def consume():
        while True:
            item = ready.get()
            if item is None:
                return
            r, x = item
            got = x.download_pcm(pinned=True)
            # (16-byte aligned file images: compare file by file)
            want_files = sets[r % 3][0]
            offs = [x.pcm_offset(i) for i in range(len(want_files))]
            parts = [got[o: o + x.infos[i].out_frames * 4] for i, o in enumerate(offs)]
            if not np.array_equal(np.concatenate(parts), sets[r % 3][1]):
                bad.append(r)
            free.put(x)
    ps = [threading.Thread(target=produce) for _ in range(3)]
    cs = [threading.Thread(target=consume) for _ in range(2)]
    for t in ps + cs:
        t.start()
    for t in ps:
        t.join()
    for _ in cs:
        ready.put(None)
    for t in cs:
        t.join()
    for x in pool:
        x.close()
    assert not bad, f"requests with wrong PCM: {bad}"
