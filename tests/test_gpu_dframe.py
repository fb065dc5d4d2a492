"""GPU: device-side framing (wvg_batch_add_files_device, wv_dframe.hip) decodes every
file exactly like the host framing, and exactly like the oracle.

The device framer handles the regular files (most of a corpus) and hands the rest
to the host framing at the same upload; the per-file output, results and .wav
images must not depend on which side framed a file."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


def _per_file(b, n):
    out = b.download()
    files = []
    for i in range(n):
        info = b.infos[i]
        if not info.open_ok:
            files.append(None)
            continue
        r = b.result(i)
        assert not (r.status_or & WVG_ST_TIMEOUT)
        seg = out[info.out_offset: info.out_offset + r.frames * info.reduced_channels].copy()
        files.append((seg, r.frames, r.crc_errors, r.exception, r.status_or, b.wav(i)))
    return files


def test_device_framing_matches_host_framing(gpu_batch_cls):
    from synth import corpora
    files = [c[1] for c in V.pcm_cases() + V.dsd_cases()] + corpora.c5(60) + \
        [c[1] for c in V.sticky_cases()[:6]] + [b"", b"RIFF" + b"\0" * 60, b"\0" * 40 + V.pcm_cases()[0][1]]
    a = gpu_batch_cls(4096)
    ia = a.add_files(files, threads=8)
    a.decode()
    a.format()
    fa = _per_file(a, len(files))
    b = gpu_batch_cls(4096)
    ib = b.add_files_device(files)
    assert ib == list(range(len(files)))
    b.decode()
    b.format()
    dev, host = b.framing_stats()
    fb = _per_file(b, len(files))
    # regular PCM files framed on the device; DSD, wvx, sticky, junk and empty ones by the host
    assert dev >= 40 and host >= 10 and dev + host == len(files), (dev, host)
    for k in range(len(files)):
        assert (ia[k] < 0) == (fa[k] is None) == (fb[k] is None), k
        if fa[k] is None:
            continue
        np.testing.assert_array_equal(fa[k][0], fb[k][0], err_msg=str(k))
        assert fa[k][1:5] == fb[k][1:5], k
        assert fa[k][5] == fb[k][5], k  # WvDemo .wav image
        ai, bi = a.infos[ia[k]], b.infos[k]
        for f in ("num_channels", "bits_per_sample", "bytes_per_sample", "sample_rate", "total_samples", "mode",
                  "version", "is_float", "lossy"):
            assert getattr(ai, f) == getattr(bi, f), (k, f)
    a.close()
    b.close()


@pytest.mark.parametrize("name,data,chunk", [c for c in V.pcm_cases() if "wvx" not in c[0]][:12],
                         ids=[c[0] for c in V.pcm_cases() if "wvx" not in c[0]][:12])
def test_device_framed_vs_oracle(gpu_batch_cls, name, data, chunk):
    ref = O.decode_file(data, chunk=chunk)
    b = gpu_batch_cls(chunk)
    b.add_files_device([data])
    b.decode()
    assert b.framing_stats() == (1, 0), name
    out = b.download()
    r, info = b.result(0), b.infos[0]
    assert r.exception == 0 and r.frames == ref.frames and r.crc_errors == ref.crc_errors, name
    np.testing.assert_array_equal(out[info.out_offset: info.out_offset + ref.frames * ref.nch], ref.samples,
                                  err_msg=name)
    b.close()


def test_c2_device_framed_roundtrip(gpu_batch_cls):
    """the 1,024-block C2 file framed on the device decodes to the encoder's input"""
    from synth import corpora
    pcm, data = corpora.c2(return_pcm=True)
    b = gpu_batch_cls(4096)
    b.add_files_device([data])
    b.decode()
    assert b.framing_stats() == (1, 0)
    assert b.num_blocks == 1024
    out = b.download()
    r = b.result(0)
    assert r.crc_errors == 0 and r.exception == 0
    np.testing.assert_array_equal(out[: pcm.size], pcm.reshape(-1))
    b.close()


def _fake_header(data: bytes, block: int, at: int, target: int) -> bytes:
    """`data` with a header-shaped 32 bytes written inside block `block`'s payload (at
    `at` bytes before its end, even offset) whose ckSize points at byte `target`"""
    off, n = V.block_spans(data)[block]
    p = off + n - at
    p -= p & 1
    hdr = bytearray(data[off:off + 32])
    hdr[4:8] = (target - p - 8).to_bytes(4, "little")
    b = bytearray(data)
    b[p:p + 32] = hdr
    return bytes(b)


def _rank_all(gpu_batch_cls, files, chunk=4096):
    """device framing with every file on the parallel header walk vs the host framing"""
    import os
    old = os.environ.get("WVG_DFRAME_RANK_MIN")
    os.environ["WVG_DFRAME_RANK_MIN"] = "0"
    try:
        b = gpu_batch_cls(chunk)
    finally:
        if old is None:
            os.environ.pop("WVG_DFRAME_RANK_MIN")
        else:
            os.environ["WVG_DFRAME_RANK_MIN"] = old
    a = gpu_batch_cls(chunk)
    a.add_files(files, threads=8)
    a.decode()
    a.format()
    fa = _per_file(a, len(files))
    b.add_files_device(files)
    b.decode()
    b.format()
    fb = _per_file(b, len(files))
    for k in range(len(files)):
        assert (fa[k] is None) == (fb[k] is None), k
        if fa[k] is not None:
            np.testing.assert_array_equal(fa[k][0], fb[k][0], err_msg=str(k))
            assert fa[k][1:5] == fb[k][1:5], k
    stats = b.framing_stats()
    a.close()
    b.close()
    return stats


def test_parallel_header_walk_matches_host(gpu_batch_cls):
    """the scan + list-ranking walk (forced for every file) against the host framing, incl.
    files with header-shaped bytes inside a payload: a dead chain (ignored), a chain
    merging into the true one (rank collision -> serial walk), junk at the head/tail"""
    from synth import corpora
    base = V.pcm_cases()[2][1]
    spans = V.block_spans(base)
    fakes = [_fake_header(base, 1, 200, spans[2][0]),             # merges into block 2
             _fake_header(base, 1, 300, len(base) + 1000),         # points past the end
             _fake_header(base, 0, 500, spans[0][0] + spans[0][1] + 6),  # points between headers
             _fake_header(base, len(spans) - 1, 100, len(base))]   # a second chain end at the file end
    files = [c[1] for c in V.pcm_cases()] + corpora.c5(30) + fakes + \
        [b"\0" * 40 + base, base + b"\0" * 40, base[:len(base) - 100]]
    dev, host = _rank_all(gpu_batch_cls, files)
    assert dev >= 30, (dev, host)


def test_parallel_header_walk_c2(gpu_batch_cls):
    """the 1,024-block C2 file takes the parallel walk by default (over 256 KiB)"""
    from synth import corpora
    pcm, data = corpora.c2(return_pcm=True)
    b = gpu_batch_cls(4096)
    b.add_files_device([data])
    b.decode()
    assert b.framing_stats() == (1, 0) and b.num_blocks == 1024
    out = b.download()
    np.testing.assert_array_equal(out[: pcm.size], pcm.reshape(-1))
    b.close()


def test_device_framing_twice_without_reset(gpu_batch_cls):
    """Files added after an upload (device- and host-framed, no reset): the earlier
    device-framed descriptors, kept on the device, survive the second device pass."""
    from synth import corpora
    first = corpora.c5(30)
    second = corpora.c5(20, start=30)
    extra = [c[1] for c in V.pcm_cases()[:3]]
    b = gpu_batch_cls(4096)
    b.add_files_device(first)
    b.upload()
    b.add_files(extra)
    b.add_files_device(second)
    b.decode()
    out = b.download()
    files = first + extra + second
    assert b.framing_stats()[0] >= 30
    for k, f in enumerate(files):
        ref = O.decode_file(f, chunk=4096)
        info = b.infos[k]
        r = b.result(k)
        assert r.exception == 0 and r.frames == ref.frames and r.crc_errors == ref.crc_errors, k
        np.testing.assert_array_equal(out[info.out_offset: info.out_offset + ref.frames * ref.nch], ref.samples,
                                      err_msg=str(k))
    b.close()
