"""GPU parity: the HIP path (through the C-ABI) vs the oracle, bit-exact.

The bar is bit-exact int32 output, the same per-file crc_errors and the same
exception outcome as the reference's WvDemo loop (restated by oracle/)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import vectors as V
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


# kernel routes: "2wave" (the product routing: compile-time shallow term lists,
# the pipelined kernel for every other list, the generic kernel for int32+wvx),
# "generic" (the wave-per-block kernel for every PCM block), "pipe" (the
# pipelined kernel for every PCM block without wvx), "lane" (the throughput
# kernel, wvg_batch_set_kernel(WVG_KERNEL_LANE): one lane per block for every
# instantiated lossless list, its hand-backs and every other block as "2wave")
ROUTES = {"2wave": {}, "generic": {"WVG_FORCE_LANE": "1"}, "pipe": {"WVG_PIPE": "2"},
          "lane": {"WVG_LANE_KERNEL": "1"}, False: {}, True: {"WVG_FORCE_LANE": "1"}}
ROUTE_VARS = ("WVG_FORCE_LANE", "WVG_PIPE", "WVG_LANE_KERNEL")


def _gpu_decode(files, chunk, batch_cls, force_lane=False):
    import os
    env = {k: ROUTES[force_lane].get(k, "0") for k in ROUTE_VARS}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        b = batch_cls(chunk)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    idx = [b.add_file(d) for d in files]
    b.decode()
    out = b.download()
    res = [b.result(i) if i >= 0 else None for i in idx]
    infos = list(b.infos)
    b.close()
    return out, res, infos


def _check_one(data, chunk, batch_cls, name, force_lane=False):
    ref = O.decode_file(data, chunk=chunk)
    out, res, infos = _gpu_decode([data], chunk, batch_cls, force_lane)
    r, info = res[0], infos[0]
    # a kernel timeout is never a reference outcome (result() raises DecoderTimeout too)
    assert r is None or not (r.status_or & WVG_ST_TIMEOUT), name
    if ref.status == -2:
        assert not info.open_ok, name
        return
    assert r is not None, name
    if ref.status == -3:
        assert r.exception == 1, name
        return
    assert r.exception == 0, name
    assert r.frames == ref.frames, name
    assert r.crc_errors == ref.crc_errors, name
    got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
    np.testing.assert_array_equal(got, ref.samples, err_msg=name)


@pytest.mark.parametrize("lane", ["2wave", "generic", "pipe", "lane"])
@pytest.mark.parametrize("case", V.pcm_cases(), ids=lambda c: c[0])
def test_pcm_modes(case, lane, gpu_batch_cls):
    name, data, chunk = case
    _check_one(data, chunk, gpu_batch_cls, name, force_lane=lane)


@pytest.mark.parametrize("case", V.dsd_cases(), ids=lambda c: c[0])
def test_dsd_modes(case, gpu_batch_cls):
    name, data, chunk = case
    _check_one(data, chunk, gpu_batch_cls, name)


@pytest.mark.parametrize("case", V.sticky_cases() + V.term0_cases(), ids=lambda c: c[0])
def test_sticky_state_chains(case, gpu_batch_cls):
    """Blocks continuing the previous decode's state (B-8): one chain per file run
    in order by wv_decode_pcm_wave, bit-exact with the oracle (tests/test_sticky.py);
    and stereo term 0, whose decode depends on the call seams (generic kernel)."""
    name, data, chunk = case
    _check_one(data, chunk, gpu_batch_cls, name)


def test_sticky_passes_lossless(gpu_batch_cls):
    """Files that decode correctly only by continuing the passes: back to the input PCM."""
    cases = V.sticky_clean_cases()
    for name, data, chunk, pcm in cases:
        out, res, infos = _gpu_decode([data], chunk, gpu_batch_cls)
        r, info = res[0], infos[0]
        assert r.exception == 0 and r.crc_errors == 0 and r.frames == pcm.shape[0], name
        np.testing.assert_array_equal(out[info.out_offset: info.out_offset + pcm.size], pcm.reshape(-1), err_msg=name)


def test_corrupted_streams(gpu_batch_cls):
    from synth import wvsynth as S
    x = S.audio_like(20000, 2, 16, seed=11)
    m = S.audio_like(20000, 1, 16, seed=12)
    base = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4000))
    basem = S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=3001))
    basex = V.int32_file(x, sent_bits=6, ones=2, wvx=2, max_width=21)
    for lane in ("2wave", "generic", "pipe", "lane"):
        for k in range(10):
            _check_one(V.corrupt(base, k), 4096, gpu_batch_cls, f"stereo#{k}", lane)
            _check_one(V.corrupt(basem, 100 + k), 1000, gpu_batch_cls, f"mono#{k}", lane)
    for k in range(10):
        _check_one(V.corrupt(basex, 200 + k), 4096, gpu_batch_cls, f"int32_wvx#{k}")
    # hybrid streams (the parser's hybrid fast path and its bails to get_word)
    h = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, hybrid_bitrate=True, bitrate_x256=768,
                                    block_samples=5000))
    hb = S.encode_pcm(x, S.EncParams(terms=S.TERMS_HIGH, hybrid=True, hybrid_bitrate=True, hybrid_balance=True,
                                     bitrate_x256=1024, block_samples=5000))
    hm = S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, hybrid=True, hybrid_bitrate=True,
                                     bitrate_x256=640, block_samples=3001))
    for k in range(8):
        _check_one(V.corrupt(h, 300 + k, start=150), 4096, gpu_batch_cls, f"hybrid#{k}")
        _check_one(V.corrupt(hb, 400 + k, start=150), 4096, gpu_batch_cls, f"hybrid_balance#{k}")
        _check_one(V.corrupt(hm, 500 + k, start=150), 1000, gpu_batch_cls, f"hybrid_mono#{k}")


def test_batch_of_many_files_matches_per_file(gpu_batch_cls):
    """All cases in ONE batch: offsets/descriptors must not interfere."""
    cases = V.pcm_cases() + V.dsd_cases()
    files = [c[1] for c in cases]
    out, res, infos = _gpu_decode(files, 4096, gpu_batch_cls)
    for (name, data, _), r, info in zip(cases, res, infos):
        ref = O.decode_file(data, chunk=4096)
        if ref.status == -3:  # the reference throws in this file
            assert r.exception == 1, name
            continue
        assert r.frames == ref.frames and r.crc_errors == ref.crc_errors, name
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        np.testing.assert_array_equal(got, ref.samples, err_msg=name)


def test_parallel_framing_matches_sequential(gpu_batch_cls):
    """wvg_batch_add_files (host threads, merged offsets) decodes exactly like the
    same files added one by one: C5-style mixed files, DSD, seeks' neighbours,
    exceptions, unopenable inputs, and the .wav images of a formatted batch."""
    from synth import corpora
    files = [c[1] for c in V.pcm_cases() + V.dsd_cases()] + corpora.c5(40) + [b"", b"RIFF" + b"\0" * 60]
    a = gpu_batch_cls(4096)
    ia = [a.add_file(f) for f in files]
    a.decode()
    a.format()
    oa = a.download()
    b = gpu_batch_cls(4096)
    ib = b.add_files(files, threads=8)
    b.decode()
    b.format()
    ob = b.download()
    assert ia == ib
    np.testing.assert_array_equal(oa, ob)
    for k, i in enumerate(ia):
        if i < 0:
            continue
        ra, rb = a.result(i), b.result(i)
        assert (ra.frames, ra.crc_errors, ra.exception, ra.status_or) == (rb.frames, rb.crc_errors, rb.exception,
                                                                          rb.status_or), k
        assert a.wav(i) == b.wav(i), k
    np.testing.assert_array_equal(a.download_pcm(), b.download_pcm())
    a.close()
    b.close()


def test_c2_full_size_roundtrip(gpu_batch_cls):
    """BASELINE config 2 at full size (1,024 blocks x 22,050 frames): lossless
    round trip to the generator's PCM, zero CRC errors (size-independent
    property; the oracle is checked on a sample of blocks)."""
    from synth import corpora
    pcm, data = corpora.c2(return_pcm=True)
    out, res, infos = _gpu_decode([data], 4096, gpu_batch_cls)
    assert res[0].crc_errors == 0
    assert res[0].frames == pcm.shape[0] == 1024 * 22050
    np.testing.assert_array_equal(out, pcm.reshape(-1))


def test_c3_full_block_high24(gpu_batch_cls):
    """C3's block shape at full size (44,100-frame 24-bit stereo blocks, 16-term 'high'
    chain) against the oracle, plus the lossless round trip."""
    from synth import wvsynth as S
    x = S.audio_like(2 * 44100 + 777, 2, 24, seed=0xC3)
    data = S.encode_pcm(x, S.EncParams(terms=S.TERMS_HIGH, bytes_per_sample=3, block_samples=44100))
    for route in ("2wave", "pipe"):
        _check_one(data, 4096, gpu_batch_cls, "c3_full_block", route)
        out, res, infos = _gpu_decode([data], 4096, gpu_batch_cls, route)
        np.testing.assert_array_equal(out[: x.size], x.reshape(-1))


def test_c4_blocks_match_oracle(gpu_batch_cls):
    """C4-shaped blocks (float32, hybrid + bitrate, default terms, 22,050 frames):
    the parser's hybrid narrow run against the oracle."""
    from synth import corpora
    data = corpora.c4(nblocks=24)
    _check_one(data, 4096, gpu_batch_cls, "c4x24")


def test_golden_fixtures(gpu_batch_cls):
    """The committed fixtures (tests/golden) decode to the manifest's SHA-256, all in one batch."""
    import hashlib

    from tests import golden
    fx = list(golden.load())
    out, res, infos = _gpu_decode([d for _, d, _ in fx], 4096, gpu_batch_cls)
    for (name, data, m), r, info in zip(fx, res, infos):
        assert r.frames == m["frames"] and r.crc_errors == m["crc_errors"], name
        got = out[info.out_offset: info.out_offset + m["frames"] * m["nch"]]
        assert hashlib.sha256(got.astype("<i4").tobytes()).hexdigest() == m["sha256_int32le"], name


def _oracle_format(ints, bps, dsd):
    import ctypes
    L = O.lib()
    L.wvo_format_samples.restype = ctypes.c_int
    L.wvo_format_samples.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_int]
    src = np.ascontiguousarray(ints, dtype=np.int32)
    buf = np.zeros(max(src.size * bps, 1), dtype=np.uint8)
    assert L.wvo_format_samples(src.ctypes.data, src.size, bps, buf.ctypes.data, buf.size, 0, dsd) == 1
    return buf[: src.size * bps]


@pytest.mark.parametrize("dsd", [0, 1])
def test_format_epilogue_matches_oracle(gpu_batch_cls, dsd):
    """The device WavpackFormatSamples epilogue (WavPackUtils.cs:288-341) over a whole
    batch equals the oracle's restatement applied to the same int32 output, for every
    mode (1/2/3/4 bytes per sample) and both values of the dsd argument."""
    cases = V.pcm_cases() + V.dsd_cases()
    b = gpu_batch_cls(4096)
    idx = [b.add_file(d) for _, d, _ in cases]
    b.decode()
    b.format(dsd=bool(dsd))
    pcm = b.download_pcm()
    np.testing.assert_array_equal(b.download_pcm(pinned=True), pcm)  # the page-locked path, same bytes
    b.download_pcm_async()  # queued behind the format; the bytes are there after sync
    b.sync()
    np.testing.assert_array_equal(b.host_pcm(), pcm)
    out = b.download()
    offs = [b.pcm_offset(i) for i in idx]
    infos = list(b.infos)
    b.close()
    seen = set()
    for (name, _, _), off, info in zip(cases, offs, infos):
        n = info.out_frames * info.reduced_channels
        bps = info.bytes_per_sample
        seen.add(bps)
        ints = out[info.out_offset: info.out_offset + n]
        np.testing.assert_array_equal(pcm[off: off + n * bps], _oracle_format(ints, bps, dsd), err_msg=name)
    assert seen == {1, 2, 3, 4}


def test_wvdemo_wav_matches_oracle():
    """WvDemo.Main (WvDemo.cs:15-168) through the GPU path: the same .wav bytes and exit
    code as the oracle's WvDemo, for every mode, config 1 (20 s, stored RIFF header,
    long enough to pass the loop_samples quirk), short files (the DivideByZero exit
    after the first call) and corrupted streams (CRC errors, C# exceptions)."""
    from synth import corpora
    from synth import wvsynth as S
    from wavpackdecoder_amd.api import wv_demo
    files = [(n, d) for n, d, c in V.pcm_cases() + V.dsd_cases() if c == 4096]
    files.append(("config1", corpora.c1()[1]))
    x = S.audio_like(450000, 2, 16, seed=21)
    files.append(("synth_wav_hdr", S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=44100))))
    base = S.encode_pcm(S.audio_like(20000, 2, 16, seed=11), S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4000))
    files += [(f"corrupt#{k}", V.corrupt(base, k)) for k in range(10)]
    files += [("empty", b""), ("not_wavpack", b"RIFF" + b"\0" * 60)]
    for name, data in files:
        rc_ref, wav_ref = O.demo(data)
        rc, wav = wv_demo(data)
        assert rc == rc_ref, name
        assert len(wav) == len(wav_ref), name
        assert wav == wav_ref, name


def test_edge_inputs(gpu_batch_cls):
    """Empty and non-WavPack inputs open with an error (WavPackUtils.cs:36-120); a batch that
    mixes them with a real file still decodes the real one; ragged block sizes and a 1-frame
    tail block decode exactly."""
    from synth import wvsynth as S
    x = S.audio_like(4097, 2, 16, seed=31)
    real = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=4096))  # 4096 + 1-frame tail
    ragged = S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=1237))
    files = [b"", b"RIFF" + b"\0" * 60, real, ragged]
    out, res, infos = _gpu_decode(files, 4096, gpu_batch_cls)
    assert not infos[0].open_ok and not infos[1].open_ok
    for k in (2, 3):
        info = infos[k]
        assert res[k].frames == 4097 and res[k].crc_errors == 0
        np.testing.assert_array_equal(out[info.out_offset: info.out_offset + 4097 * 2], x.reshape(-1))


def test_fuzzed_metadata_device_parse(gpu_batch_cls):
    """Device-side metadata parse (wv_meta_parse) on files whose
    metadata sub-blocks were fuzzed, all in one batch: the GPU output equals the
    oracle's (frames, crc errors, exception, samples) and the host-core build's
    (tests/emu: the same framing with the deferred values applied on the host).  Includes
    hybrid streams whose negative error limit makes the C# bisection loop forever
    (reported as an exception on both sides)."""
    from tests.emu import emu as E
    from tests.test_meta_defer import _bases, meta_fuzz
    files = [meta_fuzz(d, 9000 + 100 * b + s) for b, d in enumerate(_bases()) for s in range(12)]
    files.append(meta_fuzz(_bases()[3], 5312))  # the never-ending bisection
    out, res, infos = _gpu_decode(files, 4096, gpu_batch_cls)
    for k, (f, r, info) in enumerate(zip(files, res, infos)):
        assert r is None or not (r.status_or & WVG_ST_TIMEOUT), k
        n, eout, crc, st = E.decode(f)
        ref = O.decode_file(f)  # the oracle pins the GPU directly, not only through the host build
        if n == -2:
            assert not info.open_ok and ref.status == -2, k
            continue
        assert r is not None, k
        if n == -3:
            assert r.exception == 1 and ref.status == -3, k
            continue
        assert r.exception == 0 and r.frames == n == ref.frames and r.crc_errors == crc == ref.crc_errors, k
        got = out[info.out_offset: info.out_offset + len(eout)]
        np.testing.assert_array_equal(got, eout, err_msg=str(k))
        assert not (r.status_or & 0x20), k  # every layout of the corpus is decoded (no UNSUPPORTED)
        if not (r.status_or & 0x80):  # NONDET: the reference reads the caller's stale buffer there
            np.testing.assert_array_equal(got, ref.samples, err_msg=str(k))


def test_poison_then_decode_stores_every_status(gpu_batch_cls):
    """wvg_batch_poison marks every decodable block WVG_ST_UNWRITTEN; the next decode
    must store every block's status -- including the members of a sticky-state chain
    after a block that raises the reference's exception, which are never decoded
    (decode_chain gives them back the framing's status) -- and produce the same
    statuses, file results and output as a decode of the unpoisoned batch (the output
    over each file's defined frames: up to the call that throws, and nothing of a file
    whose output reads the caller's stale buffer, WVG_ST_NONDET)."""
    from wavpackdecoder_amd._lib import WVG_ST_NONDET, WVG_ST_UNWRITTEN
    sticky = [c[1] for c in V.sticky_cases()]
    files = sticky + [V.corrupt(f, 700 + k, nflips=6) for k, f in enumerate(sticky)]
    b = gpu_batch_cls(4096)
    idx = [b.add_file(f) for f in files]
    b.decode()
    out0, st0 = b.download().copy(), b.block_status().copy()

    def results():
        rs = []
        for i in idx:
            if i < 0:
                continue
            r = b.result(i)
            rs.append((r.frames, r.crc_errors, r.exception, r.exception_frame, r.status_or))
        return rs
    res0 = results()
    b.poison(0x7F)
    b.decode()
    out1, st1 = b.download(), b.block_status()
    res1 = results()
    infos = [b.infos[i] for i in idx if i >= 0]
    b.close()
    assert not np.any(st1 & WVG_ST_UNWRITTEN)
    np.testing.assert_array_equal(st1, st0)
    assert res1 == res0
    assert all(not (r[4] & WVG_ST_UNWRITTEN) for r in res1)
    assert sum(r[2] for r in res0) >= 1, "no file raised the reference's exception: the chain case is not exercised"
    compared = 0
    for r, info in zip(res1, infos):
        if r[4] & WVG_ST_NONDET:
            continue
        n = (r[3] if r[2] else r[0]) * info.reduced_channels
        a, z = info.out_offset, info.out_offset + n
        np.testing.assert_array_equal(out1[a:z], out0[a:z])
        compared += 1
    assert compared >= len(res1) // 2
