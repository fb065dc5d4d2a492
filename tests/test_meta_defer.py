"""Device-side metadata parse: deferred values == host values.

The framing defers the values of read_decorr_weights / read_decorr_samples /
read_entropy_vars / read_hybrid_profile (UnpackUtils.cs:196-360,
WordsUtils.cs:75-187) to meta_apply (csrc/wv_meta.h), which the device parse
kernel runs per block.  Here the host build of the same code (tests/emu) frames
every file twice -- values on the host, values deferred and applied by
meta_apply -- and the descriptor bytes must be identical, for well-formed files
(where every block is deferred) and for files whose metadata sub-blocks were
fuzzed (odd lengths, stale-buffer reads, missing or repeated sub-blocks: the
framing must fall back to the host readers there).  The GPU side of the same
check (descriptors after the device kernel) is in test_gpu_parity.py.
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from synth import wvsynth as S
from tests import vectors as V
from tests.emu import emu as E

from tests.emu.emu import DESC_BYTES  # noqa: E402  (sizeof(BlockDesc), from the emu build)


def frame(data: bytes, defer: bool, seek: int = -1, chunk: int = 4096):
    L = E.lib()
    f = L.emu_frame_descs
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    cap = DESC_BYTES * (len(data) // 64 + 64)
    buf = np.zeros(cap, np.uint8)
    nj = ctypes.c_int64(0)
    n = f(data, len(data), seek, chunk, int(defer), buf.ctypes.data, cap, ctypes.byref(nj))
    assert n >= 0
    return buf[: n * DESC_BYTES].tobytes(), int(n), nj.value


def same(data: bytes, seek: int = -1, chunk: int = 4096):
    full, n, _ = frame(data, False, seek, chunk)
    dfr, n2, jobs = frame(data, True, seek, chunk)
    assert n == n2
    for k in range(n):
        a, b = full[k * DESC_BYTES:(k + 1) * DESC_BYTES], dfr[k * DESC_BYTES:(k + 1) * DESC_BYTES]
        assert a == b, f"descriptor {k} differs at byte {next(i for i in range(DESC_BYTES) if a[i] != b[i])}"
    return n, jobs


def block_offsets(data: bytes):
    offs, p = [], data.find(b"wvpk")
    while 0 <= p < len(data) - 32:
        offs.append(p)
        ck = int.from_bytes(data[p + 4:p + 8], "little")
        p += 8 + ck
        if not data.startswith(b"wvpk", p):
            break
    return offs


def meta_fuzz(data: bytes, seed: int, nflips: int = 2) -> bytes:
    """Flip bits / overwrite bytes inside the metadata sub-blocks ahead of the bitstream."""
    rng = np.random.default_rng(seed)
    b = bytearray(data)
    offs = block_offsets(data)
    for _ in range(nflips):
        o = offs[int(rng.integers(0, len(offs)))]
        # the sub-blocks before ID_WV_BITSTREAM sit in the first ~120 bytes after the header
        pos = o + 32 + int(rng.integers(0, 120))
        if pos >= len(b):
            continue
        if rng.integers(0, 3) == 0:
            b[pos] = int(rng.integers(0, 256))
        else:
            b[pos] ^= 1 << int(rng.integers(0, 8))
    return bytes(b)


PCM = V.pcm_cases()
DSD = V.dsd_cases()


@pytest.mark.parametrize("name,data,chunk", PCM + DSD, ids=[c[0] for c in PCM + DSD])
def test_deferred_equals_host(name, data, chunk):
    n, jobs = same(data, chunk=chunk)
    if "dsd" not in name:
        assert jobs == n  # every PCM block's values came from meta_apply


def _bases():
    x = S.audio_like(12000, 2, 16, seed=31)
    m = S.audio_like(9000, 1, 24, seed=32)
    return [
        S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=3000)),
        S.encode_pcm(x, S.EncParams(terms=S.TERMS_HIGH, block_samples=4000)),
        S.encode_pcm(m, S.EncParams(nch=1, bytes_per_sample=3, terms=S.TERMS_MONO_HIGH, block_samples=3000)),
        S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, hybrid_bitrate=True, bitrate_x256=640,
                                    block_samples=3000)),
        S.encode_pcm(m, S.EncParams(nch=1, bytes_per_sample=3, terms=S.TERMS_MONO_HIGH, hybrid=True,
                                    bitrate_x256=900, block_samples=3000)),
        S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, bitrate_x256=700, version=0x402,
                                    block_samples=3000)),
    ]


@pytest.mark.parametrize("base", range(6))
def test_deferred_equals_host_fuzzed_metadata(base):
    data = _bases()[base]
    for seed in range(60):
        f = meta_fuzz(data, 1000 * base + seed)
        same(f)
        same(f, chunk=1000)


def test_fuzzed_metadata_decode_matches_oracle():
    """The deferred path end to end (emu decode frames with deferral) on fuzzed metadata."""
    for base, data in enumerate(_bases()):
        for seed in range(25):
            f = meta_fuzz(data, 5000 + 100 * base + seed)
            r = O.decode_file(f)
            n, out, crc, st = E.decode(f)
            if r.status != 0:
                assert n == r.status, (base, seed)
                continue
            assert n == r.frames and crc == r.crc_errors, (base, seed)
            if not (st & 0xA0):  # ST_NONDET / ST_UNSUPPORTED blocks are the host's
                assert np.array_equal(out, r.samples), (base, seed)


def test_deferred_equals_host_after_seek():
    x = S.audio_like(30000, 2, 16, seed=33)
    data = S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=5000))
    for st in (0, 1, 4999, 5000, 12345, 29999, 30000):
        same(data, seek=st)
    for seed in range(10):
        f = meta_fuzz(data, 7000 + seed)
        for st in (0, 7000, 20000):
            same(f, seek=st)
