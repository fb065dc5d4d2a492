"""Synthetic WavPack corpora for tests and bench (input generation only).

Wraps synth/wv_encoder.cpp (a WavPack-4 encoder derived as the inverse of the
reference decode path) and the signal models of SURVEY.md §8d:
  C1  one 44.1 kHz 16-bit stereo file, default terms {18,18,2,3,-2}
  C2  1,024 blocks x 22,050 frames, 16-bit stereo, fast terms {17,17}
  C3  4,096 blocks x 44,100 frames, 24-bit stereo, high 16-term chain
  C4  hybrid lossy float32 (FLOAT_DATA|HYBRID|HYBRID_BITRATE)
  C5  mixed corpus (mono/stereo, 16/24-bit, DSD modes 0/1/3)
Seeds are fixed and recorded by the callers.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libwvenc.so")
_lib = None

TERMS_FAST = [17, 17]
TERMS_DEFAULT = [18, 18, 2, 3, -2]
TERMS_HIGH = [18, 18, 2, 3, -2, 18, 2, 4, 7, 5, 3, 6, 8, -1, 18, 2]
TERMS_MONO_HIGH = [18, 18, 2, 3, 18, 2, 4, 7, 5, 3, 6, 8, 18, 2, 17, 1]
TERMS_HIGH10 = [18, 18, 18, -2, 2, 3, 5, -1, 17, 4]  # [ext] WavPack 4 'high' (10 terms)
TERMS_X3 = [18, -3, 1, 17, 2, -1, 3, -3, 18, 1]      # 'extra'-style list: cross-channel -3 and term 1


class _Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "nch", "bytes_per_sample", "shift", "joint_stereo", "false_stereo", "num_terms")] + [
        ("terms", ctypes.c_int32 * 16), ("deltas", ctypes.c_int32 * 16)] + [
        (n, ctypes.c_int32) for n in (
            "block_samples", "sample_rate", "version", "hybrid", "hybrid_bitrate", "hybrid_balance",
            "bitrate_x256", "float_data", "float_flags", "float_shift", "float_max_exp", "float_norm_exp",
            "int32_zeros", "write_riff", "config_flags", "write_history", "reset_state", "block_index_start",
            "total_unknown", "extras", "mag_override", "int32_sent_bits", "int32_ones", "int32_dups", "wvx",
            "wvx_max_width", "wvx_short")] + [("total_override", ctypes.c_int64), ("sticky_passes", ctypes.c_int32), ("wvc", ctypes.c_int32),
                                                          ("float_exact", ctypes.c_int32)]


class _DsdParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "nch", "false_stereo", "mode", "block_samples", "rate_multiplier_log2", "sample_rate",
        "history_bits", "rle_tables", "rate_i")]


@dataclass
class EncParams:
    nch: int = 2
    bytes_per_sample: int = 2
    shift: int = 0
    joint_stereo: bool = True
    false_stereo: bool = False
    terms: list = field(default_factory=lambda: list(TERMS_FAST))
    deltas: list | None = None
    block_samples: int = 22050
    sample_rate: int = 44100
    version: int = 0x407
    hybrid: bool = False
    hybrid_bitrate: bool = False
    hybrid_balance: bool = False
    bitrate_x256: int = 0
    float_data: bool = False
    float_flags: int = 0
    float_shift: int = 0
    float_max_exp: int = 126
    float_norm_exp: int = 127
    int32_zeros: int = 0
    write_riff: bool = False
    config_flags: int = 0
    write_history: bool = True
    reset_state: bool = False
    block_index_start: int = 0
    total_unknown: bool = False
    extras: int = 0
    mag_override: int = -1
    int32_sent_bits: int = 0
    int32_ones: int = 0
    int32_dups: int = 0
    wvx: int = 0            # 0 none, 1 ID_WVX_BITSTREAM, 2 ID_WVX_NEW_BITSTREAM (UnpackUtils.cs:115-147)
    wvx_max_width: int = 0  # NEW variant's int32_max_width
    wvx_short: int = 0      # bytes dropped from every wvx payload (the reference then over-reads and throws)
    total_override: int = 0  # > 0: header total_samples (parts encoded in parallel, then concatenated)
    sticky_passes: bool = False  # blocks after the first continue the decoder's passes (no pass metadata)
    wvc: bool = False            # hybrid: also write the .wvc correction file (encode_pcm_wvc)
    float_exact: bool = False    # float_data: samples are float32 bit patterns (encode_float_exact)

    def to_c(self) -> _Params:
        p = _Params()
        p.nch, p.bytes_per_sample, p.shift = self.nch, self.bytes_per_sample, self.shift
        p.joint_stereo, p.false_stereo = int(self.joint_stereo), int(self.false_stereo)
        p.num_terms = len(self.terms)
        deltas = self.deltas if self.deltas is not None else [2] * len(self.terms)
        for i, t in enumerate(self.terms):
            p.terms[i] = t
            p.deltas[i] = deltas[i]
        for n in ("block_samples", "sample_rate", "version", "bitrate_x256", "float_flags", "float_shift",
                  "float_max_exp", "float_norm_exp", "int32_zeros", "config_flags", "block_index_start",
                  "extras", "mag_override", "int32_sent_bits", "int32_ones", "int32_dups", "wvx", "wvx_max_width",
                  "wvx_short", "total_override"):
            setattr(p, n, int(getattr(self, n)))
        for n in ("hybrid", "hybrid_bitrate", "hybrid_balance", "float_data", "write_riff", "write_history",
                  "reset_state", "total_unknown", "sticky_passes", "wvc", "float_exact"):
            setattr(p, n, int(bool(getattr(self, n))))
        return p


def encode_pcm_parallel(samples: np.ndarray, params: EncParams, workers: int | None = None) -> bytes:
    """encode_pcm over whole-block parts in worker processes, concatenated: the
    same stream as one encode_pcm call whenever the blocks do not carry state
    (reset_state) -- and in any case a valid stream whose parts start from a
    fresh encoder state (the decoder re-reads every block's state)."""
    import dataclasses
    from concurrent.futures import ProcessPoolExecutor
    x = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1, params.nch)
    frames = x.shape[0]
    B = params.block_samples
    nblocks = (frames + B - 1) // B
    if workers is None:
        workers = min(16, int(os.environ.get("OMP_NUM_THREADS", "8") or 8), os.cpu_count() or 1)
    if workers <= 1 or nblocks < 2 * workers:
        return encode_pcm(x, params)
    per = (nblocks + workers - 1) // workers
    jobs = []
    for k in range(0, nblocks, per):
        p = dataclasses.replace(params, block_index_start=params.block_index_start + k * B, total_override=frames,
                                write_riff=params.write_riff and k == 0)
        jobs.append((x[k * B:(k + per) * B], p))
    with ProcessPoolExecutor(max_workers=workers) as ex:
        parts = list(ex.map(_encode_job, jobs))
    return b"".join(parts)


def _encode_job(job):
    x, p = job
    return encode_pcm(x, p)


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.wvenc_encode_pcm.restype = ctypes.c_int64
        L.wvenc_encode_pcm.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_Params), ctypes.c_void_p,
                                       ctypes.c_int64]
        L.wvenc_encode_pcm_wvc.restype = ctypes.c_int64
        L.wvenc_encode_pcm_wvc.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_Params), ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.POINTER(ctypes.c_int64)]
        L.wvenc_encode_dsd.restype = ctypes.c_int64
        L.wvenc_encode_dsd.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_DsdParams),
                                       ctypes.c_void_p, ctypes.c_int64]
        L.wvenc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def encode_pcm(samples: np.ndarray, params: EncParams) -> bytes:
    """samples: int32 array shaped (frames, nch) (or flat interleaved)."""
    x = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1)
    frames = x.size // params.nch
    p = params.to_c()
    L = lib()
    n = L.wvenc_encode_pcm(x.ctypes.data, frames, ctypes.byref(p), None, 0)
    if n < 0:
        raise RuntimeError("wvenc: " + L.wvenc_last_error().decode())
    out = np.empty(n, dtype=np.uint8)
    m = L.wvenc_encode_pcm(x.ctypes.data, frames, ctypes.byref(p), out.ctypes.data, n)
    if m != n:
        raise RuntimeError("wvenc: size mismatch " + L.wvenc_last_error().decode())
    return out.tobytes()


def encode_pcm_wvc(samples: np.ndarray, params: EncParams):
    """Hybrid PCM -> (.wv bytes, .wvc bytes): the .wv decodes lossy (the reference's
    output); with the .wvc correction the residuals are exact and the decode is lossless."""
    x = np.ascontiguousarray(samples, dtype=np.int32).reshape(-1)
    frames = x.size // params.nch
    params.hybrid = True
    params.wvc = True
    p = params.to_c()
    L = lib()
    nc = ctypes.c_int64(0)
    n = L.wvenc_encode_pcm_wvc(x.ctypes.data, frames, ctypes.byref(p), None, 0, None, 0, ctypes.byref(nc))
    if n < 0:
        raise RuntimeError("wvenc: " + L.wvenc_last_error().decode())
    out = np.empty(n, dtype=np.uint8)
    cout = np.empty(max(nc.value, 1), dtype=np.uint8)
    m = L.wvenc_encode_pcm_wvc(x.ctypes.data, frames, ctypes.byref(p), out.ctypes.data, n, cout.ctypes.data,
                               cout.size, ctypes.byref(nc))
    if m != n:
        raise RuntimeError("wvenc: " + L.wvenc_last_error().decode())
    return out.tobytes(), cout[: nc.value].tobytes()


def encode_float_exact(x: np.ndarray, params: EncParams, wvc: bool = False):
    """float32 samples (frames, nch) -> a FLOAT_DATA .wv whose integers are the
    mantissas shifted to each block's largest exponent, with a classic wvx stream
    holding what the shift dropped, the floats it took to 0, -0.0 and inf/nan
    (beyond the reference, which scales the integers to 24-bit PCM and never
    reads the stream).  wvc: hybrid .wv + .wvc, the wvx stream in the .wvc.
    Returns the .wv bytes, or (.wv, .wvc) with wvc."""
    bits = np.ascontiguousarray(x, dtype=np.float32).view(np.int32)
    params.float_data = True
    params.float_exact = True
    params.bytes_per_sample = 4
    return encode_pcm_wvc(bits, params) if wvc else encode_pcm(bits, params)


@dataclass
class DsdParams:
    nch: int = 2
    false_stereo: bool = False
    mode: int = 3
    block_samples: int = 44100
    rate_multiplier_log2: int = 0
    sample_rate: int = 44100
    history_bits: int = 5
    rle_tables: bool = False
    rate_i: int = 3

    def to_c(self) -> _DsdParams:
        p = _DsdParams()
        for n in ("nch", "mode", "block_samples", "rate_multiplier_log2", "sample_rate", "history_bits", "rate_i"):
            setattr(p, n, int(getattr(self, n)))
        p.false_stereo = int(self.false_stereo)
        p.rle_tables = int(self.rle_tables)
        return p


def encode_dsd(samples: np.ndarray, params: DsdParams) -> bytes:
    x = np.ascontiguousarray(samples, dtype=np.uint8).reshape(-1)
    frames = x.size // params.nch
    p = params.to_c()
    L = lib()
    n = L.wvenc_encode_dsd(x.ctypes.data, frames, ctypes.byref(p), None, 0)
    if n < 0:
        raise RuntimeError("wvenc: " + L.wvenc_last_error().decode())
    out = np.empty(n, dtype=np.uint8)
    m = L.wvenc_encode_dsd(x.ctypes.data, frames, ctypes.byref(p), out.ctypes.data, n)
    assert m == n
    return out.tobytes()


# ---------------------------------------------------------------------------
# signal models
# ---------------------------------------------------------------------------
def _one_channel(rng: np.random.Generator, frames: int, rate: float, full_scale: float, sigma: float) -> np.ndarray:
    t = np.arange(frames, dtype=np.float64) / rate
    y = np.zeros(frames, dtype=np.float64)
    for _ in range(4):
        f = np.exp(rng.uniform(np.log(40.0), np.log(6000.0)))
        a_db = rng.uniform(-20.0, -3.0)
        ph = rng.uniform(0, 2 * np.pi)
        y += (10 ** (a_db / 20.0)) * 0.25 * np.sin(2 * np.pi * f * t + ph)
    return y * full_scale + rng.normal(0.0, sigma, frames)


def audio_like(frames: int, nch: int = 2, bits: int = 16, seed: int = 0, sigma: float | None = None,
               kind: str = "music") -> np.ndarray:
    """int32 (frames, nch): 4 sinusoids + Gaussian noise; R = 0.7 L + 0.3 indep.

    kind: "music" (the model above), "zeros" (digital silence, exercises the
    zero-run coder), "noise" (full-scale white noise, exercises escapes)."""
    rng = np.random.default_rng(seed)
    fs = float(2 ** (bits - 1) - 1)
    lo, hi = -(2 ** (bits - 1)), 2 ** (bits - 1) - 1
    if kind == "zeros":
        return np.zeros((frames, nch), dtype=np.int32)
    if kind == "noise":
        return rng.integers(lo, hi + 1, size=(frames, nch), dtype=np.int64).astype(np.int32)
    if sigma is None:
        sigma = 64.0 * (2 ** (bits - 16)) if bits >= 16 else 1.0
    left = _one_channel(rng, frames, 44100.0, fs, sigma)
    if nch == 1:
        chans = [left]
    else:
        other = _one_channel(rng, frames, 44100.0, fs, sigma)
        chans = [left, 0.7 * left + 0.3 * other]
    x = np.stack(chans, axis=1)
    return np.clip(np.rint(x), lo, hi).astype(np.int32)


def float_mantissas(x: np.ndarray, max_exp: int = 126) -> np.ndarray:
    """float32 in [-1, 1) -> the integer values a FLOAT_DATA block carries:
    round(f * 2^(150 - max_exp)); the decoder returns v << (max_exp - 127)
    clipped to 24 bits (FloatUtils.cs:32-56)."""
    v = np.rint(x.astype(np.float64) * float(2 ** (150 - max_exp)))
    return np.clip(v, -(2 ** 30), 2 ** 30).astype(np.int32)


def int32_layout(y: np.ndarray, sent_bits: int = 0, zeros: int = 0, ones: int = 0, dups: int = 0,
                 max_width: int = 0, seed: int = 0) -> np.ndarray:
    """int32 samples that an INT32_DATA block with these int32 info fields (and a wvx
    stream carrying `sent_bits` low bits, NEW variant when max_width > 0) represents
    exactly (UnpackUtils.cs:1271-1314): y is the main-stream word, random low bits are
    appended (truncated as max_width requires), then zeros/ones/dups are applied."""
    rng = np.random.default_rng(seed)
    v = y.astype(np.int64)
    if sent_bits:
        low = rng.integers(0, 1 << sent_bits, size=y.shape, dtype=np.int64)
        if max_width:
            pv = np.where(v < 0, ~v, v)
            width = np.array([int(a).bit_length() for a in pv.reshape(-1)], dtype=np.int64).reshape(y.shape) + sent_bits
            btr = np.where(width <= max_width, sent_bits, sent_bits - (width - max_width))
            btr = np.clip(btr, 0, sent_bits)
            low = (low >> (sent_bits - btr)) << (sent_bits - btr)
        v = (v << sent_bits) | low
    if zeros:
        v = v << zeros
    elif ones:
        v = ((v + 1) << ones) - 1
    elif dups:
        v = ((v + (v & 1)) << dups) - (v & 1)
    assert v.min() >= -(2 ** 31) and v.max() < 2 ** 31, "int32 range"
    return v.astype(np.int32)


def dsd_like(frames: int, nch: int = 2, seed: int = 0) -> np.ndarray:
    """1-bit sigma-delta modulation of a slow sine mix, packed MSB first."""
    rng = np.random.default_rng(seed)
    nbits = frames * 8
    t = np.arange(nbits, dtype=np.float64)
    out = []
    for c in range(nch):
        f1, f2 = rng.uniform(1e-5, 4e-4, size=2)
        s = 0.4 * np.sin(2 * np.pi * f1 * t) + 0.2 * np.sin(2 * np.pi * f2 * t + c)
        # first-order sigma-delta
        bits = np.empty(nbits, dtype=np.uint8)
        acc = 0.0
        for i in range(0, nbits, 65536):
            seg = s[i:i + 65536]
            b = np.empty(seg.size, dtype=np.uint8)
            for j, v in enumerate(seg):
                acc += v - (1.0 if acc > 0 else -1.0)
                b[j] = 1 if acc > 0 else 0
            bits[i:i + seg.size] = b
        out.append(np.packbits(bits.reshape(-1, 8), axis=1, bitorder="big").reshape(-1))
    return np.stack(out, axis=1).astype(np.uint8)


def dsd_random_like(frames: int, nch: int = 2, seed: int = 0, density: float = 0.5) -> np.ndarray:
    """Fast DSD-ish bytes: biased random bits (no Python loops)."""
    rng = np.random.default_rng(seed)
    bits = (rng.random((frames * 8, nch)) < density).astype(np.uint8)
    packed = np.packbits(bits.T.reshape(nch, frames, 8), axis=2, bitorder="big").reshape(nch, frames)
    return np.ascontiguousarray(packed.T)
