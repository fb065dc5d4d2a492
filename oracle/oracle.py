"""ctypes binding of the C oracle (oracle/wv_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (wavpackdecoder_amd/) never imports it.

The oracle restates the reference C# decoder line by line; each C function
cites the reference file:line it follows (e.g. get_words -> WordsUtils.cs:272).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.wvo_decode_file.restype = ctypes.c_int64
        L.wvo_decode_file.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_int)]
        L.wvo_demo.restype = ctypes.c_int
        L.wvo_demo.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_size_t)]
        L.wvo_free.argtypes = [ctypes.c_void_p]
        L.wvo_open.restype = ctypes.c_void_p
        L.wvo_open.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.wvo_close.argtypes = [ctypes.c_void_p]
        L.wvo_unpack_samples.restype = ctypes.c_int64
        L.wvo_unpack_samples.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        for name in ("wvo_get_num_samples",):
            getattr(L, name).restype = ctypes.c_int64
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_int]
        for name in ("wvo_get_sample_index", "wvo_get_num_errors", "wvo_get_sample_rate"):
            getattr(L, name).restype = ctypes.c_int64
            getattr(L, name).argtypes = [ctypes.c_void_p]
        for name in ("wvo_lossy", "wvo_get_num_channels", "wvo_get_bits_per_sample", "wvo_get_bytes_per_sample",
                     "wvo_get_reduced_channels", "wvo_get_mode", "wvo_get_version", "wvo_get_is_float",
                     "wvo_get_is_five", "wvo_get_file_format", "wvo_exception"):
            getattr(L, name).restype = ctypes.c_int
            getattr(L, name).argtypes = [ctypes.c_void_p]
        L.wvo_get_error_message.restype = ctypes.c_char_p
        L.wvo_get_error_message.argtypes = [ctypes.c_void_p]
        L.wvo_exp2s.restype = ctypes.c_int
        L.wvo_exp2s.argtypes = [ctypes.c_int]
        L.wvo_mylog2.restype = ctypes.c_int
        L.wvo_mylog2.argtypes = [ctypes.c_int64]
        L.wvo_log2s.restype = ctypes.c_int
        L.wvo_log2s.argtypes = [ctypes.c_int]
        L.wvo_count_bits.restype = ctypes.c_int
        L.wvo_count_bits.argtypes = [ctypes.c_int64]
        L.wvo_restore_weight.restype = ctypes.c_int
        L.wvo_restore_weight.argtypes = [ctypes.c_int8]
        L.wvo_read_code_bytes.restype = ctypes.c_int64
        L.wvo_read_code_bytes.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


class DecodeResult:
    def __init__(self, samples, frames, nch, crc_errors, lossy, status):
        self.samples = samples      # int32, frames x nch interleaved (flat)
        self.frames = frames
        self.nch = nch
        self.crc_errors = crc_errors
        self.lossy = lossy
        self.status = status        # 0 ok, -2 open error, -3 C# exception

    def __repr__(self):
        return (f"DecodeResult(frames={self.frames}, nch={self.nch}, crc_errors={self.crc_errors}, "
                f"lossy={self.lossy}, status={self.status})")


def decode_file(data: bytes, chunk: int = 4096, max_frames: int | None = None) -> DecodeResult:
    """WvDemo's loop (WvDemo.cs:110-135): WavpackUnpackSamples(chunk) until 0."""
    L = lib()
    if max_frames is None:
        max_frames = max(len(data) * 8, 1 << 16)  # generous bound; grows below if needed
    while True:
        cap = max_frames * 2
        out = np.zeros(cap, dtype=np.int32)
        crc = ctypes.c_int64(0)
        lossy = ctypes.c_int(0)
        nch = ctypes.c_int(0)
        n = L.wvo_decode_file(data, len(data), out.ctypes.data, cap, chunk, ctypes.byref(crc),
                              ctypes.byref(lossy), ctypes.byref(nch))
        if n >= 0 and n * max(nch.value, 1) > cap:
            max_frames = int(n) + 16
            continue
        if n < 0:
            return DecodeResult(np.zeros(0, np.int32), 0, nch.value, crc.value, lossy.value, int(n))
        return DecodeResult(out[: n * nch.value].copy(), int(n), nch.value, crc.value, lossy.value, 0)


def decode_file_from(data: bytes, start: int, chunk: int = 4096):
    """WavpackOpenFileInput + SetSample(start) (WavPackUtils.cs:509-594) + the
    WvDemo loop from there -> (DecodeResult, seek_rc): seek_rc 1 positioned,
    0 SetSample returned false, -1 an exception escaped it."""
    L = lib()
    f = L.wvo_decode_file_from
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    max_frames = max(len(data) * 8, 1 << 16)
    while True:
        cap = max_frames * 2
        out = np.zeros(cap, dtype=np.int32)
        crc, nch, src = ctypes.c_int64(0), ctypes.c_int(0), ctypes.c_int(0)
        n = f(data, len(data), int(start), out.ctypes.data, cap, chunk, ctypes.byref(crc), ctypes.byref(nch),
              ctypes.byref(src))
        if n >= 0 and n * max(nch.value, 1) > cap:
            max_frames = int(n) + 16
            continue
        if n < 0:
            return DecodeResult(np.zeros(0, np.int32), 0, nch.value, crc.value, 0, int(n)), src.value
        return DecodeResult(out[: n * nch.value].copy(), int(n), nch.value, crc.value, 0, 0), src.value


def demo(data: bytes):
    """WvDemo.Main equivalent -> (exit_code, wav_bytes)."""
    L = lib()
    p = ctypes.c_void_p()
    n = ctypes.c_size_t()
    rc = L.wvo_demo(data, len(data), ctypes.byref(p), ctypes.byref(n))
    wav = ctypes.string_at(p.value, n.value) if p.value else b""
    if p.value:
        L.wvo_free(p)
    return rc, wav


def read_code(buf: bytes, maxcode: int):
    used = ctypes.c_int(0)
    code = lib().wvo_read_code_bytes(buf, len(buf), maxcode, ctypes.byref(used))
    return int(code), int(used.value)


def decode_many(files, chunk: int = 4096, threads: int | None = None) -> list:
    """decode_file over many files on host threads (ctypes drops the GIL; one oracle
    context per call) -- for parity runs at the BASELINE configs' own sizes."""
    from concurrent.futures import ThreadPoolExecutor
    if threads is None:
        threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8") or 8), os.cpu_count() or 1))

    def one(f):
        # frames bound from the headers (block_samples per block), not the generous default
        i, fr = 0, 0
        while i + 32 <= len(f) and f[i:i + 4] == b"wvpk":
            fr += int.from_bytes(f[i + 20:i + 24], "little")
            i += 8 + int.from_bytes(f[i + 4:i + 8], "little")
        return decode_file(f, chunk=chunk, max_frames=max(fr, 1 << 16))
    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(one, files))
