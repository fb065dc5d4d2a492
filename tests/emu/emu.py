"""TEST-ONLY ctypes binding of tests/emu/libwvemu.so (host build of the device decode core)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_L = None

INFO_FIELDS = ("open_ok", "total_samples", "sample_rate", "num_channels", "bits_per_sample", "bytes_per_sample",
               "reduced_channels", "mode", "version", "is_float", "out_frames", "out_nch", "num_blocks",
               "dsd_multiplier")


def lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(os.path.join(_HERE, "libwvemu.so"))
        L.emu_decode.restype = ctypes.c_int64
        L.emu_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_uint32)]
        L.emu_file_info.restype = ctypes.c_int
        L.emu_file_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        _L = L
    return _L


def decode(data: bytes, chunk: int = 4096):
    """-> (frames or -2/-3, samples int32 flat, crc_errors, status_or)"""
    cap = max(len(data) * 16, 1 << 16)
    while True:
        out = np.zeros(cap, dtype=np.int32)
        crc = ctypes.c_int64(0)
        nch = ctypes.c_int(0)
        st = ctypes.c_uint32(0)
        n = lib().emu_decode(data, len(data), chunk, out.ctypes.data, cap, ctypes.byref(crc), ctypes.byref(nch),
                             ctypes.byref(st))
        if n == -4:
            cap *= 4
            continue
        if n < 0:
            return int(n), np.zeros(0, np.int32), crc.value, st.value
        return int(n), out[: n * nch.value].copy(), crc.value, st.value


def decode_from(data: bytes, start: int, chunk: int = 4096):
    """SetSample(start) then the chunked loop -> (frames or -2/-3, samples, crc_errors, status_or, seek_rc)"""
    L = lib()
    f = L.emu_decode_from
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32),
                  ctypes.POINTER(ctypes.c_int)]
    cap = max(len(data) * 16, 1 << 16)
    while True:
        out = np.zeros(cap, dtype=np.int32)
        crc, nch, st, src = ctypes.c_int64(0), ctypes.c_int(0), ctypes.c_uint32(0), ctypes.c_int(0)
        n = f(data, len(data), int(start), chunk, out.ctypes.data, cap, ctypes.byref(crc), ctypes.byref(nch),
              ctypes.byref(st), ctypes.byref(src))
        if n == -4:
            cap *= 4
            continue
        if n < 0:
            return int(n), np.zeros(0, np.int32), crc.value, st.value, src.value
        return int(n), out[: n * nch.value].copy(), crc.value, st.value, src.value


def file_info(data: bytes) -> dict:
    vals = np.zeros(len(INFO_FIELDS), dtype=np.int64)
    lib().emu_file_info(data, len(data), vals.ctypes.data, len(INFO_FIELDS))
    return dict(zip(INFO_FIELDS, (int(v) for v in vals)))


INFO_FIELDS_FULL = INFO_FIELDS + ("lossy_blocks", "is_five", "file_format", "header_off", "header_len", "trailer_off",
                                  "trailer_len", "first_call_frames", "config_flags", "sample_index0", "exception",
                                  "nondet")


def _desc_layout():
    v = np.zeros(7, dtype=np.int64)
    f = lib().emu_desc_layout
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f(v.ctypes.data, 7)
    return (int(x) for x in v)


# sizeof(BlockDesc) and offsetof kind / dsd_table_off / inherit / median / bits_off / bits_len (wv_desc.h)
DESC_BYTES, DESC_KIND, DESC_DSD_TABLE_OFF, DESC_INHERIT, DESC_MEDIAN, DESC_BITS_OFF, DESC_BITS_LEN = _desc_layout()
KIND_DSD_FAST = 2


def file_info_full(data: bytes, chunk: int = 4096) -> dict:
    f = lib().emu_file_info_chunk
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    vals = np.zeros(len(INFO_FIELDS_FULL), dtype=np.int64)
    f(data, len(data), chunk, vals.ctypes.data, len(vals))
    return dict(zip(INFO_FIELDS_FULL, (int(v) for v in vals)))


def frame_descs(data: bytes, chunk: int = 4096, seek: int = -1) -> bytes:
    """host framing (deferred values applied) -> descriptor bytes"""
    f = lib().emu_frame_descs
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                  ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    cap = (len(data) // 32 + 16) * DESC_BYTES
    out = np.zeros(cap, np.uint8)
    nj = ctypes.c_int64(0)
    n = f(data, len(data), seek, chunk, 1, out.ctypes.data, cap, ctypes.byref(nj))
    assert n >= 0
    return out[: n * DESC_BYTES].tobytes()


def dframe(data: bytes, chunk: int = 4096):
    """device framing run on the host -> (descriptor bytes, info dict) or (None, why)"""
    f = lib().emu_dframe
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                  ctypes.c_int]
    cap = (len(data) // 32 + 16) * DESC_BYTES
    out = np.zeros(cap, np.uint8)
    vals = np.zeros(len(INFO_FIELDS_FULL), dtype=np.int64)
    n = f(data, len(data), chunk, out.ctypes.data, cap, vals.ctypes.data, len(vals))
    if n < 0:
        return None, int(-n - 1)
    return out[: n * DESC_BYTES].tobytes(), dict(zip(INFO_FIELDS_FULL, (int(v) for v in vals)))


def decode_wvc(data: bytes, wvc: bytes | None, chunk: int = 4096, open_flags: int = 0):
    """.wv (+ .wvc) through the device core on the host -> (frames, samples, crc_errors, status_or)"""
    f = lib().emu_decode_wvc
    f.restype = ctypes.c_int64
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32,
                  ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int),
                  ctypes.POINTER(ctypes.c_uint32)]
    cap = max(len(data) * 32, 1 << 16)
    out = np.zeros(cap, dtype=np.int32)
    crc, nch, st = ctypes.c_int64(0), ctypes.c_int(0), ctypes.c_uint32(0)
    wvc = wvc or b""
    n = f(data, len(data), wvc, len(wvc), chunk, open_flags, out.ctypes.data, cap, ctypes.byref(crc),
          ctypes.byref(nch), ctypes.byref(st))
    if n < 0:
        return int(n), np.zeros(0, np.int32), crc.value, st.value
    return int(n), out[: n * nch.value].copy(), crc.value, st.value
