"""ctypes binding of libwvgpu.so (include/wvgpu.h).

The product path has exactly one implementation: the HIP kernels inside
libwvgpu.so.  There is no CPU fallback -- if the library is missing or no
GPU is visible, every decode entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WVG_LIB") or os.path.join(_PKG, "build", "libwvgpu.so")  # WVG_LIB: experiment builds

WVG_ST_CRC_CHECKED = 0x01
WVG_ST_CRC_ERROR = 0x02
WVG_ST_MUTED = 0x04
WVG_ST_BITS_ERROR = 0x08
WVG_ST_EXCEPTION = 0x10
WVG_ST_UNSUPPORTED = 0x20
WVG_ST_DSD_MUTE = 0x40
WVG_ST_NONDET = 0x80
WVG_ST_TIMEOUT = 0x100
WVG_ST_REDONE = 0x200  # block status only: decoded by the lane kernel's fallback
WVG_ST_UNWRITTEN = 0x40000000  # block status only: no decode stored it since wvg_batch_poison
WVG_ERR_ARG = -2
WVG_ERR_OPEN = -3
WVG_ERR_TIMEOUT = -5
WVG_ERR_EXCEPTION = -6
WVG_KERNEL_TWO_WAVE = 0
WVG_KERNEL_LANE = 1
WVG_KERNEL_AUTO = 2


class WvgFileInfo(ctypes.Structure):
    _fields_ = [
        ("open_ok", ctypes.c_int32), ("num_channels", ctypes.c_int32), ("reduced_channels", ctypes.c_int32),
        ("bits_per_sample", ctypes.c_int32), ("bytes_per_sample", ctypes.c_int32), ("version", ctypes.c_int32),
        ("mode", ctypes.c_int32), ("is_float", ctypes.c_int32), ("is_five", ctypes.c_int32),
        ("file_format", ctypes.c_int32), ("lossy", ctypes.c_int32), ("dsd_multiplier", ctypes.c_uint32),
        ("sample_rate", ctypes.c_int64), ("total_samples", ctypes.c_int64), ("out_frames", ctypes.c_int64),
        ("out_offset", ctypes.c_int64), ("header_off", ctypes.c_int64), ("header_len", ctypes.c_int64),
        ("trailer_off", ctypes.c_int64), ("trailer_len", ctypes.c_int64), ("error", ctypes.c_char * 96),
        ("seek_result", ctypes.c_int32), ("reserved", ctypes.c_int32), ("sample_index0", ctypes.c_int64),
    ]


class WvgFileResult(ctypes.Structure):
    _fields_ = [
        ("frames", ctypes.c_int64), ("crc_errors", ctypes.c_int64), ("lossy", ctypes.c_int32),
        ("exception", ctypes.c_int32), ("status_or", ctypes.c_uint32), ("num_blocks", ctypes.c_int32),
        ("exception_frame", ctypes.c_int64),
    ]


_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def build() -> str:
    """Compile libwvgpu.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-C", _PKG])
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} is missing: build it with `make -C wavpackdecoder_amd` (or __graft_entry__.build()). "
            "There is no CPU fallback for the decode path.")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
    sig = {
        "wvg_open": (vp, [i32]),
        "wvg_close": (None, [vp]),
        "wvg_last_error": (ctypes.c_char_p, [vp]),
        "wvg_batch_new": (vp, [vp, i32]),
        "wvg_batch_free": (None, [vp]),
        "wvg_batch_add_file": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, u32, ctypes.POINTER(WvgFileInfo)]),
        "wvg_batch_add_file_at": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, u32, i64, ctypes.POINTER(WvgFileInfo)]),
        "wvg_batch_add_files": (i32, [vp, i32, vp, vp, u32, i32, vp, vp]),
        "wvg_batch_add_files_device": (i32, [vp, i32, vp, vp, vp]),
        "wvg_batch_add_file_wvc": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, u32,
                                         ctypes.POINTER(WvgFileInfo)]),
        "wvg_batch_file_info": (i32, [vp, i32, ctypes.POINTER(WvgFileInfo)]),
        "wvg_batch_file_infos": (i32, [vp, i32, i32, vp]),
        "wvg_batch_framing_stats": (i32, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
        "wvg_batch_lane_groups": (i32, [vp, ctypes.POINTER(ctypes.c_uint32)]),
        "wvg_batch_upload": (i32, [vp]),
        "wvg_batch_reset": (i32, [vp]),
        "wvg_batch_decode": (i32, [vp, vp]),
        "wvg_batch_sync": (i32, [vp]),
        "wvg_batch_stream": (vp, [vp]),
        "wvg_batch_poison": (i32, [vp, i32]),
        "wvg_batch_set_timing": (i32, [vp, i32]),
        "wvg_batch_set_kernel": (i32, [vp, i32]),
        "wvg_batch_timed": (i32, [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]),
        "wvg_batch_group_times": (i32, [vp, vp, i32]),
        "wvg_batch_out_ints": (i64, [vp]),
        "wvg_batch_device_out": (vp, [vp]),
        "wvg_batch_num_blocks": (i64, [vp]),
        "wvg_batch_bytes_in": (i64, [vp]),
        "wvg_batch_frames": (i64, [vp]),
        "wvg_batch_download": (i32, [vp, vp, i64]),
        "wvg_batch_host_out": (vp, [vp]),
        "wvg_batch_file_result": (i32, [vp, i32, ctypes.POINTER(WvgFileResult)]),
        "wvg_batch_block_status": (i32, [vp, vp, i64]),
        "wvg_batch_lane_counters": (i32, [vp, i32, vp, i64]),
        "wvg_batch_file_blocks": (i32, [vp, i32, vp, vp, i64]),
        "wvg_batch_time": (i32, [vp, i32, ctypes.POINTER(ctypes.c_float)]),
        "wvg_decode_file": (i32, [vp, ctypes.c_char_p, ctypes.c_size_t, i32, vp, i64, ctypes.POINTER(WvgFileInfo),
                                  ctypes.POINTER(WvgFileResult)]),
        "wvg_probe_file": (i32, [ctypes.c_char_p, ctypes.c_size_t, u32, i32, ctypes.POINTER(WvgFileInfo)]),
        "wvg_format_samples": (i32, [vp, i64, i32, vp, i64, i32, i32]),
        "wvg_batch_format": (i32, [vp, i32, vp]),
        "wvg_batch_pcm_bytes": (i64, [vp]),
        "wvg_batch_pcm_offset": (i64, [vp, i32]),
        "wvg_batch_device_pcm": (vp, [vp]),
        "wvg_batch_download_pcm": (i32, [vp, vp, i64]),
        "wvg_batch_host_pcm": (vp, [vp]),
        "wvg_batch_download_pcm_async": (i32, [vp]),
        "wvg_batch_wav": (i32, [vp, i32, vp, i64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]),
        "wvg_stream_open": (vp, [vp, ctypes.c_char_p, ctypes.c_size_t, u32, i64, ctypes.POINTER(WvgFileInfo)]),
        "wvg_stream_unpack": (i64, [vp, vp, i64]),
        "wvg_stream_set_sample": (i32, [vp, i64]),
        "wvg_stream_state": (i32, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
        "wvg_stream_close": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if os.environ.get("WVG_LIB"):  # an older experiment build (A/B runs): entry points it lacks stay unbound
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


EXPORTED = ("wvg_open", "wvg_close", "wvg_last_error", "wvg_batch_new", "wvg_batch_free", "wvg_batch_add_file",
            "wvg_batch_add_file_at", "wvg_batch_add_files", "wvg_batch_add_files_device", "wvg_batch_file_info", "wvg_batch_file_infos",
            "wvg_batch_add_file_wvc",
            "wvg_batch_framing_stats", "wvg_batch_lane_groups",
            "wvg_batch_upload", "wvg_batch_reset", "wvg_batch_decode", "wvg_batch_sync", "wvg_batch_stream", "wvg_batch_poison", "wvg_batch_set_timing", "wvg_batch_set_kernel",
            "wvg_batch_timed", "wvg_batch_group_times", "wvg_batch_out_ints", "wvg_batch_device_out",
            "wvg_batch_num_blocks", "wvg_batch_bytes_in", "wvg_batch_frames", "wvg_batch_download", "wvg_batch_host_out",
            "wvg_batch_file_result", "wvg_batch_block_status", "wvg_batch_lane_counters", "wvg_batch_file_blocks", "wvg_batch_time", "wvg_decode_file",
            "wvg_probe_file", "wvg_format_samples", "wvg_batch_format", "wvg_batch_pcm_bytes", "wvg_batch_pcm_offset",
            "wvg_batch_device_pcm", "wvg_batch_download_pcm", "wvg_batch_host_pcm", "wvg_batch_download_pcm_async",
            "wvg_batch_wav",
            "wvg_stream_open", "wvg_stream_unpack", "wvg_stream_set_sample", "wvg_stream_state", "wvg_stream_close")
