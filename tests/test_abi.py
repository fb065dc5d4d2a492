"""The drop-in boundary: libwvgpu.so loads without a GPU and exports exactly
what include/wvgpu.h declares; host-only entry points behave like the oracle.

No GPU compute is called here (wvg_open and the batch calls need a device);
wvg_format_samples is host code (WavPackUtils.cs:288-341) and is checked
against the oracle's restatement.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from wavpackdecoder_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wvgpu.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wvg_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "wavpackdecoder_amd")])
    return ctypes.CDLL(_lib.LIB_PATH)


def test_header_matches_binding():
    assert declared() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol(lib):
    for name in declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    syms = set(re.findall(r" T (wvg_[a-z_]+)$", out, flags=re.M))
    assert set(declared()) <= syms


def test_binding_loads_and_types(lib):
    L = _lib.lib()  # loads and sets argtypes; no device call
    for name in _lib.EXPORTED:
        assert getattr(L, name).restype is not None or name in ("wvg_close", "wvg_batch_free", "wvg_stream_close")


def _fmt(fn, src, samcnt, bps, cap, offset=0, dsd=0):
    buf = np.full(cap, 0xAB, dtype=np.uint8)
    ok = fn(src.ctypes.data, samcnt, bps, buf.ctypes.data, cap, offset, dsd)
    return ok, buf


@pytest.mark.parametrize("bps", [1, 2, 3, 4])
@pytest.mark.parametrize("dsd", [0, 1])
def test_format_samples_matches_oracle(lib, bps, dsd):
    rng = np.random.default_rng(bps * 10 + dsd)
    src = rng.integers(-(1 << 31), (1 << 31) - 1, size=257, dtype=np.int64).astype(np.int32)
    lib.wvg_format_samples.restype = ctypes.c_int
    lib.wvg_format_samples.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_int, ctypes.c_int]
    Lo = O.lib()
    Lo.wvo_format_samples.restype = ctypes.c_int
    Lo.wvo_format_samples.argtypes = lib.wvg_format_samples.argtypes
    for samcnt, cap, off in ((257, 257 * 4 + 8, 0), (100, 1024, 5), (257, 10, 0), (0, 16, 0)):
        a = _fmt(lib.wvg_format_samples, src, samcnt, bps, cap, off, dsd)
        b = _fmt(Lo.wvo_format_samples, src, samcnt, bps, cap, off, dsd)
        assert a[0] == b[0]
        assert np.array_equal(a[1], b[1])
