"""Output-range reservation of a multi-file batch (wv_framing.cpp file_out_extent,
used by wvg_batch_add_file): every descriptor's writes stay inside its file's
reserved range.  A file that raises the reference's C# exception mid-call keeps
the descriptor of that call, which writes past the file's reported frames; with
only the reported values reserved it overwrote the next file's first block on
the GPU (a race between the two blocks' stores).  Host framing only (tests/emu)."""
import ctypes

import numpy as np

from tests.emu import emu as E
from tests.test_meta_defer import _bases, meta_fuzz


def _ranges(files, chunk=4096):
    L = E.lib()
    f = L.emu_batch_ranges
    f.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    f.restype = None
    blob = bytearray()
    offs, lens = [], []
    for d in files:
        blob += b"\0" * ((-len(blob)) % 16)
        offs.append(len(blob))
        lens.append(len(d))
        blob += d
    offs = np.array(offs, dtype=np.uint64)
    lens = np.array(lens, dtype=np.uint64)
    bad_r, bad_v = ctypes.c_int64(), ctypes.c_int64()
    f(bytes(blob), offs.ctypes.data, lens.ctypes.data, len(files), chunk, ctypes.byref(bad_r), ctypes.byref(bad_v))
    return bad_r.value, bad_v.value


def test_exception_file_range_is_reserved():
    # the GPU test's batch (test_gpu_parity.test_fuzzed_metadata_device_parse):
    # files 1 and 17 raise the exception with a block still open
    files = [meta_fuzz(d, 9000 + 100 * b + s) for b, d in enumerate(_bases()) for s in range(12)]
    bad_reserved, bad_values = _ranges(files)
    assert bad_values > 0  # the batch does hold descriptors past their file's reported frames
    assert bad_reserved == 0


def test_plain_batch_ranges():
    files = [d for d in _bases()]
    assert _ranges(files) == (0, 0)
    assert _ranges(files, chunk=1000) == (0, 0)
