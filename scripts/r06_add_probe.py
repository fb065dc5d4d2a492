"""Where a C5 slice's wvg_batch_add_files time goes (WVG_ADD_TRACE=1 prints copy / push / frame / merge
inside the library) against the Python call's wall time, for slices of 12,500 files."""
import os
import sys
import time

os.environ["WVG_ADD_TRACE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from synth import corpora  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

files = corpora.c5(25000)
b = DecodeBatch(4096)
for rep in range(3):
    for k in range(2):
        sl = files[k * 12500:(k + 1) * 12500]
        t0 = time.perf_counter()
        b.reset()
        t1 = time.perf_counter()
        b.add_files(sl)
        t2 = time.perf_counter()
        b.upload()
        t3 = time.perf_counter()
        print(f"rep {rep} slice {k}: reset {1e3 * (t1 - t0):.2f} ms, add_files {1e3 * (t2 - t1):.2f} ms, "
              f"upload {1e3 * (t3 - t2):.2f} ms", flush=True)
b.close()

# the same slices framed on the device (wvg_batch_add_files_device: the header / sub-block walk in kernels,
# the host keeping the files it declines)
os.environ["WVG_DFRAME_TRACE"] = "1"
b = DecodeBatch(4096)
for rep in range(3):
    for k in range(2):
        sl = files[k * 12500:(k + 1) * 12500]
        t0 = time.perf_counter()
        b.reset()
        t1 = time.perf_counter()
        b.add_files_device(sl)
        t2 = time.perf_counter()
        b.upload()
        t3 = time.perf_counter()
        print(f"device rep {rep} slice {k}: reset {1e3 * (t1 - t0):.2f} ms, add_files_device {1e3 * (t2 - t1):.2f} ms, "
              f"upload {1e3 * (t3 - t2):.2f} ms, framed (device, host) {b.framing_stats()}", flush=True)
b.close()
