"""Host-side mirror of the reference's public API for the decode path.

Reference (C#, Quake4/WavPackDecoder WavPackUtils.cs):
    WavpackOpenFileInput(BinaryReader, uint flags=0)      :36-120
    WavpackUnpackSamples(WavpackContext, int[] buffer, long samples)  :200-282
    WavpackFormatSamples(int[] src, long samcnt, int bps, byte[] pcm, int offset=0, bool dsd=false) :288-341
    WavpackGetNumSamples / GetSampleIndex / GetNumErrors / Lossy / GetSampleRate /
    GetNumChannels / GetBitsPerSample / GetBytesPerSample / GetReducedChannels /
    GetMode / GetFileFormat / GetFileExtension / GetErrorMessage / GetHeader /
    GetTrailer / GetIsFive / GetVersion / GetIsFloat       :346-499

Same names, same argument meaning and the same error behaviour (errors are
reported through GetErrorMessage; a call that the reference would abort with a
C# exception raises WavpackException here, after every earlier call has
returned its frames).  Underneath, the whole file is decoded by the MI355X
kernels on the first WavpackUnpackSamples call and served from the decoded
buffer; the chunk schedule is the caller's request size (the reference's
seams are a function of it).  GetSampleIndex / GetNumErrors follow the calls
made so far (WavPackUtils.cs:273-275, 355-366).  A caller that changes its
request size mid-stream gets the samples of a decode scheduled at the first
request size: identical for every well-formed stream (seams only matter for
the (short) weight store of pathological weights and for the mute granularity
of corrupted streams), and reported through `schedule_changed`.

For throughput use DecodeBatch: many files, one upload, one decode.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib as _L  # noqa: E402


def configure_hw_queues(n: int = 16) -> None:
    """Opt-in: ask HIP for `n` hardware queues per process (GPU_MAX_HW_QUEUES; HIP's
    default is 4).  A decode runs its launch groups on streams of their own and a
    server keeps several batches in flight; streams beyond the process's queues
    share one and their kernels serialise.  It only takes effect before the
    process's first HIP call, and it applies to every HIP user of the process, so
    the library never sets it by itself: call this (or export the variable in the
    launcher) first.  Measured (profiles/r06_pipe_pc.jsonl): a producer/consumer
    server over 16-20 batches serves ~7,000 Msamples/s of C2 PCM on HIP's 4 queues
    and 9,500-10,400 on 24 (bench.py's setting)."""
    if not 1 <= int(n) <= 32:
        raise ValueError("GPU_MAX_HW_QUEUES must be in 1..32")
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))

SAMPLE_BUFFER_SIZE = 4096  # Defines.cs:18
OPEN_2CH_MAX = 0x8         # Defines.cs:26
# beyond the reference: float files decode to float32 bit patterns, exact via the wvx stream
# (WVG_OPEN_EXACT_FLOAT, include/wvgpu.h)
OPEN_EXACT_FLOAT = 0x40000000


class WavpackException(RuntimeError):
    """The reference would have raised a C# exception (WvDemo.cs:144 catch)."""


class DecoderTimeout(RuntimeError):
    """A decode kernel's bounded wait ran out (WVG_ST_TIMEOUT): a decoder fault, never a
    property of the stream and never reported as a reference exception."""


_ctx = None


def _context():
    global _ctx
    if _ctx is None:
        L = _L.lib()
        _ctx = L.wvg_open(-1)
        if not _ctx:
            raise RuntimeError("wvg_open failed: no HIP device visible (the decode path is GPU-only)")
    return _ctx


def _file_arrays(files):
    """(the files as bytes objects, a c_char_p array of them, their lengths as a uint64
    array) for the C-ABI's file-array calls; bytes inputs are passed as they are."""
    bufs = files if all(type(f) is bytes for f in files) else [bytes(f) for f in files]
    ptrs = (ctypes.c_char_p * len(bufs))(*bufs)
    lens = np.fromiter(map(len, bufs), dtype=np.uint64, count=len(bufs))
    return bufs, ptrs, lens


class DecodeBatch:
    """A batch of .wv files decoded together on one GPU (files shard across GPUs)."""

    def __init__(self, chunk_frames: int = SAMPLE_BUFFER_SIZE):
        self._L = _L.lib()
        self._b = self._L.wvg_batch_new(_context(), int(chunk_frames))
        if not self._b:
            raise RuntimeError("wvg_batch_new failed")
        self.infos: list = []
        self._dev_infos: list = []  # indices of device-framed files (their infos come with the upload)
        self._uploaded = False
        self._data: list = []

    def add_file(self, data: bytes, open_flags: int = 0, start_sample: int | None = None, wvc: bytes | None = None):
        """Frame one file; with start_sample, as a caller that calls SetSample(start_sample)
        right after WavpackOpenFileInput (WavPackUtils.cs:509-594).  wvc: the hybrid file's
        .wvc correction file -- its hybrid blocks then decode exactly (beyond the reference)."""
        info = _L.WvgFileInfo()
        if wvc is not None:
            if start_sample is not None:
                raise ValueError("wvc with start_sample is not supported")
            idx = self._L.wvg_batch_add_file_wvc(self._b, data, len(data), wvc, len(wvc), int(open_flags),
                                                 ctypes.byref(info))
        elif start_sample is None:
            idx = self._L.wvg_batch_add_file(self._b, data, len(data), int(open_flags), ctypes.byref(info))
        else:
            idx = self._L.wvg_batch_add_file_at(self._b, data, len(data), int(open_flags), int(start_sample),
                                                ctypes.byref(info))
        # the C side reserves a file slot on success and on WVG_ERR_OPEN (an input that
        # does not open); any other negative code reserved nothing, so infos[i] must
        # not grow either (it mirrors the C file index i)
        if idx < 0 and idx != _L.WVG_ERR_OPEN:
            self._check(idx)
        self.infos.append(info)
        self._uploaded = False
        return idx

    def reset(self):
        """Drop every file, keep the device and page-locked buffers (wvg_batch_reset)."""
        self._check(self._L.wvg_batch_reset(self._b))
        self.infos = []
        self._dev_infos = []
        self._uploaded = False

    def add_files(self, files, open_flags: int = 0, threads: int = 0):
        """Frame many files on host threads (wvg_batch_add_files); returns their indices."""
        n = len(files)
        if n == 0:
            return []
        bufs, ptrs, lens = _file_arrays(files)
        infos = (_L.WvgFileInfo * n)()
        idx = np.empty(n, dtype=np.int32)
        rc = self._L.wvg_batch_add_files(self._b, n, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                         int(open_flags), int(threads), ctypes.cast(infos, ctypes.c_void_p),
                                         idx.ctypes.data)
        if rc < 0:
            self._check(rc)
        self.infos.extend(infos)
        self._uploaded = False
        return idx.tolist()

    def add_files_device(self, files):
        """Queue files for device-side framing at the next upload
        (wvg_batch_add_files_device); returns their indices.  Their infos are
        filled in by upload()."""
        n = len(files)
        if n == 0:
            return []
        bufs, ptrs, lens = _file_arrays(files)
        idx = np.empty(n, dtype=np.int32)
        rc = self._L.wvg_batch_add_files_device(self._b, n, ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data,
                                                idx.ctypes.data)
        if rc < 0:
            self._check(rc)
        self._dev_infos.extend(range(len(self.infos), len(self.infos) + n))
        self.infos.extend(_L.WvgFileInfo() for _ in range(n))
        self._uploaded = False
        return idx.tolist()

    def framing_stats(self):
        """(files framed on the device, files framed by the host fallback)"""
        dev, host = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._L.wvg_batch_framing_stats(self._b, ctypes.byref(dev), ctypes.byref(host)))
        return int(dev.value), int(host.value)

    def lane_groups(self) -> int:
        """Diagnostics: the launch groups the last decode ran on lane / row kernels (bit t:
        PCM term set t; 8 .wvc; 9 DSD mode 3; 10 DSD mode 1) -- wvg_batch_lane_groups."""
        m = ctypes.c_uint32()
        self._check(self._L.wvg_batch_lane_groups(self._b, ctypes.byref(m)))
        return int(m.value)

    def upload(self):
        self._check(self._L.wvg_batch_upload(self._b))
        if self._dev_infos:  # device-framed files get their infos here (one call for the lot)
            lo, hi = min(self._dev_infos), max(self._dev_infos) + 1
            arr = (_L.WvgFileInfo * (hi - lo))()
            got = self._L.wvg_batch_file_infos(self._b, lo, hi - lo, ctypes.cast(arr, ctypes.c_void_p))
            for i in self._dev_infos:
                if i - lo < got:
                    self.infos[i] = arr[i - lo]
            self._dev_infos = []
        self._uploaded = True

    def decode(self, stream=None):
        if not self._uploaded:
            self.upload()
        self._check(self._L.wvg_batch_decode(self._b, stream))

    def sync(self):
        self._check(self._L.wvg_batch_sync(self._b))

    def poison(self, byte: int = 0x7F):
        """Overwrite the output with `byte` and mark every decodable block's status
        WVG_ST_UNWRITTEN (wvg_batch_poison): what a later download shows was written by
        the decodes issued after this call."""
        if not self._uploaded:
            self.upload()
        self._check(self._L.wvg_batch_poison(self._b, int(byte)))

    def set_kernel(self, kernel: str):
        """'auto' (the default: the lane kernels once the context has had batches in
        flight together, until then one workgroup per block for groups of up to 2,048
        blocks), 'lane' (one lane per
        block: the most blocks per second with batches in flight) or 'two_wave' (one
        workgroup per block: lowest latency for a batch alone) -- wvg_batch_set_kernel;
        results are identical in every mode."""
        k = {"two_wave": _L.WVG_KERNEL_TWO_WAVE, "lane": _L.WVG_KERNEL_LANE, "auto": _L.WVG_KERNEL_AUTO}[kernel]
        self._check(self._L.wvg_batch_set_kernel(self._b, k))

    def set_timing(self, on: bool = True):
        """Record a device event pair around every following decode (wvg_batch_set_timing)."""
        self._check(self._L.wvg_batch_set_timing(self._b, int(bool(on))))

    def timed(self):
        """(mean ms, count) of the decodes recorded since set_timing(True)."""
        ms, n = ctypes.c_float(), ctypes.c_int()
        self._check(self._L.wvg_batch_timed(self._b, ctypes.byref(ms), ctypes.byref(n)))
        return float(ms.value), int(n.value)

    def group_times(self):
        """With timing on: {group: ms from the last decode's start to the group's end}
        (groups: 'ts0'..'ts7' term sets, 'pcm' generic, 'dsd', 'dsd1')."""
        ms = (ctypes.c_float * 11)()
        rc = self._L.wvg_batch_group_times(self._b, ms, 11)
        if rc < 0:
            self._check(rc)
        names = [f"ts{i}" for i in range(8)] + ["pcm", "dsd", "dsd1"]
        return {n: round(float(v), 3) for n, v in zip(names, ms) if v >= 0}

    def time(self, iters: int) -> float:
        ms = ctypes.c_float()
        self._check(self._L.wvg_batch_time(self._b, int(iters), ctypes.byref(ms)))
        return float(ms.value)

    @property
    def out_ints(self) -> int:
        return int(self._L.wvg_batch_out_ints(self._b))

    @property
    def num_blocks(self) -> int:
        return int(self._L.wvg_batch_num_blocks(self._b))

    @property
    def frames(self) -> int:
        return int(self._L.wvg_batch_frames(self._b))

    @property
    def bytes_in(self) -> int:
        return int(self._L.wvg_batch_bytes_in(self._b))

    def device_out_ptr(self) -> int:
        return int(self._L.wvg_batch_device_out(self._b) or 0)

    def download(self, pinned: bool = False) -> np.ndarray:
        """The int32 output.  pinned=True: DMA into the batch's page-locked buffer and
        return a view of it (valid until the next download or close)."""
        if pinned:
            self._check(self._L.wvg_batch_download(self._b, None, -1))
            p = self._L.wvg_batch_host_out(self._b)
            n = self.out_ints
            if not p or n == 0:
                return np.zeros(0, dtype=np.int32)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int32)), shape=(n,))
        out = np.empty(max(self.out_ints, 1), dtype=np.int32)
        self._check(self._L.wvg_batch_download(self._b, out.ctypes.data, out.size))
        return out[: self.out_ints]

    def block_status(self) -> np.ndarray:
        n = self.num_blocks + 1024
        st = np.zeros(n, dtype=np.uint32)
        k = self._L.wvg_batch_block_status(self._b, st.ctypes.data, n)
        if k < 0:
            raise RuntimeError("block status unavailable (download first)")
        return st[:k]

    def lane_counters(self, ts: int) -> np.ndarray:
        """Diagnostics (a batch made with WVG_LANE_COUNTERS=1): per parser wave of term set
        `ts`'s last lane decode [cycles, groups, bulk, norun, split, fast, checked, replay,
        wait_consumed, wait_loads, words, stage, 0...] (wvg_batch_lane_counters)."""
        buf = np.zeros(16 * 4096, dtype=np.uint32)
        k = self._L.wvg_batch_lane_counters(self._b, int(ts), buf.ctypes.data, buf.size)
        if k < 0:
            raise RuntimeError("lane counters unavailable (WVG_LANE_COUNTERS=1 before the batch is made)")
        return buf[: 16 * k].reshape(k, 16)

    def file_blocks(self, i: int):
        """(end_frame, status) per block of file i (wvg_batch_file_blocks)."""
        n = self.num_blocks + 1
        ends = np.zeros(n, dtype=np.int64)
        st = np.zeros(n, dtype=np.uint32)
        k = self._L.wvg_batch_file_blocks(self._b, int(i), ends.ctypes.data, st.ctypes.data, n)
        if k < 0:
            raise RuntimeError("file blocks unavailable (download first)")
        return ends[:k], st[:k]

    def format(self, dsd: bool = False, stream=None):
        """WavpackFormatSamples (WavPackUtils.cs:288-341) over the decoded batch, on the device."""
        self._check(self._L.wvg_batch_format(self._b, int(bool(dsd)), stream))

    def pcm_offset(self, i: int) -> int:
        return int(self._L.wvg_batch_pcm_offset(self._b, int(i)))

    def download_pcm_async(self):
        """Queue the PCM download into the batch's page-locked buffer behind the format
        (wvg_batch_download_pcm_async); after sync(), host_pcm() is the image."""
        self._check(self._L.wvg_batch_download_pcm_async(self._b))

    def host_pcm(self) -> np.ndarray:
        """The page-locked PCM image of the last pinned / async download (a view)."""
        n = int(self._L.wvg_batch_pcm_bytes(self._b))
        p = self._L.wvg_batch_host_pcm(self._b)
        if not p or n == 0:
            return np.zeros(0, dtype=np.uint8)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))

    def download_pcm(self, pinned: bool = False) -> np.ndarray:
        """The formatted PCM bytes.  pinned=True: DMA into the batch's page-locked
        buffer and return a view of it (valid until the next such download or close)."""
        n = int(self._L.wvg_batch_pcm_bytes(self._b))
        if pinned:
            self._check(self._L.wvg_batch_download_pcm(self._b, None, -1))
            p = self._L.wvg_batch_host_pcm(self._b)
            if not p or n == 0:
                return np.zeros(0, dtype=np.uint8)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(n,))
        out = np.empty(max(n, 1), dtype=np.uint8)
        self._check(self._L.wvg_batch_download_pcm(self._b, out.ctypes.data, out.size))
        return out[:n]

    def wav(self, i: int):
        """WvDemo.Main for file i (WvDemo.cs:15-168): (exit_code, .wav bytes)."""
        n, rc = ctypes.c_int64(), ctypes.c_int32()
        self._check(self._L.wvg_batch_wav(self._b, int(i), None, 0, ctypes.byref(n), ctypes.byref(rc)))
        buf = np.empty(max(n.value, 1), dtype=np.uint8)
        self._check(self._L.wvg_batch_wav(self._b, int(i), buf.ctypes.data, buf.size, ctypes.byref(n), ctypes.byref(rc)))
        return int(rc.value), buf[: n.value].tobytes()

    def result(self, i: int) -> _L.WvgFileResult:
        r = _L.WvgFileResult()
        self._check(self._L.wvg_batch_file_result(self._b, int(i), ctypes.byref(r)))
        return r

    def _check(self, rc: int):
        if rc == _L.WVG_ERR_TIMEOUT:
            raise DecoderTimeout(self._L.wvg_last_error(_context()).decode())
        if rc != 0:
            raise RuntimeError(f"libwvgpu error {rc}: {self._L.wvg_last_error(_context()).decode()}")

    def close(self):
        if self._b:
            self._L.wvg_batch_free(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WavpackContext:
    """Opaque context (WavpackContext.cs:13-35) over a wvg_stream: the file is decoded
    on the device by the first WavpackUnpackSamples call and served a window at a
    time, so host memory holds the compressed file and two windows, not the output."""

    def __init__(self, data: bytes, open_flags: int, window_frames: int = 0):
        self._data = data
        self._flags = open_flags
        self._window = int(window_frames)
        self._info = _L.WvgFileInfo()
        self._s = None
        self.error_message = None

    def _stream(self):
        if self._s is None:
            self._s = _L.lib().wvg_stream_open(_context(), self._data, len(self._data), int(self._flags),
                                               self._window, ctypes.byref(self._info))
            if not self._s:
                raise RuntimeError("wvg_stream_open failed: " + _L.lib().wvg_last_error(_context()).decode())
        return self._s

    def _state(self):
        idx, err = ctypes.c_int64(), ctypes.c_int64()
        lossy, changed = ctypes.c_int32(), ctypes.c_int32()
        _L.lib().wvg_stream_state(self._stream(), ctypes.byref(idx), ctypes.byref(err), ctypes.byref(lossy),
                                  ctypes.byref(changed))
        return int(idx.value), int(err.value), bool(lossy.value), bool(changed.value)

    @property
    def schedule_changed(self) -> bool:
        return self._state()[3] if self._s else False

    def close(self):
        if self._s:
            _L.lib().wvg_stream_close(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def WavpackOpenFileInput(reader, flags: int = 0, window_frames: int = 0) -> WavpackContext:
    """WavPackUtils.cs:36-120.  `reader` is bytes or a binary file object."""
    data = reader if isinstance(reader, (bytes, bytearray, memoryview)) else reader.read()
    data = bytes(data)
    wpc = WavpackContext(data, flags, window_frames)
    L = _L.lib()
    rc = L.wvg_probe_file(data, len(data), int(flags), SAMPLE_BUFFER_SIZE, ctypes.byref(wpc._info))  # host only
    if rc < 0 or not wpc._info.open_ok:
        wpc.error_message = wpc._info.error.decode() or "not compatible with this version of WavPack file!"
    return wpc


def WavpackUnpackSamples(wpc: WavpackContext, buffer: np.ndarray, samples: int) -> int:
    """WavPackUtils.cs:200-282: fill `buffer` (int32, >= samples * reduced channels)."""
    if wpc.error_message:
        return 0
    nch = max(int(wpc._info.reduced_channels), 1)
    if buffer.dtype != np.int32 or not buffer.flags.c_contiguous or buffer.size < int(samples) * nch:
        raise ValueError("buffer: contiguous int32 of samples x reduced channels")
    n = _L.lib().wvg_stream_unpack(wpc._stream(), buffer.ctypes.data, int(samples))
    if n == _L.WVG_ERR_EXCEPTION:
        raise WavpackException("the reference decoder raises an exception in this call")
    if n == _L.WVG_ERR_TIMEOUT:
        raise DecoderTimeout(_L.lib().wvg_last_error(_context()).decode())
    if n < 0:
        raise RuntimeError(f"libwvgpu error {n}: {_L.lib().wvg_last_error(_context()).decode()}")
    return int(n)


def SetSample(wpc: WavpackContext, sample: int) -> bool:
    """WavPackUtils.cs:509-594.  The block search runs on the host framing; the file
    is then decoded from the block the reference's search lands on (its discard
    calls included), and the result is the C# return value.  (After samples were
    already handed out, the block search of the reference starts from the current
    block; for well-formed files it ends on the same block, which is what this
    mirror decodes from.)"""
    if wpc.error_message:
        return False
    rc = _L.lib().wvg_stream_set_sample(wpc._stream(), int(sample))
    if rc == _L.WVG_ERR_EXCEPTION:
        raise WavpackException("the reference's SetSample raises an exception on this file")
    if rc == _L.WVG_ERR_TIMEOUT:
        raise DecoderTimeout(_L.lib().wvg_last_error(_context()).decode())
    if rc < 0:
        raise RuntimeError(f"libwvgpu error {rc}: {_L.lib().wvg_last_error(_context()).decode()}")
    return rc == 1


def SetTime(wpc: WavpackContext, milliseconds: int) -> bool:
    """WavPackUtils.cs:504-507: SetSample(ms / 1000 * sample_rate) (integer division first)."""
    return SetSample(wpc, int(milliseconds) // 1000 * int(wpc._info.sample_rate))


def WavpackFormatSamples(src: np.ndarray, samcnt: int, bps: int, pcm_buffer: bytearray, offset: int = 0,
                         dsd: bool = False) -> bool:
    """WavPackUtils.cs:288-341 (host C implementation in libwvgpu)."""
    L = _L.lib()
    s = np.ascontiguousarray(src, dtype=np.int32)
    if pcm_buffer is None or len(pcm_buffer) < int(samcnt) * int(bps) + int(offset):
        return False
    if int(bps) in (1, 2, 3, 4) and int(samcnt) > s.size:  # src[counter2++] past the array
        raise WavpackException("IndexOutOfRangeException in WavpackFormatSamples")
    view = (ctypes.c_uint8 * len(pcm_buffer)).from_buffer(pcm_buffer)
    return bool(L.wvg_format_samples(s.ctypes.data, int(samcnt), int(bps), ctypes.addressof(view), len(pcm_buffer),
                                     int(offset), int(bool(dsd))))


def wv_demo(data: bytes):
    """WvDemo.Main (WvDemo.cs:15-168) on the GPU path: (exit_code, .wav bytes).

    Decode (WavpackUnpackSamples calls of SAMPLE_BUFFER_SIZE frames), the
    WavpackFormatSamples epilogue on the device, then the header / PCM /
    trailer layout WvDemo writes."""
    b = DecodeBatch(SAMPLE_BUFFER_SIZE)
    try:
        idx = b.add_file(bytes(data))
        if idx < 0:
            return 1, b""
        b.decode()
        b.format(dsd=False)
        return b.wav(idx)
    finally:
        b.close()


def WavpackGetNumSamples(wpc, native: bool = False) -> int:
    t = wpc._info.total_samples
    return t * 8 if native and wpc._info.dsd_multiplier > 0 else t


def WavpackGetSampleIndex(wpc) -> int:
    """stream.sample_index (WavPackUtils.cs:355-358): where the next call starts."""
    if wpc.error_message:
        return int(wpc._info.sample_index0)
    return wpc._state()[0]


def WavpackGetNumErrors(wpc) -> int:
    """crc_errors: blocks whose last frame a call has unpacked and whose check failed
    (WavPackUtils.cs:273-275), SetSample's discard calls included."""
    if wpc.error_message:
        return 0
    return wpc._state()[1]


def WavpackLossy(wpc) -> bool:
    if wpc.error_message:
        return bool(wpc._info.lossy)
    return wpc._state()[2]


# wvg_file_info carries the getters' results (wv_api.cpp fill_info applies
# WavPackUtils.cs:379-442: DSD rate x multiplier x 8, bits / 8, defaults).
def WavpackGetSampleRate(wpc) -> int:
    return int(wpc._info.sample_rate)


def WavpackGetNumChannels(wpc) -> int:
    return int(wpc._info.num_channels)


def WavpackGetBitsPerSample(wpc) -> int:
    return int(wpc._info.bits_per_sample)


def WavpackGetBytesPerSample(wpc) -> int:
    return int(wpc._info.bytes_per_sample)


def WavpackGetReducedChannels(wpc) -> int:
    return int(wpc._info.reduced_channels)


def WavpackGetMode(wpc) -> int:
    return int(wpc._info.mode)


def WavpackGetFileFormat(wpc) -> int:
    return int(wpc._info.file_format)


def WavpackGetErrorMessage(wpc):
    return wpc.error_message


def WavpackGetVersion(wpc) -> int:
    return int(wpc._info.version)


def WavpackGetIsFloat(wpc) -> bool:
    return bool(wpc._info.is_float)


def WavpackGetIsFive(wpc) -> bool:
    return bool(wpc._info.is_five)


def WavpackGetHeader(wpc):
    i = wpc._info
    return None if i.header_off < 0 else wpc._data[i.header_off:i.header_off + i.header_len]


def WavpackGetTrailer(wpc):
    i = wpc._info
    return None if i.trailer_off < 0 else wpc._data[i.trailer_off:i.trailer_off + i.trailer_len]
