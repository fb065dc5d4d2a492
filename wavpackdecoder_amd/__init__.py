"""wavpackdecoder_amd -- MI355X-native WavPack block decode (drop-in for the
reference's WavPackUtils.WavpackUnpackSamples hot path).

Layout:
  csrc/wv_wave2.h         two-wave PCM kernel: scalar parser wave + VALU reconstruction wave
  csrc/wv_decode.hip      HIP kernels for gfx950 (instantiations, lane-per-block PCM/DSD kernels)
  csrc/wv_decode_core.h   per-block decode (host+device source; lane kernels, tests/emu)
  csrc/wv_framing.cpp     host framing: .wv bytes -> block descriptors
  csrc/wv_api.cpp         C-ABI (include/wvgpu.h) -> build/libwvgpu.so
  api.py                  mirror of the reference's WavPackUtils API
  shard.py                per-GPU file partition (multi-GPU, no collectives)
"""
from .api import (  # noqa: F401
    DecodeBatch, WavpackContext, WavpackException, WavpackFormatSamples, WavpackGetBitsPerSample,
    WavpackGetBytesPerSample, WavpackGetErrorMessage, WavpackGetFileFormat, WavpackGetHeader, WavpackGetIsFive,
    WavpackGetIsFloat, WavpackGetMode, WavpackGetNumChannels, WavpackGetNumErrors, WavpackGetNumSamples,
    WavpackGetReducedChannels, WavpackGetSampleIndex, WavpackGetSampleRate, WavpackGetTrailer, WavpackGetVersion,
    WavpackLossy, WavpackOpenFileInput, WavpackUnpackSamples, wv_demo, SetSample, SetTime,
)
from ._lib import build, lib  # noqa: F401
