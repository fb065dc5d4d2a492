#!/usr/bin/env python3
"""Regenerate the committed golden fixtures.

Each fixture is a small .wv stream written by the repo's own generator
(synth/, fixed seeds) plus, in manifest.json, what the oracle (the C
restatement of the reference path) decodes from it with 4096-frame calls:
frame count, status, crc_errors, the SHA-256 of the int32 output and its
first/last 64 samples.  The reference ships no fixtures of its own (SURVEY.md
§8c), so these pin the oracle and every decoder built here to one another and
to the generator's lossless input; they are data, not reference code.

usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from synth import wvsynth as S  # noqa: E402

F = 6000


def cases():
    x = S.audio_like(F, 2, 16, seed=101)
    x24 = S.audio_like(F, 2, 24, seed=102)
    m = S.audio_like(F, 1, 16, seed=103)
    mant = S.float_mantissas(x.astype(np.float32) / 32768.0)
    yield "stereo16_fast", S.encode_pcm(x, S.EncParams(terms=S.TERMS_FAST, block_samples=2500,
                                                       config_flags=0x200)), x
    yield "stereo16_default", S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=2500)), x
    yield "stereo16_high_nojoint", S.encode_pcm(x, S.EncParams(terms=S.TERMS_HIGH, joint_stereo=False,
                                                               block_samples=2500)), x
    yield "stereo24_high", S.encode_pcm(x24, S.EncParams(terms=S.TERMS_HIGH, bytes_per_sample=3,
                                                         block_samples=3000)), x24
    yield "mono16_high", S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, block_samples=2001)), m
    yield "false_stereo", S.encode_pcm(np.repeat(m, 2, axis=1), S.EncParams(
        nch=2, false_stereo=True, terms=S.TERMS_MONO_HIGH[:5], block_samples=2500)), np.repeat(m, 2, axis=1)
    yield "zeros", S.encode_pcm(S.audio_like(F, 2, 16, kind="zeros"), S.EncParams(block_samples=2500)), None
    yield "int32_zeros8", S.encode_pcm((x24.astype(np.int64) << 8).astype(np.int32), S.EncParams(
        terms=S.TERMS_DEFAULT, bytes_per_sample=4, int32_zeros=8, block_samples=2500)), None
    yield "hybrid_bitrate", S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, hybrid=True, hybrid_bitrate=True,
                                                        bitrate_x256=768, block_samples=2500)), None
    yield "float_hybrid", S.encode_pcm(mant, S.EncParams(terms=S.TERMS_FAST, bytes_per_sample=4, float_data=True,
                                                         hybrid=True, hybrid_bitrate=True, bitrate_x256=896,
                                                         block_samples=2500)), None
    for mode in (0, 1, 3):
        dd = S.dsd_random_like(F, 2, seed=104 + mode, density=0.35)
        yield f"dsd_mode{mode}", S.encode_dsd(dd, S.DsdParams(nch=2, mode=mode, block_samples=2500)), dd
    base = bytearray(S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=2500)))
    rng = np.random.default_rng(105)
    for _ in range(3):
        base[int(rng.integers(200, len(base)))] ^= 1 << int(rng.integers(0, 8))
    yield "corrupt_default", bytes(base), None


def main():
    manifest = {}
    for name, data, pcm in cases():
        r = O.decode_file(data, chunk=4096)
        if pcm is not None:
            assert np.array_equal(r.samples, pcm.reshape(-1)), name
        with open(os.path.join(HERE, name + ".wv"), "wb") as f:
            f.write(data)
        s = r.samples.astype("<i4")
        manifest[name] = {
            "file": name + ".wv", "bytes": len(data), "chunk": 4096, "frames": r.frames, "nch": r.nch,
            "status": r.status, "crc_errors": r.crc_errors, "lossless_input_checked": pcm is not None,
            "sha256_int32le": hashlib.sha256(s.tobytes()).hexdigest(),
            "head64": s[:64].tolist(), "tail64": s[-64:].tolist(),
        }
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(manifest)} fixtures, {sum(v['bytes'] for v in manifest.values())} bytes")


if __name__ == "__main__":
    main()
