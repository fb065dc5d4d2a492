"""The BASELINE.json configurations as synthetic corpora.

C1  one 44.1 kHz 16-bit stereo file, 20 s (>= 409,600 frames, the WvDemo
    progress-modulo quirk WvDemo.cs:112,130), default terms, seed 1
C2  1,024 blocks x 22,050 frames, 16-bit stereo, fast {17,17}, joint stereo;
    ~2% all-zero blocks, ~1% full-scale noise blocks; seed 0xC2 + block
C3  4,096 blocks x 44,100 frames, 24-bit stereo, high 16-term chain (tests use
    fewer blocks; the bench names the count it ran)
C4  1,024 x 22,050 stereo FLOAT_DATA|HYBRID|HYBRID_BITRATE, 3.5 bits/sample
C5  mixed corpus: stereo16 / mono16 (some FALSE_STEREO) / stereo24 / mono24 /
    DSD modes 0/1/3, 1-2 blocks of 4,410-22,050 frames per file
Data is synthetic (no network, no datasets); every stream is produced by the
repo's own encoder (synth/wv_encoder.cpp).
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

from . import wvsynth as S

_CACHE = os.environ.get("WVSYNTH_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "wvsynth"))
_VERSION = "v2"


def _cached(key: str, make):
    os.makedirs(_CACHE, exist_ok=True)
    h = hashlib.sha1((_VERSION + key).encode()).hexdigest()[:16]
    path = os.path.join(_CACHE, f"{h}.npz")
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    d = make()
    tmp = path + f".{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        np.savez(f, **d)
    os.replace(tmp, path)
    return d


def c2_pcm(nblocks: int = 1024, block: int = 22050, seed0: int = 0xC2) -> np.ndarray:
    parts = []
    for b in range(nblocks):
        seed = seed0 + b
        r = (seed * 2654435761) % 100
        kind = "zeros" if r < 2 else ("noise" if r < 3 else "music")
        parts.append(S.audio_like(block, 2, 16, seed=seed, kind=kind))
    return np.concatenate(parts, axis=0)


def c2(nblocks: int = 1024, block: int = 22050, return_pcm: bool = False):
    def make():
        pcm = c2_pcm(nblocks, block)
        data = S.encode_pcm(pcm, S.EncParams(terms=S.TERMS_FAST, block_samples=block, joint_stereo=True,
                                             config_flags=0x200))
        return {"pcm": pcm, "wv": np.frombuffer(data, dtype=np.uint8)}
    d = _cached(f"c2-{nblocks}-{block}", make)
    data = d["wv"].tobytes()
    return (d["pcm"], data) if return_pcm else data


def _workers() -> int:
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "8") or 8), os.cpu_count() or 1))


def _c3_part(job):
    """Blocks [k0, k1) of C3: their PCM and their encoded stream (a run of whole
    blocks that starts at block_index k0 * block, as encode_pcm_parallel's parts)."""
    k0, k1, nblocks, block = job
    pcm = np.concatenate([S.audio_like(block, 2, 24, seed=0xC3 + b, sigma=4096.0) for b in range(k0, k1)], axis=0)
    p = S.EncParams(terms=S.TERMS_HIGH, bytes_per_sample=3, block_samples=block, config_flags=0x800 | 0x1000,
                    block_index_start=k0 * block, total_override=nblocks * block)
    return pcm, S.encode_pcm(pcm, p)


def c3(nblocks: int = 4096, block: int = 44100, return_pcm: bool = False):
    def make():
        # the PCM and the encode of whole-block parts in worker processes (the same stream
        # as encode_pcm_parallel over the concatenated PCM)
        from concurrent.futures import ProcessPoolExecutor
        w = _workers()
        per = max(1, (nblocks + w - 1) // w)
        jobs = [(k, min(k + per, nblocks), nblocks, block) for k in range(0, nblocks, per)]
        if len(jobs) == 1:
            parts = [_c3_part(jobs[0])]
        else:
            with ProcessPoolExecutor(max_workers=w) as ex:
                parts = list(ex.map(_c3_part, jobs))
        pcm = np.concatenate([p for p, _ in parts], axis=0)
        data = b"".join(d for _, d in parts)
        return {"pcm": pcm, "wv": np.frombuffer(data, dtype=np.uint8)}
    d = _cached(f"c3-{nblocks}-{block}", make)
    data = d["wv"].tobytes()
    return (d["pcm"], data) if return_pcm else data


def c4(nblocks: int = 1024, block: int = 22050):
    def make():
        pcm = c2_pcm(nblocks, block, seed0=0xC4)
        f = pcm.astype(np.float32) / 32768.0
        mant = S.float_mantissas(f)
        data = S.encode_pcm(mant, S.EncParams(terms=S.TERMS_DEFAULT, bytes_per_sample=4, float_data=True,
                                              hybrid=True, hybrid_bitrate=True, bitrate_x256=896,
                                              block_samples=block, config_flags=0x8 | 0x80))
        return {"wv": np.frombuffer(data, dtype=np.uint8)}
    return _cached(f"c4-{nblocks}-{block}", make)["wv"].tobytes()


def c4_wvc(nblocks: int = 1024, block: int = 22050):
    """C4 with its .wvc correction file -> (wv, wvc, the same mantissas encoded lossless)."""
    def make():
        pcm = c2_pcm(nblocks, block, seed0=0xC4)
        mant = S.float_mantissas(pcm.astype(np.float32) / 32768.0)
        common = dict(terms=S.TERMS_DEFAULT, bytes_per_sample=4, float_data=True, block_samples=block)
        wv, wvc = S.encode_pcm_wvc(mant, S.EncParams(hybrid_bitrate=True, bitrate_x256=896, config_flags=0x8 | 0x80,
                                                     **common))
        lossless = S.encode_pcm(mant, S.EncParams(**common))
        return {k: np.frombuffer(v, dtype=np.uint8) for k, v in (("wv", wv), ("wvc", wvc), ("ll", lossless))}
    d = _cached(f"c4wvc-{nblocks}-{block}", make)
    return d["wv"].tobytes(), d["wvc"].tobytes(), d["ll"].tobytes()


def c1(seconds: float = 20.0):
    frames = int(44100 * seconds)
    def make():
        pcm = S.audio_like(frames, 2, 16, seed=1)
        data = S.encode_pcm(pcm, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=22050, write_riff=True))
        return {"pcm": pcm, "wv": np.frombuffer(data, dtype=np.uint8)}
    d = _cached(f"c1-{frames}", make)
    return d["pcm"], d["wv"].tobytes()


def c5_file(i: int) -> bytes:
    """File i of the mixed corpus (deterministic in i)."""
    rng = np.random.default_rng(0xC5 * 1_000_003 + i)
    u = rng.random()
    nblk = int(rng.integers(1, 3))
    B = int(rng.integers(4410, 22051))
    frames = nblk * B - int(rng.integers(0, B // 2))
    if u < 0.40:
        x = S.audio_like(frames, 2, 16, seed=i)
        return S.encode_pcm(x, S.EncParams(terms=S.TERMS_DEFAULT if rng.random() < 0.5 else S.TERMS_FAST,
                                           block_samples=B))
    if u < 0.60:
        m = S.audio_like(frames, 1, 16, seed=i)
        if rng.random() < 0.10:
            return S.encode_pcm(np.repeat(m, 2, axis=1), S.EncParams(nch=2, false_stereo=True,
                                                                     terms=S.TERMS_MONO_HIGH[:5], block_samples=B))
        return S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH[:5], block_samples=B))
    if u < 0.85:
        x = S.audio_like(frames, 2, 24, seed=i)
        return S.encode_pcm(x, S.EncParams(terms=S.TERMS_HIGH, bytes_per_sample=3, block_samples=B))
    if u < 0.90:
        m = S.audio_like(frames, 1, 24, seed=i)
        return S.encode_pcm(m, S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH, bytes_per_sample=3, block_samples=B))
    mode = (0, 1, 3)[int(rng.integers(0, 3))]
    dd = S.dsd_random_like(frames, 2, seed=i, density=float(rng.uniform(0.3, 0.7)))
    return S.encode_dsd(dd, S.DsdParams(nch=2, mode=mode, block_samples=B))


# relative device cost per frame of a block of each C5 kind: shard.KIND_COST, the table
# shard.file_cost applies to a file's own header (the same cost in bench.py's split and
# in shard.run_rank)
from wavpackdecoder_amd.shard import KIND_COST as C5_COST  # noqa: E402


def c5_meta(i: int):
    """(kind, frames) of file i of the mixed corpus without encoding it (the same
    draws as c5_file)."""
    rng = np.random.default_rng(0xC5 * 1_000_003 + i)
    u = rng.random()
    nblk = int(rng.integers(1, 3))
    B = int(rng.integers(4410, 22051))
    frames = nblk * B - int(rng.integers(0, B // 2))
    if u < 0.40:
        return "stereo16", frames
    if u < 0.60:
        return "mono16", frames
    if u < 0.85:
        return "stereo24", frames
    if u < 0.90:
        return "mono24", frames
    return "dsd%d" % (0, 1, 3)[int(rng.integers(0, 3))], frames


def c5_cost(i: int) -> float:
    kind, frames = c5_meta(i)
    return C5_COST[kind] * frames


def _c5_range(job):
    lo, hi = job
    return [c5_file(i) for i in range(lo, hi)]


def c5_files(indices, progress: bool = False, workers: int | None = None):
    """The corpus files with the given indices (worker processes; progress lines on
    stderr for long lists)."""
    import sys
    idx = list(indices)
    w = workers if workers is not None else _workers()
    if len(idx) < 64 or w <= 1:
        return [c5_file(i) for i in idx]
    from concurrent.futures import ProcessPoolExecutor
    step = 256
    jobs = [idx[k:k + step] for k in range(0, len(idx), step)]
    out = []
    with ProcessPoolExecutor(max_workers=w) as ex:
        for n, part in enumerate(ex.map(_c5_list, jobs)):
            out += part
            if progress and n % 40 == 39:
                print(f"c5: {len(out)} of {len(idx)} files", file=sys.stderr, flush=True)
    return out


def _c5_list(ids):
    return [c5_file(i) for i in ids]


def c5(nfiles: int, start: int = 0, workers: int | None = None):
    """Files start .. start + nfiles - 1 of the mixed corpus (generated in worker
    processes for large slices; the files do not depend on how they are split)."""
    w = workers if workers is not None else _workers()
    if nfiles < 64 or w <= 1:
        return [c5_file(i) for i in range(start, start + nfiles)]
    from concurrent.futures import ProcessPoolExecutor
    step = max(16, (nfiles + 4 * w - 1) // (4 * w))
    jobs = [(i, min(i + step, start + nfiles)) for i in range(start, start + nfiles, step)]
    with ProcessPoolExecutor(max_workers=w) as ex:
        return [f for part in ex.map(_c5_range, jobs) for f in part]


def c2_shard(rank: int, nblocks: int = 1024, block: int = 22050) -> bytes:
    """A C2-shaped batch for GPU `rank` > 0 of a weak-scaling run (own seeds)."""
    def make():
        pcm = c2_pcm(nblocks, block, seed0=0xC2 + 1_000_003 * rank)
        data = S.encode_pcm(pcm, S.EncParams(terms=S.TERMS_FAST, block_samples=block, joint_stereo=True,
                                             config_flags=0x200))
        return {"wv": np.frombuffer(data, dtype=np.uint8)}
    return _cached(f"c2s-{rank}-{nblocks}-{block}", make)["wv"].tobytes()
