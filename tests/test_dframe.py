"""Device-side framing (wv_dframe.h) against the host framing.

The device framer's header walk and sub-block walk are host+device code; here
they run on the host (tests/emu) and must produce, for every file they accept,
exactly the descriptors (byte for byte, padding included) and the FileInfo the
host framing (wv_framing.cpp, itself checked against the oracle) produces with
the deferred metadata values applied.  Files outside the device scope must be
declined (and are framed by the host on the product path).
"""
import pytest

from synth import corpora
from tests import vectors as V
from tests.emu import emu as E
from tests.test_meta_defer import _bases, meta_fuzz

PCM = V.pcm_cases()
DSD = V.dsd_cases()

# the PCM cases WavPack itself writes: every block carries its own state and no wvx stream
EXPECT_DEVICE = {n for n, _, _ in PCM if "wvx" not in n}


def check_same(data: bytes, chunk: int):
    """-> True when the device framer accepted the file (and matched the host), False when it declined."""
    d, info = E.dframe(data, chunk)
    if d is None:
        return False
    ref = E.frame_descs(data, chunk)
    assert len(d) == len(ref), "block count differs"
    for k in range(len(d) // E.DESC_BYTES):
        a, b = d[k * E.DESC_BYTES:(k + 1) * E.DESC_BYTES], ref[k * E.DESC_BYTES:(k + 1) * E.DESC_BYTES]
        if int.from_bytes(a[E.DESC_KIND:E.DESC_KIND + 4], "little") == E.KIND_DSD_FAST:
            # DSD mode 1: the host framing also builds the reference's tables (for the host
            # decode core); the device framer leaves them to the decode kernel, which builds
            # them from the probability data -- dsd_table_off is the only field that differs
            o = E.DESC_DSD_TABLE_OFF
            a, b = a[:o] + a[o + 8:], b[:o] + b[o + 8:]
        if a != b:
            i = next(i for i in range(E.DESC_BYTES) if a[i] != b[i])
            raise AssertionError(f"descriptor {k} differs from the host framing's at byte {i}")
    ri = E.file_info_full(data, chunk)
    diffs = {k: (info[k], ri[k]) for k in info if info[k] != ri[k]}
    assert not diffs, f"FileInfo differs (device, host): {diffs}"
    return True


@pytest.mark.parametrize("name,data,chunk", PCM, ids=[c[0] for c in PCM])
def test_device_framing_equals_host(name, data, chunk):
    accepted = check_same(data, chunk)
    assert accepted == (name in EXPECT_DEVICE), f"{name}: device framing accepted={accepted}"


@pytest.mark.parametrize("chunk", [1, 13, 4096, 22050, 1 << 20])
def test_device_framing_chunk_schedules(chunk):
    data = PCM[0][1]
    assert check_same(data, chunk)


@pytest.mark.parametrize("name,data,chunk", DSD, ids=[c[0] for c in DSD])
def test_dsd_modes_on_device(name, data, chunk):
    """DSD modes 0 (raw bytes), 1 (the probability data; the kernel builds the
    tables) and 3 (rate + filter bytes; the kernel builds the ptable) are framed on
    the device, equal to the host framing; FALSE_STEREO DSD stays with the host"""
    accepted = check_same(data, chunk)
    assert accepted == (name.startswith(("dsd_m0", "dsd_m1", "dsd_m3", "dsd_fast")) and "fs1" not in name), name


def test_odd_files_declined_or_equal():
    """sticky-state files, term-0 lists, dropped blocks, stripped metadata, truncation,
    leading/trailing junk: accepted only when every block still carries its own state
    (then equal to the host framing), declined otherwise"""
    cases = V.sticky_cases() + V.term0_cases()
    base = PCM[2][1]
    spans = V.block_spans(base)
    cases += [("drop1", V.drop_block(base, 1), 4096),
              ("trunc", base[:len(base) - 100], 4096),
              ("junk_head", b"\0" * 40 + base, 4096),
              ("junk_tail", base + b"\0" * 40, 4096),
              ("junk_tail_short", base + b"\0" * 7, 4096),
              ("first_block_only", base[:spans[0][1]], 4096),
              ("empty", b"", 4096),
              ("not_wavpack", b"RIFF" + bytes(200), 4096)]
    must_decline = ("drop1", "trunc", "junk", "first_block_only", "empty", "not_wavpack", "sticky_enc", "_gap",
                    "_e", "_bits", "_all", "wvx")
    for name, data, chunk in cases:
        accepted = check_same(data, chunk)
        if any(t in name for t in must_decline) and not name.endswith("_w") and "_w2" not in name:
            assert not accepted, name
        if name.startswith("term0"):
            assert accepted, name  # read_decorr_terms accepts term 0: an ordinary block


def test_corrupted_streams_declined_or_equal():
    for base in (PCM[0][1], PCM[4][1], PCM[8][1]):
        for seed in range(20):
            check_same(V.corrupt(base, seed), 4096)


@pytest.mark.parametrize("base", range(6))
def test_fuzzed_metadata_declined_or_equal(base):
    data = _bases()[base]
    accepted = 0
    for seed in range(40):
        accepted += check_same(meta_fuzz(data, seed), 4096)
    # base 5 is a version 0x402 hybrid file: its decorr samples reader runs past the
    # sub-block (quirk B-7 with the 4-byte skip), which only the host framing restates
    assert check_same(data, 4096) == (base != 5)


def test_c5_corpus_files():
    n = 0
    for i in range(120):
        kind, _ = corpora.c5_meta(i)
        accepted = check_same(corpora.c5_file(i), 4096)
        assert accepted, (i, kind)  # every kind of the corpus, DSD mode 1 included
        n += accepted
    assert n == 120
