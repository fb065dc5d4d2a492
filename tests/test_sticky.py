"""Sticky decode state (Appendix B-8, UnpackUtils.cs:24-68): blocks that do not
re-send their decorrelation weights / samples, entropy medians, hybrid profile
or bitstream, and blocks read without unpack_init (a dropped block ahead of
them, WavPackUtils.cs:219-251), continue the state the previous decode left.

The framing groups them into chains (wv_framing.cpp chain_blocks) that the
device decodes in order, carrying PcmState (wv_decode_core.h).  Here the host
build of the same code (tests/emu) is checked against the oracle, and the
encoder's sticky_passes files -- correct only when the passes continue -- are
checked against their input PCM (a truth independent of the oracle).  The GPU
side is test_gpu_parity.py::test_sticky_state_chains."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import vectors as V
from tests.emu import emu as E

ST_UNSUPPORTED, ST_NONDET = 0x20, 0x80


@pytest.mark.parametrize("case", V.sticky_cases(), ids=lambda c: c[0])
def test_chain_matches_oracle(case):
    name, data, chunk = case
    r = O.decode_file(data, chunk=chunk)
    n, out, crc, st = E.decode(data, chunk)
    assert not (st & ST_UNSUPPORTED), name  # every block is decoded, none left to the host
    if r.status != 0:
        assert n == r.status, name
        return
    assert n == r.frames and crc == r.crc_errors, name
    if not (st & ST_NONDET):
        np.testing.assert_array_equal(out, r.samples, err_msg=name)


@pytest.mark.parametrize("case", V.sticky_clean_cases(), ids=lambda c: c[0])
def test_sticky_passes_lossless(case):
    name, data, chunk, pcm = case
    n, out, crc, st = E.decode(data, chunk)
    assert n == pcm.shape[0] and crc == 0 and st & 0xFF == 0x01, name  # CRC checked, no error
    np.testing.assert_array_equal(out, pcm.reshape(-1), err_msg=name)


def _descs(data, chunk=4096):
    from tests.test_meta_defer import DESC_BYTES, frame
    raw, n, _ = frame(data, True, -1, chunk)
    # BlockDesc: inherit, inherit_passes, chain_len (wv_desc.h)
    o = E.DESC_INHERIT
    return [np.frombuffer(raw[k * DESC_BYTES + o:k * DESC_BYTES + o + 12], np.uint32) for k in range(n)]


def test_chain_layout():
    name, data, chunk, _ = V.sticky_clean_cases()[0]
    tails = _descs(data, chunk)
    assert tails[0][2] == len(tails) and tails[0][0] == 0  # one chain from the first block
    for t in tails[1:]:
        assert t[0] & 0x80000000 and t[2] == 0  # INH_MEMBER
        assert t[1] & 0xFFFF0000 and t[1] & 0xFFFF  # samples and weights continue
    # a well-formed file has no chains
    plain = V.pcm_cases()[0][1]
    assert all(t[0] == 0 and t[1] == 0 and t[2] == 0 for t in _descs(plain))


@pytest.mark.parametrize("case", V.term0_cases(), ids=lambda c: c[0])
def test_stereo_term0_matches_oracle(case):
    name, data, chunk = case
    r = O.decode_file(data, chunk=chunk)
    n, out, crc, st = E.decode(data, chunk)
    assert not (st & ST_UNSUPPORTED), name
    if r.status != 0:
        assert n == r.status, name
        return
    assert n == r.frames and crc == r.crc_errors, name
    if not (st & ST_NONDET):
        np.testing.assert_array_equal(out, r.samples, err_msg=name)


@pytest.mark.parametrize("case", V.dsd_sticky_cases(), ids=lambda c: c[0])
def test_dsd_chain_matches_oracle(case):
    """DSD chains (decode_dsd_chained): blocks without ID_DSD_BLOCK, or read without
    unpack_init, continue the DSD state -- formerly declined (ST_UNSUPPORTED).  Samples
    are compared unless the reference reads its caller's stale buffer (ST_NONDET: a
    continuing mode-0 block past its data, a failed mode-1 symbol)."""
    name, data, chunk = case
    r = O.decode_file(data, chunk=chunk)
    n, out, crc, st = E.decode(data, chunk)
    assert not (st & ST_UNSUPPORTED), name
    if r.status != 0:
        assert n == r.status, name
        return
    assert n == r.frames and crc == r.crc_errors, name
    if not (st & ST_NONDET):
        np.testing.assert_array_equal(out, r.samples, err_msg=name)


def test_dsd_chain_cases_cover_kinds():
    """the DSD chain cases compare samples in every mode (not all NONDET)"""
    seen = set()
    for name, data, chunk in V.dsd_sticky_cases():
        n, out, crc, st = E.decode(data, chunk)
        if not (st & ST_NONDET) and n > 0:
            seen.add(name.split("_")[2])
    assert seen == {"m0", "m1", "m3"} or seen >= {"m1", "m3"}
