"""Committed golden fixtures (tests/golden, written by make_golden.py).

The oracle and the host build of the device core must both reproduce the
manifest exactly: SHA-256 of the int32 output, head/tail samples, frames and
crc_errors.  The GPU kernels are checked against the same manifest in
test_gpu_parity.py.
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden
from tests.emu import emu as E

FIX = list(golden.load())


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i4").tobytes()).hexdigest()


@pytest.mark.parametrize("name,data,m", FIX, ids=[f[0] for f in FIX])
def test_oracle_reproduces_manifest(name, data, m):
    r = O.decode_file(data, chunk=m["chunk"])
    assert (r.frames, r.nch, r.status, r.crc_errors) == (m["frames"], m["nch"], m["status"], m["crc_errors"])
    assert _sha(r.samples) == m["sha256_int32le"]
    assert r.samples[:64].tolist() == m["head64"]


@pytest.mark.parametrize("name,data,m", FIX, ids=[f[0] for f in FIX])
def test_device_core_reproduces_manifest(name, data, m):
    n, out, crc_errors, st = E.decode(data, m["chunk"])
    assert n == m["frames"] and crc_errors == m["crc_errors"]
    assert _sha(out) == m["sha256_int32le"]
    assert out[-64:].tolist() == m["tail64"]
