"""GPU: the malformed layouts of tests/test_layout_quirks.py (a block whose ints per
frame differ from the file's, FALSE_STEREO with MONO_FLAG, INT32 sent_bits past 32)
decode on the device as the reference does: equal to the host build of the device
core always, and to the oracle unless the reference reads the caller's stale buffer
(ST_NONDET); none is declined (ST_UNSUPPORTED)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.emu import emu as E
from tests.test_layout_quirks import CASES
from wavpackdecoder_amd._lib import WVG_ST_NONDET, WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", ["lane", "two_wave"])
def test_gpu_layout_quirks(kernel):
    from wavpackdecoder_amd.api import DecodeBatch
    for chunk in sorted({c for _, _, c in CASES}):
        cases = [c for c in CASES if c[2] == chunk]
        b = DecodeBatch(chunk)
        b.set_kernel(kernel)
        idx = [b.add_file(d) for _, d, _ in cases]
        b.decode()
        out = b.download()
        res = [b.result(i) for i in idx]
        infos = list(b.infos)
        st = b.block_status()
        b.close()
        assert int(np.count_nonzero(st & 0x20)) == 0
        for (name, data, _), r, info in zip(cases, res, infos):
            n, eout, crc, est = E.decode(data, chunk)
            ref = O.decode_file(data, chunk=chunk)
            assert not (r.status_or & WVG_ST_TIMEOUT), name
            if n == -3:
                assert r.exception == 1 and ref.status == -3, name
                continue
            assert r.exception == 0 and r.frames == n == ref.frames, name
            assert r.crc_errors == crc == ref.crc_errors, name
            got = out[info.out_offset: info.out_offset + len(eout)]
            np.testing.assert_array_equal(got, eout, err_msg=name)
            if not (r.status_or & WVG_ST_NONDET):
                np.testing.assert_array_equal(got, ref.samples, err_msg=name)
