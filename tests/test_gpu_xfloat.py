"""GPU: exact float output (WVG_OPEN_EXACT_FLOAT, SURVEY §8f-4, beyond the
reference; parity = round trip to the encoder's float input, see
test_xfloat.py), for .wv files with their wvx stream and hybrid files with a
.wvc; the same files opened without the flag decode exactly as the oracle."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.test_xfloat import CASES, EXACT, _bits
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,wv,wvc,x,chunk", CASES, ids=[c[0] for c in CASES])
def test_gpu_xfloat_roundtrip(gpu_batch_cls, name, wv, wvc, x, chunk):
    b = gpu_batch_cls(chunk)
    i = b.add_file(wv, open_flags=EXACT, wvc=wvc)
    j = b.add_file(wv)  # the reference's decode: 24-bit integers
    b.decode()
    out = b.download()
    ri, rj = b.result(i), b.result(j)
    assert not ((ri.status_or | rj.status_or) & WVG_ST_TIMEOUT)
    assert ri.crc_errors == 0 and ri.exception == 0, name
    exact = _bits(x)
    oi, oj = b.infos[i].out_offset, b.infos[j].out_offset
    np.testing.assert_array_equal(out[oi: oi + exact.size], exact, err_msg=name)
    ref = O.decode_file(wv, chunk=chunk)
    assert rj.crc_errors == ref.crc_errors
    np.testing.assert_array_equal(out[oj: oj + ref.samples.size], ref.samples, err_msg=name)
    b.close()
