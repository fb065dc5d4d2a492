"""GPU: hybrid files with their .wvc correction files decode exactly (SURVEY §8f-4,
beyond the reference; parity unpinned = round trip to the encoder's input, circular
for stereo terms -1/-2 whose rule the encoder shares, see test_wvc.py),
and the same .wv files without the correction decode exactly as the oracle."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.test_wvc import CASES
from wavpackdecoder_amd._lib import WVG_ST_TIMEOUT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,wv,wvc,exact,chunk", CASES, ids=[c[0] for c in CASES])
def test_gpu_wvc_roundtrip(gpu_batch_cls, name, wv, wvc, exact, chunk):
    b = gpu_batch_cls(chunk)
    i = b.add_file(wv, wvc=wvc)
    j = b.add_file(wv)  # the same stream without its correction: the reference's lossy decode
    b.decode()
    out = b.download()
    ri, rj = b.result(i), b.result(j)
    assert not ((ri.status_or | rj.status_or) & WVG_ST_TIMEOUT)
    assert ri.crc_errors == 0 and ri.exception == 0, name
    oi, oj = b.infos[i].out_offset, b.infos[j].out_offset
    np.testing.assert_array_equal(out[oi: oi + exact.size], exact, err_msg=name)
    ref = O.decode_file(wv, chunk=chunk)
    assert rj.crc_errors == ref.crc_errors
    np.testing.assert_array_equal(out[oj: oj + ref.samples.size], ref.samples, err_msg=name)
    b.close()


def test_gpu_wvc_c4_corpus():
    """C4's own corpus layout (float32, hybrid + bitrate, default terms {18,18,2,3,-2},
    22,050-frame blocks) with its .wvc: the exact decode equals the oracle's decode of
    the same mantissas encoded losslessly, on every block."""
    from synth import corpora
    from wavpackdecoder_amd.api import DecodeBatch
    wv, wvc, lossless = corpora.c4_wvc(nblocks=24)
    ref = O.decode_file(lossless)
    assert ref.crc_errors == 0
    b = DecodeBatch(4096)
    i = b.add_file(wv, wvc=wvc)
    b.decode()
    out = b.download()
    r = b.result(i)
    assert r.crc_errors == 0 and r.exception == 0 and r.frames == 24 * 22050
    np.testing.assert_array_equal(out[: ref.samples.size], ref.samples)
    b.close()
