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


def _decode_wvc(pairs, kernel, chunk=4096):
    from wavpackdecoder_amd.api import DecodeBatch
    b = DecodeBatch(chunk)
    b.set_kernel(kernel)
    idx = [b.add_file(wv, wvc=wvc) for wv, wvc in pairs]
    b.decode()
    out = b.download()
    res = [b.result(i) for i in idx]
    infos = list(b.infos)
    st = b.block_status()
    b.close()
    return out, res, infos, st


def test_gpu_wvc_lane_route():
    """The .wvc lane kernel (wv_lane.h HY == 2: WavPack's default list, hybrid + bitrate,
    stereo, integer or float): every case decodes on the lane route exactly as on the
    generic kernel (the route the two-wave choice takes), and the default-list cases stay
    on the lanes (no hand-back)."""
    from wavpackdecoder_amd._lib import WVG_ST_REDONE
    pairs = [(wv, wvc) for _, wv, wvc, _, _ in CASES]
    o_l, r_l, i_l, st_l = _decode_wvc(pairs, "lane")
    o_w, r_w, i_w, st_w = _decode_wvc(pairs, "two_wave")
    for (name, _, _, exact, _), rl, il, rw, iw in zip(CASES, r_l, i_l, r_w, i_w):
        assert not ((rl.status_or | rw.status_or) & WVG_ST_TIMEOUT), name
        assert rl.crc_errors == rw.crc_errors == 0 and rl.frames == rw.frames, name
        np.testing.assert_array_equal(o_l[il.out_offset: il.out_offset + exact.size], exact, err_msg=name)
        np.testing.assert_array_equal(o_w[iw.out_offset: iw.out_offset + exact.size], exact, err_msg=name)
    assert int(np.count_nonzero(st_l & WVG_ST_REDONE)) == 0


def test_gpu_wvc_c4_full_lanes():
    """C4 + .wvc at its own size (1,024 float hybrid blocks) on the .wvc lane kernel: the
    exact decode equals the oracle's decode of the same mantissas encoded losslessly."""
    from synth import corpora
    from wavpackdecoder_amd._lib import WVG_ST_REDONE
    wv, wvc, lossless = corpora.c4_wvc()
    ref = O.decode_file(lossless)
    assert ref.crc_errors == 0
    out, res, infos, st = _decode_wvc([(wv, wvc)], "lane")
    r = res[0]
    assert r.crc_errors == 0 and r.exception == 0 and r.frames == 1024 * 22050
    np.testing.assert_array_equal(out[: ref.samples.size], ref.samples)
    print("c4+wvc lane hand-backs:", int(np.count_nonzero(st & WVG_ST_REDONE)))


def test_gpu_wvc_lane_corrupted_matches_generic():
    """Corrupted correction streams (and main streams) on the .wvc lane route decode
    exactly as on the generic kernel: CRC errors, mutes and exceptions included (parity
    unpinned: the reference never reads the stream; the generic kernel is the host
    core's twin, tests/test_wvc.py)."""
    from tests import vectors as V
    base = [c for c in CASES if c[0] in ("stereo16_default_br3", "float_hybrid_default_br3")]
    pairs = []
    for k in range(8):
        for _, wv, wvc, _, _ in base:
            pairs.append((wv, V.corrupt(wvc, 600 + k, start=40)))
            pairs.append((V.corrupt(wv, 700 + k, start=150), wvc))
    o_l, r_l, i_l, _ = _decode_wvc(pairs, "lane")
    o_w, r_w, i_w, _ = _decode_wvc(pairs, "two_wave")
    for k, (rl, il, rw, iw) in enumerate(zip(r_l, i_l, r_w, i_w)):
        assert not ((rl.status_or | rw.status_or) & WVG_ST_TIMEOUT), k
        assert (rl.exception, rl.crc_errors) == (rw.exception, rw.crc_errors), k
        if rl.exception:
            continue
        assert rl.frames == rw.frames, k
        n = rl.frames * i_l[k].reduced_channels
        np.testing.assert_array_equal(o_l[il.out_offset: il.out_offset + n], o_w[iw.out_offset: iw.out_offset + n],
                                      err_msg=str(k))
