"""GPU: the routes the environment knobs select (read once per process, so each case runs
in a child process), against the oracle bit for bit:

* WVG_LANE_HIGH16=ct -- WavPack's 16-term lists on their compile-time lane instantiations
  (the default runs them on the run-time list pipeline, wv_pcm_lane_rt3);
* WVG_DSD_STREAM=1 -- a mixed batch's DSD groups on a second stream of its own while other
  batches of the context run (batches in flight together, C5-style files)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import json, sys
sys.path.insert(0, ROOT)
import numpy as np
from oracle import oracle as O
from synth import corpora, wvsynth as S
from wavpackdecoder_amd.api import DecodeBatch
case = sys.argv[1]
if case == "high16":
    files = [S.encode_pcm(S.audio_like(20000, 2, 24, seed=700 + k), S.EncParams(terms=S.TERMS_HIGH, block_samples=4000,
                                                                              bytes_per_sample=3)) for k in range(3)]
    files += [S.encode_pcm(S.audio_like(20000, 1, 16, seed=710 + k), S.EncParams(nch=1, terms=S.TERMS_MONO_HIGH,
                                                                               block_samples=3000)) for k in range(3)]
    copies = 1
else:
    files = corpora.c5(200)
    copies = 3
batches = []
for _ in range(copies):
    b = DecodeBatch(4096)
    b.set_kernel("lane")
    b.add_files(files)
    b.upload()
    batches.append(b)
for b in batches:      # issued back to back: the later ones find the earlier running
    b.decode()
for b in batches:
    b.sync()
refs = O.decode_many(files)
bad = compared = frames = 0
for b in batches:
    out = b.download()
    for i, ref in enumerate(refs):
        info = b.infos[i]
        r = b.result(i)
        if ref.status != 0:
            continue
        compared += 1
        frames += r.frames
        got = out[info.out_offset: info.out_offset + ref.frames * ref.nch]
        if r.frames != ref.frames or r.crc_errors != ref.crc_errors or not np.array_equal(got, ref.samples):
            bad += 1
    groups = b.lane_groups()
    b.close()
print(json.dumps({"case": case, "files": len(files), "copies": copies, "compared": compared, "frames": frames,
                  "lane_groups": groups, "mismatches": bad}))
'''


def _child(case, env_extra):
    env = dict(os.environ, **env_extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    code = "ROOT = " + repr(ROOT) + "\n" + _CHILD
    r = subprocess.run([sys.executable, "-c", code, case], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    print(r.stdout[-400:])
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.timeout(300)
def test_high16_compile_time_route():
    d = _child("high16", {"WVG_LANE_HIGH16": "ct"})
    assert d["compared"] == d["files"] and d["frames"] == 6 * 20000 and d["lane_groups"] != 0
    assert d["mismatches"] == 0


@pytest.mark.timeout(300)
def test_dsd_own_stream_route():
    d = _child("c5", {"WVG_DSD_STREAM": "1"})
    assert d["compared"] == d["files"] * d["copies"] and d["frames"] > 0
    assert d["mismatches"] == 0
