"""GPU: the routes the environment knobs select (read once per process, so each case runs
in a child process), against the oracle bit for bit:

* WVG_LANE_HIGH16=ct -- WavPack's 16-term lists on their compile-time lane instantiations
  (the default runs them on the run-time list pipeline, wv_pcm_lane_rt3);
* WVG_DSD_STREAM=1 -- a mixed batch's DSD groups on a second stream of its own while other
  batches of the context run (batches in flight together, C5-style files);
* the default own-stream policy -- a batch's launch groups on up to three streams of its own
  while others run, as far as the hardware-queue budget (GPU_MAX_HW_QUEUES) leaves each batch
  in flight -- and WVG_DSD_STREAM=0, which keeps every group on the batch's one stream.
The routes are read from the decodes' WVG_DECODE_LOG lines (streams taken, own streams)."""
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
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    # WVG_DECODE_LOG=1: "wvg decode <p>: groups G, others running R, streams S, own O, auto A"
    d["decodes"] = []
    for ln in r.stderr.splitlines():
        if ln.startswith("wvg decode "):
            kv = dict(x.strip().rsplit(" ", 1) for x in ln.split(":", 1)[1].split(","))
            d["decodes"].append({k: int(v) for k, v in kv.items()})
    return d


@pytest.mark.timeout(300)
def test_high16_compile_time_route():
    d = _child("high16", {"WVG_LANE_HIGH16": "ct"})
    assert d["compared"] == d["files"] and d["frames"] == 6 * 20000 and d["lane_groups"] != 0
    assert d["mismatches"] == 0


@pytest.mark.timeout(300)
def test_dsd_own_stream_route():
    d = _child("c5", {"WVG_DSD_STREAM": "1", "WVG_DECODE_LOG": "1"})
    assert d["compared"] == d["files"] * d["copies"] and d["frames"] > 0
    assert d["mismatches"] == 0
    # the route was taken: a decode that found others running, on two streams of its own
    assert any(x["others running"] >= 1 and x["own"] == 1 and x["streams"] == 2 for x in d["decodes"]), d["decodes"]


@pytest.mark.timeout(300)
def test_own_streams_queue_budget_route():
    """The default policy: with 24 hardware queues and 3 batches in flight each decode that
    finds the others running takes 3 streams of its own (24 / 3 >= kLanes); with 4 queues
    (HIP's default) it keeps one."""
    d = _child("c5", {"GPU_MAX_HW_QUEUES": "24", "WVG_DECODE_LOG": "1"})
    assert d["mismatches"] == 0 and d["compared"] == d["files"] * d["copies"]
    assert any(x["others running"] >= 1 and x["own"] == 1 and x["streams"] == 3 for x in d["decodes"]), d["decodes"]
    d = _child("c5", {"GPU_MAX_HW_QUEUES": "4", "WVG_DECODE_LOG": "1"})
    assert d["mismatches"] == 0
    run = [x for x in d["decodes"] if x["others running"] >= 1]
    assert run and all(x["streams"] <= max(1, 4 // (x["others running"] + 1)) for x in run), d["decodes"]
    d = _child("c5", {"GPU_MAX_HW_QUEUES": "24", "WVG_DSD_STREAM": "0", "WVG_DECODE_LOG": "1"})
    assert d["mismatches"] == 0
    run = [x for x in d["decodes"] if x["others running"] >= 1]
    assert run and all(x["streams"] == 1 and x["own"] == 0 for x in run), d["decodes"]
