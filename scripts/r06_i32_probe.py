"""Why INT32 lossless (shift-only fixup) blocks run slower in flight than alone: 1,024 x 22,050-frame
16-bit stereo PCM as INT32_DATA with int32 zeros=4, 20 copies in flight on the lane kernel, each
decode's host call timed (a blocking call shows here) -- run under rocprofv3 --kernel-trace --stats."""
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "24")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
from synth import corpora, wvsynth as S  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pcm = corpora.c2_pcm(nb)
x = S.int32_layout(pcm, zeros=4, seed=6)
data = S.encode_pcm_parallel(x, S.EncParams(terms=S.TERMS_DEFAULT, block_samples=22050, joint_stereo=True,
                                            bytes_per_sample=4, int32_zeros=4))
copies = []
for _ in range(20):
    c = DecodeBatch(4096)
    c.set_kernel("lane")
    c.add_files([data])
    c.upload()
    copies.append(c)
for c in copies:
    c.decode()
for c in copies:
    c.sync()
calls = []
t = time.perf_counter()
for k in range(40):
    t0 = time.perf_counter()
    copies[k % 20].decode()
    calls.append(time.perf_counter() - t0)
for c in copies:
    c.sync()
dt = time.perf_counter() - t
copies[0].download()
st = copies[0].block_status()
print(json.dumps({"Mframes_per_s_inflight": round(copies[0].frames * 40 / dt / 1e6, 1),
                  "decode_call_ms": {"mean": round(float(np.mean(calls)) * 1e3, 3),
                                     "max": round(float(np.max(calls)) * 1e3, 3)},
                  "lane_groups": copies[0].lane_groups(),
                  "redone": None if st is None else int(np.count_nonzero(np.asarray(st) & 0x200))}))
for c in copies:
    c.close()
