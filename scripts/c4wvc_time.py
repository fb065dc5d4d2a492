"""Six decodes of the C4 + .wvc batch on the .wvc lane kernel and nothing else (no
verification): a short program for rocprofv3 kernel traces of experiment builds."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from synth import corpora  # noqa: E402
from wavpackdecoder_amd.api import DecodeBatch  # noqa: E402

wv, wvc, _ = corpora.c4_wvc()
b = DecodeBatch(4096)
b.set_kernel("lane")
b.add_file(wv, wvc=wvc)
b.upload()
for _ in range(6):
    b.decode()
b.sync()
print("done")
