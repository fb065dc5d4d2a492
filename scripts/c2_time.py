"""Six lane-kernel decodes of the C2 batch and nothing else (no verification): a short
program for rocprofv3 kernel traces of experiment builds (WVG_LIB=...), e.g.
  rocprofv3 --kernel-trace --stats -d out -- python3 scripts/c2_time.py"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from synth import corpora
from wavpackdecoder_amd.api import DecodeBatch
data = corpora.c2()
b = DecodeBatch(4096)
b.set_kernel("lane")
b.add_file(data)
b.upload()
for _ in range(6):
    b.decode()
b.sync()
print("done")
