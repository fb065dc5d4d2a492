"""GPU: bench.py's multi-rank path with the HIP decode -- `--gpus 2`
spawns two rank processes (children, gloo barrier and max/sum reduces, no collective on
the data path), each decoding its share on the device, rank 0 printing the job line.
The box has one GPU, so both ranks open device 0 (WVG_BENCH_SAME_DEVICE=1); the
driver's N-GPU runs give each rank its own.  C2 (weak scaling: every rank the whole
batch, verified right after the timed region) and a C5 slice (strong scaling: the
files partitioned over the ranks, shard.partition)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args):
    env = dict(os.environ, WVG_BENCH_SAME_DEVICE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + args, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_two_ranks_c2_weak():
    d = _bench(["--steps", "4", "--warmup", "1", "--inflight", "4", "--no-cpu", "--timed-only", "--blocks", "256"])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    v = d["verified"]
    assert v["crc_errors"] == 0 and v["redo_blocks"] == 0 and v["unwritten_blocks"] == 0 and v["pcm_equal"]


@pytest.mark.timeout(300)
def test_bench_two_ranks_c5_strong():
    d = _bench(["--workload", "c5", "--c5-files", "400", "--steps", "2", "--warmup", "1", "--no-cpu"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["value"] > 0
    assert d["config"]["frames_total"] > d["config"]["frames_rank0"] > 0
