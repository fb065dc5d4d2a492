"""bench.py's multi-rank layout on CPU (gloo): `python bench.py --gpus 2` spawns
its own two rank processes (the parent touches no GPU), WORLD_SIZE must agree
with --gpus, and the host reductions (max/sum/gather) see every rank."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=e)


@pytest.mark.timeout(300)
def test_spawn_two_ranks_gloo():
    r = _run(["--gpus", "2", "--selftest-dist"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    d = lines[0]
    assert d["n_gpus"] == 2 and d["sum"] == 3.0 and d["max"] == 1.0 and d["gathered"] == [0.0, 11.0]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--selftest-dist"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_single_rank_selftest():
    r = _run(["--selftest-dist"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
