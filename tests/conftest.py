"""Shared test setup.

Markers: `gpu` tests run on an MI355X (pytest -m gpu); everything else runs
on CPU (pytest -m "not gpu").  The oracle (oracle/) is the checker only.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def _make(path):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, path)])


@pytest.fixture(scope="session", autouse=True)
def native_test_libs():
    """The CPU-side helpers (oracle, generator, host emulator) build in seconds."""
    _make("oracle")
    _make("synth")
    _make("tests/emu")
    yield


@pytest.fixture(scope="session")
def gpu_batch_cls():
    from wavpackdecoder_amd import api
    return api.DecodeBatch
