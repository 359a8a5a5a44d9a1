"""The C++ host mirror of the reference StateMachine interface (tigerbeetle_amd/host/): it builds
against the C ABI on a machine without a GPU, fails loudly there, and (GPU) replays every golden
table of the reference through tb::StateMachine -> tbgpu_commit."""
import os
import subprocess

import pytest

from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def runner():
    from tigerbeetle_amd import build
    build.build(verbose=False)
    return build.RUNNER


def test_host_mirror_builds(runner):
    assert os.access(runner, os.X_OK)


def test_host_mirror_fails_loudly_without_gpu(runner):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = subprocess.run([runner, os.path.join(GOLDEN, "state_machine_tables.txt")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 255 and "init failed" in r.stderr


@pytest.mark.gpu
def test_host_mirror_golden_tables(runner):
    r = subprocess.run([runner, os.path.join(GOLDEN, "state_machine_tables.txt"), "0"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "18 tables, 0 failed" in r.stdout
