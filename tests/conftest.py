import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Every stream of the node engine on its own hardware queue, as on N real devices (HIP's default is
# 4 per process, under which a 2-shard node's 7 streams share queues and serialise; round 5's
# sequencer balance race showed only with 8). Set here, before any test module imports torch or
# loads libtbgpu.so, i.e. before HIP reads it. The GPU box exports its own value (4), so it is
# overridden; `TBGPU_TEST_HW_QUEUES=4 pytest ...` runs the old case.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("TBGPU_TEST_HW_QUEUES", "8")


def pytest_report_header(config):
    return "GPU_MAX_HW_QUEUES=%s (set before HIP initialises)" % os.environ.get("GPU_MAX_HW_QUEUES")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running parity sweep")


@pytest.fixture
def gpu_engine_factory():
    """Fresh small engines on cuda:0 (the HIP library must be built; no fallback)."""
    from tigerbeetle_amd.state_machine import Engine, Options

    made = []

    def make(**kw):
        opts = dict(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64)
        opts.update(kw)
        e = Engine(Options(**opts))
        made.append(e)
        return e

    yield make
    for e in made:
        e.close()
