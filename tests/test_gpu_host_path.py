"""The replica's call pattern on the GPU: one prepare per tbgpu_commit with the body inside host
memory registered once (tbgpu_register_host, the message pool), so kernel 1 reads it over PCIe and
writes it through to HBM.  Bit-exact against the oracle, like tests/test_gpu_differential.py."""
import ctypes

import numpy as np
import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import make_scenario, run_oracle
from tests.test_gpu_differential import CONFIGS, assert_same_state
from tigerbeetle_amd import _lib

pytestmark = pytest.mark.gpu


class RegisteredPool:
    """All prepare bodies of a scenario back to back in one registered buffer."""

    def __init__(self, engine, sc):
        bodies = [b"".join(step[3]) for step in sc.steps if step[0] == "commit"]
        self.offsets = np.concatenate([[0], np.cumsum([len(b) for b in bodies])]).astype(np.int64)
        self.buf = np.zeros(max(int(self.offsets[-1]), 4096), dtype=np.uint8)
        for k, b in enumerate(bodies):
            self.buf[self.offsets[k]:self.offsets[k + 1]] = np.frombuffer(b, dtype=np.uint8)
        self.engine = engine
        _lib.check(engine.lib.tbgpu_register_host(engine.h, self.buf.ctypes.data, self.buf.nbytes))

    def close(self):
        _lib.check(self.engine.lib.tbgpu_unregister_host(self.engine.h, self.buf.ctypes.data))


def run_registered(sc, engine):
    pool = RegisteredPool(engine, sc)
    replies, k = [], 0
    try:
        for step in sc.steps:
            if step[0] == "setup":
                engine.set_balances(*step[1:])
                continue
            _, op, ts, _events = step
            n = int(pool.offsets[k + 1] - pool.offsets[k])
            out = ctypes.create_string_buffer(max(n // 128 * 8, 8))
            out_len = ctypes.c_uint32(0)
            src = ctypes.c_void_p(pool.buf.ctypes.data + int(pool.offsets[k])) if n else None
            _lib.check(engine.lib.tbgpu_commit(engine.h, op, ts, src, n, out, len(out), ctypes.byref(out_len)))
            replies.append(out.raw[:out_len.value])
            k += 1
    finally:
        pool.close()
    return replies


@pytest.mark.parametrize("config", ["mixed", "chains", "two_phase", "clean", "big_batches"])
def test_registered_bodies(config, gpu_engine_factory):
    sc = make_scenario(4242 + sum(map(ord, config)), **CONFIGS[config])
    oracle = OracleEngine()
    expected = run_oracle(sc, oracle)
    engine = gpu_engine_factory()
    actual = run_registered(sc, engine)
    assert expected == actual
    assert_same_state(oracle, engine)
