"""AOF replay through the GPU engine (tigerbeetle_amd/aof.py): every reply and the final grooves
equal the oracle's replay of the same file."""
import pytest

from tests.harness.oracle import OracleEngine
from tests.test_aof import scenario_prepares
from tests.test_gpu_differential import CONFIGS, assert_same_state
from tigerbeetle_amd import aof

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config", ["mixed", "two_phase", "chains", "limits", "big_batches"])
def test_aof_replay_gpu(tmp_path, config, gpu_engine_factory):
    _, prepares = scenario_prepares(600 + sum(map(ord, config)), **CONFIGS[config])
    path = tmp_path / "replica.aof"
    aof.write_aof(path, prepares)
    recorded = aof.read_prepares(path)
    oracle, engine = OracleEngine(), gpu_engine_factory()
    assert aof.replay(recorded, engine) == aof.replay(recorded, oracle)
    assert_same_state(oracle, engine)


def test_aof_replay_state_machine(tmp_path):
    """The replica's own call sequence (prepare -> prefetch -> commit(client, op, ...)) through the
    StateMachine mirror, from a file with real vsr checksums."""
    from tigerbeetle_amd.state_machine import Options, StateMachine

    _, prepares = scenario_prepares(611, **CONFIGS["mixed"])
    path = tmp_path / "replica.aof"
    aof.write_aof(path, prepares)
    recorded = aof.read_prepares(path)
    oracle = OracleEngine()
    sm = StateMachine(Options(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64))
    try:
        assert aof.replay(recorded, sm) == aof.replay(recorded, oracle)
        assert sm.commit_timestamp == oracle.commit_timestamp
        assert_same_state(oracle, sm.engine)
    finally:
        sm.deinit()
