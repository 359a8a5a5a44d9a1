"""GPU vs oracle on seeded random workloads covering every dependency class (duplicate ids,
limit accounts, balancing, two-phase in the same/later prepare, expiry, linked chains, invalid
events, near-overflow balances).  Bit-exact: every reply byte, every account, every transfer, the
posted groove and commit_timestamp."""
import numpy as np
import pytest

from tests.harness.oracle import OracleEngine, OraclePanic
from tests.harness.workload import make_scenario, run_many, run_oracle
from tigerbeetle_amd._lib import EnginePanic

pytestmark = pytest.mark.gpu

CONFIGS = {
    "mixed": dict(),
    "chains": dict(p_linked=0.35, p_invalid=0.08),
    "two_phase": dict(p_pending=0.5, p_post_void=0.4, p_timeout=0.7),
    "limits": dict(p_limit=0.5, p_balancing=0.2, n_accounts=16),
    "hot_ids": dict(id_space=300, p_dup=0.2),
    "clean": dict(p_limit=0, p_linked=0, p_pending=0, p_post_void=0, p_balancing=0, p_dup=0, p_invalid=0,
                  n_accounts=256, batch_len=(500, 2000), id_space=1 << 60),
    "overflow": dict(near_overflow=True, p_limit=0.2, n_accounts=32),
    "huge_amounts": dict(p_huge=0.05, p_limit=0.1, n_accounts=24),
    "big_batches": dict(batch_len=(4000, 8190), n_transfer_batches=4, n_accounts=512, id_space=1 << 20),
}


def assert_same_state(oracle, engine):
    a_o, a_g = oracle.export_accounts(), engine.export_accounts()
    assert len(a_o) == len(a_g)
    assert a_o.tobytes() == a_g.tobytes()
    t_o, t_g = oracle.export_transfers(), engine.export_transfers()
    assert len(t_o) == len(t_g)
    assert t_o.tobytes() == t_g.tobytes()
    assert np.array_equal(oracle.export_posted(), engine.export_posted())
    assert oracle.commit_timestamp == engine.commit_timestamp


def _run(sc, oracle, engine, many):
    try:
        expected = run_oracle(sc, oracle)
    except OraclePanic:
        with pytest.raises(EnginePanic):
            (run_many if many else run_oracle)(sc, engine)
        return
    actual = (run_many if many else run_oracle)(sc, engine)
    assert len(expected) == len(actual)
    for k, (e, a) in enumerate(zip(expected, actual)):
        assert e == a, "reply of prepare %d differs" % k
    assert_same_state(oracle, engine)


@pytest.mark.parametrize("config", sorted(CONFIGS))
@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("many", [False, True], ids=["commit", "commit_many"])
def test_differential(config, seed, many, gpu_engine_factory):
    sc = make_scenario(seed * 7919 + sum(map(ord, config)), **CONFIGS[config])
    engine = gpu_engine_factory()
    if seed != 1:  # seeds 2, 3: the sorted balance legs on every pass (default: passes >= 256K events)
        engine.legs_min_events(0)
    _run(sc, OracleEngine(), engine, many)


def test_small_passes_split_batches(gpu_engine_factory):
    # pass_events_max smaller than the workload: commit_many spans several device passes.
    sc = make_scenario(99, batch_len=(50, 300), n_transfer_batches=12, p_linked=0.2, p_post_void=0.3)
    _run(sc, OracleEngine(), gpu_engine_factory(pass_events_max=8191, pass_batches_max=3), True)
