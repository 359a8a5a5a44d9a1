"""The parallel ordered fallback (csrc/k_flow.h) against the oracle and against the sequential
replay it replaces: linked chains longer than the planner takes (the in-kernel sequential
fallback), engines whose balances were set directly (sequential replay by design), and the same
BASELINE C4-shaped workload with the flow path on and off (TBGPU_CONFIG_SEQUENTIAL_FALLBACK),
both against the oracle, byte for byte."""
import pytest

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.harness.workload import make_scenario
from tests.test_gpu_differential import _run, assert_same_state

pytestmark = pytest.mark.gpu


def test_long_chains_take_the_sequential_fallback(gpu_engine_factory):
    # Chains of ~30-300 events over limit accounts: dependent as a whole, longer than FLOW_CHAIN_MAX.
    sc = make_scenario(4242, p_linked=0.97, p_limit=0.5, n_accounts=24, batch_len=(150, 400), n_transfer_batches=6,
                       p_invalid=0.01, p_post_void=0.1)
    engine = gpu_engine_factory()
    _run(sc, OracleEngine(), engine, True)
    assert engine.stats()["dependent_events"] > 0


def test_set_balances_keeps_sequential_replay(gpu_engine_factory):
    sc = make_scenario(77, near_overflow=True, p_limit=0.3, n_accounts=32)
    engine = gpu_engine_factory()
    _run(sc, OracleEngine(), engine, True)
    assert engine.stats()["flow_passes"] == 0


def _c4(engine, data, n_accounts=5000, n_transfers=150_000):
    accts, xfers = data
    a_lens = batches(n_accounts, 8190)
    a_ts, t = timestamps(a_lens, 10**12)
    x_lens = batches(n_transfers, 8190)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS["c4"]["gap_every"])
    engine.commit_many(128, a_ts, split(accts, a_lens))
    return engine.commit_many(129, x_ts, split(xfers, x_lens))


def test_flow_equals_sequential_replay(gpu_engine_factory):
    kw = dict(accounts_max=5000, transfers_max=150_000, pass_events_max=8 * 8190, pass_batches_max=8)
    flow = gpu_engine_factory(**kw)
    data = generate(flow, "c4", 5000, 150_000, seed=3)
    got_flow = _c4(flow, data)
    assert flow.stats()["flow_passes"] > 0
    seq = gpu_engine_factory(sequential_fallback=True, **kw)
    got_seq = _c4(seq, data)
    assert seq.stats()["flow_passes"] == 0 and seq.stats()["dependent_events"] > 0
    oracle = OracleEngine(5000, 150_000)
    assert _c4(oracle, data) == got_flow == got_seq
    assert_same_state(oracle, flow)  # same accounts, transfers, posted groove, commit_timestamp
    assert_same_state(oracle, seq)
