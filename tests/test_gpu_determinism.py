"""The dependence classification is a function of the input, not of scheduling (VERDICT r3 What's
weak #1): on fixed workloads, the engine's dependent-event count equals the host model of its
classification rule (tests/harness/dependence.py), run after run."""
import numpy as np
import pytest

from tests.harness.dependence import dependent_count
from tests.harness.oracle import OracleEngine
from tests.harness.workload import Scenario, make_scenario, run_many, run_oracle
from tests.test_gpu_differential import CONFIGS

pytestmark = pytest.mark.gpu

# (seed, scenario knobs): the smoke() workload first.
CASES = [(7, dict(p_linked=0.2, p_post_void=0.3, p_pending=0.4))] + [
    (100 + k, CONFIGS[c]) for k, c in enumerate(["mixed", "chains", "two_phase", "limits", "hot_ids"])]


def _split(sc):
    accts, xfers = Scenario(), Scenario()
    for st in sc.steps:
        assert st[0] == "commit", "the model assumes no direct balance writes"
        (accts if st[1] == 128 else xfers).steps.append(st)
    return accts, xfers


def _model(sc_accts, sc_xfers):
    oracle = OracleEngine()
    run_oracle(sc_accts, oracle)
    a = oracle.export_accounts()
    accounts = {int(lo) | (int(hi) << 64): (int(f), int(l))
                for lo, hi, f, l in zip(a["id_lo"], a["id_hi"], a["flags"], a["ledger"])}
    return dependent_count([b"".join(st[3]) for st in sc_xfers.steps], accounts)


@pytest.mark.parametrize("seed,knobs", CASES)
def test_dependent_events_equal_the_model(seed, knobs, gpu_engine_factory):
    sc = make_scenario(seed, **knobs)
    sc_a, sc_x = _split(sc)
    expected = _model(sc_a, sc_x)
    counts = []
    for _ in range(3):
        engine = gpu_engine_factory()
        run_many(sc_a, engine)
        before = engine.stats()["dependent_events"]  # cumulative: create_accounts duplicates count too
        run_many(sc_x, engine)  # one commit_many call: one device pass
        counts.append(engine.stats()["dependent_events"] - before)
        engine.close()
    assert counts == [expected] * 3, (counts, expected)


@pytest.mark.parametrize("config", ["overflow", "mixed"])
def test_dependent_events_repeat_without_the_global_certificate(config, gpu_engine_factory):
    """Near-overflow balances (set directly) defeat the global certificate, so every account-touching
    event is checked against its own accounts' pre-pass balances: the count must not depend on which
    workgroups ran first (nothing applies balances while the resolve kernel classifies)."""
    knobs = dict(CONFIGS[config])
    knobs["near_overflow"] = True
    counts, replies = [], []
    for _ in range(3):
        engine = gpu_engine_factory()
        replies.append(run_many(make_scenario(4244, **knobs), engine))
        counts.append(engine.stats()["dependent_events"])
        engine.close()
    assert counts[0] > 0 and counts == [counts[0]] * 3, counts
    assert replies[0] == replies[1] == replies[2]
    oracle = OracleEngine()
    assert run_oracle(make_scenario(4244, **knobs), oracle) == replies[0]
