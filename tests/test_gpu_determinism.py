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


def test_failed_event_that_collides_is_replayed_exactly(gpu_engine_factory):
    """An event that fails the account checks still claims its id (k_validate.h), so a valid event
    with the same id in the same pass collides with it and both are replayed in order (HZ_SELFDEP).
    Both replies must be the oracle's, and the dependent count the host model's."""
    from tigerbeetle_amd.types import pack_account, pack_transfer
    from tests.harness.workload import account_id

    sc = Scenario()
    accts = [pack_account(id=account_id(i), ledger=1 + (i == 3), code=1) for i in range(4)]
    sc.steps.append(("commit", 128, 10**12, accts))
    missing = account_id(99)
    xfer = lambda tid, dr, cr, **kw: pack_transfer(id=tid, debit_account_id=dr, credit_account_id=cr, amount=5,
                                                   ledger=kw.pop("ledger", 1), code=1, **kw)
    batch1 = [
        xfer(100, missing, account_id(1)),            # debit_account_not_found, claims 100
        xfer(100, account_id(0), account_id(1)),      # ok: 100 does not exist yet
        xfer(101, account_id(0), account_id(3)),      # accounts_must_have_the_same_ledger, claims 101
        xfer(101, account_id(0), account_id(2)),      # ok
        xfer(102, account_id(0), account_id(1)),      # ok, claims 102
        xfer(102, missing, account_id(1)),            # debit_account_not_found (account checks come first)
        xfer(103, account_id(0), account_id(1), ledger=2),  # transfer_must_have_the_same_ledger_as_accounts
        xfer(103, account_id(0), account_id(1), ledger=2),  # the same failure again
        xfer(104, account_id(1), missing),            # credit_account_not_found
    ]
    batch2 = [
        xfer(100, account_id(0), account_id(1)),      # exists
        xfer(104, account_id(1), account_id(2)),      # ok (the failed 104 never existed)
        xfer(104, missing, account_id(2)),            # debit_account_not_found before the exists check
    ]
    sc.steps.append(("commit", 129, 10**12 + 100, batch1))
    sc.steps.append(("commit", 129, 10**12 + 200, batch2))
    expected = run_oracle(sc, OracleEngine())
    assert any(expected[1:]), "the scenario must hold failures"
    sc_a, sc_x = _split(sc)
    model = _model(sc_a, sc_x)
    engine = gpu_engine_factory()
    got = run_many(sc_a, engine)
    before = engine.stats()["dependent_events"]
    got += run_many(sc_x, engine)  # both prepares in one device pass
    assert got == expected
    assert engine.stats()["dependent_events"] - before == model > 0
    engine.close()
