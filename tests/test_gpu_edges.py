"""Edge cases of the commit path, GPU vs the CPU oracle byte for byte (replies, every account, every
transfer, the posted groove, commit_timestamp), one prepare at a time and as multi-prepare passes.

The shapes follow the limits the reference's own code and tests exercise:
  * empty prepares (execute's loop over zero events, state_machine.zig:612-698) between full ones;
  * the largest batch, 8191 events (constants.batch_max for 1 MiB messages; the table DSL commits
    beyond the test config's batch_max), with every event failing — the largest
    reply, 8 B per event in ascending index (tigerbeetle.zig:109-249);
  * one linked chain over the whole batch, closed (all ok) and open at the batch end (every event
    linked_event_failed, the last linked_event_chain_open, :632-640, :669-676);
  * ragged prepares in one pass (1, 0, 8191, 3, 0, 2 events);
  * extreme ids and amounts: id = maxInt(u128) - 1, amounts at maxInt(u128) and maxInt(u64), the
    u128 overflow checks of create_transfer (:848-861) and the exists comparisons (:886-905);
  * create_accounts at 8191 events with duplicate ids inside the batch (:738-777);
  * amounts summing past 2^128 on fresh accounts (the overflow certificate must not trust a
    saturated sum).
"""
import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import Scenario, run_many, run_oracle
from tigerbeetle_amd.types import AccountFlags as AF, TransferFlags as TF, U128_MAX, pack_account, pack_transfer

U64_MAX = (1 << 64) - 1
BATCH_MAX = 8191
LEDGER = 7


def _accounts(n, first=1, flags=0):
    return [pack_account(id=first + i, ledger=LEDGER, code=1, flags=flags) for i in range(n)]


class _Builder:
    def __init__(self, start_ts=10**12):
        self.sc = Scenario()
        self.ts = start_ts

    def commit(self, op, events):
        # prepare: prepare_timestamp += len (state_machine.zig:336-343); the header timestamp is the
        # last event's, and empty prepares still advance it by one (unit-test rule :1483-1485).
        self.ts += 1 + len(events)
        self.sc.steps.append(("commit", op, self.ts, list(events)))
        return self

    def setup(self, account_id, dp, dpost, cp, cpost):
        self.sc.steps.append(("setup", account_id, dp, dpost, cp, cpost))
        return self


def scenario_empty_prepares():
    b = _Builder()
    b.commit(128, [])
    b.commit(128, _accounts(4))
    b.commit(129, [])
    b.commit(129, [pack_transfer(id=100 + i, debit_account_id=1, credit_account_id=2, amount=5, ledger=LEDGER, code=1)
                   for i in range(3)])
    b.commit(129, [])
    b.commit(128, [])
    return b.sc


def scenario_max_batch_all_failing():
    b = _Builder()
    b.commit(128, _accounts(2))
    evs = []
    for i in range(BATCH_MAX):
        k = i % 4
        if k == 0:
            evs.append(pack_transfer(id=0, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1))
        elif k == 1:
            evs.append(pack_transfer(id=1000 + i, debit_account_id=1, credit_account_id=1, amount=1, ledger=LEDGER, code=1))
        elif k == 2:
            evs.append(pack_transfer(id=1000 + i, debit_account_id=1, credit_account_id=99, amount=1, ledger=LEDGER, code=1))
        else:
            evs.append(pack_transfer(id=1000 + i, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER + 1,
                                     code=1))
    b.commit(129, evs)
    # max-size create_accounts with every event failing too (reserved field / zero ledger / id 0)
    b.commit(128, [pack_account(id=0 if i % 3 == 0 else 10**6 + i, ledger=LEDGER if i % 3 != 1 else 0, code=1,
                                reserved=1 if i % 3 == 2 else 0) for i in range(BATCH_MAX)])
    return b.sc


def scenario_whole_batch_chains():
    b = _Builder()
    b.commit(128, _accounts(8))
    ok_chain = [pack_transfer(id=10 + i, debit_account_id=1 + i % 8, credit_account_id=1 + (i + 1) % 8, amount=1 + i % 5,
                              ledger=LEDGER, code=1, flags=TF.linked if i < BATCH_MAX - 1 else 0)
                for i in range(BATCH_MAX)]
    b.commit(129, ok_chain)
    open_chain = [pack_transfer(id=10**6 + i, debit_account_id=1 + i % 8, credit_account_id=1 + (i + 3) % 8, amount=2,
                                ledger=LEDGER, code=1, flags=TF.linked) for i in range(BATCH_MAX)]
    b.commit(129, open_chain)
    # the same ids again: one chain that fails at its middle event (exists) rolls everything back
    mid = BATCH_MAX // 2
    retry = [pack_transfer(id=10**7 + i if i != mid else 10 + 5, debit_account_id=1 + i % 8,
                           credit_account_id=1 + (i + 1) % 8, amount=3, ledger=LEDGER, code=1,
                           flags=TF.linked if i < BATCH_MAX - 1 else 0) for i in range(BATCH_MAX)]
    b.commit(129, retry)
    return b.sc


def scenario_ragged_pass():
    b = _Builder()
    b.commit(128, _accounts(16))
    k = [0]

    def tr(n):
        out = []
        for _ in range(n):
            i = k[0]
            k[0] += 1
            out.append(pack_transfer(id=5000 + i, debit_account_id=1 + i % 16, credit_account_id=1 + (i * 7 + 3) % 16
                                     if (i * 7 + 3) % 16 != i % 16 else 1 + (i + 1) % 16,
                                     amount=1 + i % 9, ledger=LEDGER, code=1,
                                     flags=TF.pending if i % 11 == 0 else 0, timeout=5 if i % 11 == 0 else 0))
        return out

    for n in (1, 0, BATCH_MAX, 3, 0, 2):
        b.commit(129, tr(n))
    return b.sc


def scenario_extreme_values():
    big = U128_MAX - 1
    b = _Builder()
    b.commit(128, [pack_account(id=big, ledger=LEDGER, code=1), pack_account(id=big - 1, ledger=LEDGER, code=1),
                   pack_account(id=1, ledger=LEDGER, code=1), pack_account(id=2, ledger=LEDGER, code=1),
                   pack_account(id=U128_MAX, ledger=LEDGER, code=1), pack_account(id=0, ledger=LEDGER, code=1)])
    b.setup(1, 0, U128_MAX - 10, 0, 0)
    b.setup(2, 0, 0, 0, U64_MAX)
    evs = [
        pack_transfer(id=big, debit_account_id=big, credit_account_id=big - 1, amount=U128_MAX, ledger=LEDGER, code=1),
        pack_transfer(id=big - 1, debit_account_id=big, credit_account_id=big - 1, amount=1, ledger=LEDGER, code=1),
        pack_transfer(id=7, debit_account_id=1, credit_account_id=2, amount=11, ledger=LEDGER, code=1),  # dpost overflow
        pack_transfer(id=8, debit_account_id=1, credit_account_id=2, amount=10, ledger=LEDGER, code=1),
        pack_transfer(id=9, debit_account_id=2, credit_account_id=1, amount=U64_MAX, ledger=LEDGER, code=1),
        pack_transfer(id=10, debit_account_id=big - 1, credit_account_id=big, amount=U128_MAX, ledger=LEDGER, code=1,
                      flags=TF.pending, timeout=U64_MAX >> 32),
        pack_transfer(id=U128_MAX, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1),
        pack_transfer(id=11, debit_account_id=U128_MAX, credit_account_id=2, amount=1, ledger=LEDGER, code=1),
        pack_transfer(id=12, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1,
                      user_data_128=U128_MAX, user_data_64=U64_MAX, user_data_32=(1 << 32) - 1),
    ]
    b.commit(129, evs)
    # exists with different fields against the extreme records
    b.commit(129, [
        pack_transfer(id=big - 1, debit_account_id=big, credit_account_id=big - 1, amount=2, ledger=LEDGER, code=1),
        pack_transfer(id=12, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1,
                      user_data_128=U128_MAX, user_data_64=U64_MAX, user_data_32=(1 << 32) - 2),
        pack_transfer(id=12, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1,
                      user_data_128=U128_MAX, user_data_64=U64_MAX, user_data_32=(1 << 32) - 1),
        pack_transfer(id=13, pending_id=10, amount=0, flags=TF.post_pending_transfer),
    ])
    return b.sc


def scenario_huge_amounts_fresh_accounts():
    """Balances start at zero (the engine's bound is 0) and the pass's amounts sum past 2^128: the
    saturated sum must not certify the pass (overflows_debits_posted / _credits_posted, :848-861)."""
    b = _Builder()
    b.commit(128, _accounts(4))
    half = 1 << 127
    b.commit(129, [
        pack_transfer(id=1, debit_account_id=1, credit_account_id=2, amount=half, ledger=LEDGER, code=1),
        pack_transfer(id=2, debit_account_id=1, credit_account_id=3, amount=half, ledger=LEDGER, code=1),
        pack_transfer(id=3, debit_account_id=4, credit_account_id=2, amount=half, ledger=LEDGER, code=1),
        pack_transfer(id=4, debit_account_id=3, credit_account_id=4, amount=U128_MAX, ledger=LEDGER, code=1),
        pack_transfer(id=5, debit_account_id=3, credit_account_id=4, amount=1, ledger=LEDGER, code=1),
        pack_transfer(id=6, debit_account_id=2, credit_account_id=1, amount=half - 1, ledger=LEDGER, code=1,
                      flags=TF.pending, timeout=1),
    ])
    return b.sc


def scenario_accounts_duplicates():
    b = _Builder()
    evs = []
    for i in range(BATCH_MAX):
        aid = 1 + (i % 2000)  # every id repeats ~4 times inside the batch
        flags = AF.linked if (i % 97 == 5 and i < BATCH_MAX - 1) else 0
        evs.append(pack_account(id=aid, ledger=LEDGER + (i % 3 == 0 and i >= 2000), code=1 + (i >= 4000), flags=flags,
                                user_data_64=i // 2000))
    b.commit(128, evs)
    b.commit(128, _accounts(10, first=1995))
    return b.sc


SCENARIOS = {
    "empty_prepares": scenario_empty_prepares,
    "max_batch_all_failing": scenario_max_batch_all_failing,
    "whole_batch_chains": scenario_whole_batch_chains,
    "ragged_pass": scenario_ragged_pass,
    "extreme_values": scenario_extreme_values,
    "accounts_duplicates": scenario_accounts_duplicates,
    "huge_amounts_fresh_accounts": scenario_huge_amounts_fresh_accounts,
}


def _state(engine):
    return (engine.export_accounts().tobytes(), engine.export_transfers().tobytes(), engine.export_posted().tobytes(),
            engine.commit_timestamp)


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_oracle_runs_edge_scenarios(name):
    """CPU: the scenarios are well-formed and the oracle answers them (non-trivial replies)."""
    sc = SCENARIOS[name]()
    replies = run_oracle(sc, OracleEngine())
    assert len(replies) == sum(1 for s in sc.steps if s[0] == "commit")
    if name == "max_batch_all_failing":
        assert len(replies[1]) == 8 * BATCH_MAX and len(replies[2]) == 8 * BATCH_MAX
    if name == "whole_batch_chains":
        assert replies[1] == b"" and len(replies[2]) == 8 * BATCH_MAX and len(replies[3]) == 8 * BATCH_MAX


@pytest.mark.gpu
@pytest.mark.parametrize("many", [False, True], ids=["commit", "commit_many"])
@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_gpu_edges(name, many, gpu_engine_factory):
    sc = SCENARIOS[name]()
    oracle = OracleEngine()
    expected = run_oracle(sc, oracle)
    engine = gpu_engine_factory(accounts_max=8192, transfers_max=1 << 16, pass_events_max=8192 * 8, pass_batches_max=8)
    actual = run_many(sc, engine) if many else run_oracle(sc, engine)
    assert actual == expected
    assert _state(engine) == _state(oracle)


@pytest.mark.gpu
def test_transfer_log_full_is_refused_whole(gpu_engine_factory):
    """Capacity contract: the transfer log is sized at init (every stored transfer
    and every speculative record of a pass takes a position).  A commit that would overflow it is
    refused with INVALID before anything runs — no prepare of the call commits — and the engine
    keeps working for calls that fit."""
    from tigerbeetle_amd._lib import EngineError

    engine = gpu_engine_factory(accounts_max=64, transfers_max=1024, pass_events_max=2048, pass_batches_max=4)
    oracle = OracleEngine()
    b = _Builder().commit(128, _accounts(4))
    first = [pack_transfer(id=100 + i, debit_account_id=1 + i % 4, credit_account_id=1 + (i + 1) % 4, amount=1,
                           ledger=LEDGER, code=1) for i in range(1000)]
    b.commit(129, first)
    assert run_oracle(b.sc, oracle) == run_oracle(b.sc, engine)
    over = [pack_transfer(id=5000 + i, debit_account_id=1, credit_account_id=2, amount=1, ledger=LEDGER, code=1)
            for i in range(100)]
    with pytest.raises(EngineError, match="transfer log full"):
        engine.commit(129, b.ts + 200, b"".join(over))
    from tests.test_gpu_differential import assert_same_state as assert_same
    assert_same(oracle, engine)
    fits = b"".join(over[:20])
    assert engine.commit(129, b.ts + 300, fits) == oracle.commit(129, b.ts + 300, fits)
    assert_same(oracle, engine)
