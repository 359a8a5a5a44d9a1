"""The limit-check sweep as per-account walkers (k_flow.h fl_walk) against the oracle, and against
round 2's one-wave window sweep (TBGPU_CONFIG_SWEEP_WINDOW) on the same inputs.

* Mixed limit flags: debits_must_not_exceed_credits AND credits_must_not_exceed_debits accounts
  among a few hot accounts, so many units carry two open checks (a debits-limited debit account and
  a credits-limited credit account): the walkers' paired-verdict protocol (b_vw), Y legs waiting on
  other accounts' checks, failures on either side in the reference's order (:863-864).
* The adversarial C3 (tests/harness/configs.py "c3h": the hottest Zipf account limited too): one
  heavy segment with most of the pass's undecided checks on a wave of its own."""
import numpy as np
import pytest

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.test_gpu_differential import assert_same_state
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, CreateTransferResult

pytestmark = pytest.mark.gpu

AF_DEBITS_MUST_NOT_EXCEED_CREDITS = 1 << 1
AF_CREDITS_MUST_NOT_EXCEED_DEBITS = 1 << 2


def mixed_limits(n_acc, n_xfer, seed, wide=False):
    rng = np.random.default_rng(seed)
    acc = np.zeros(n_acc, dtype=ACCOUNT_DTYPE)
    acc["id_lo"] = np.arange(1, n_acc + 1)
    acc["ledger"] = 1
    acc["code"] = 1
    kind = np.arange(n_acc) % 4  # 0, 1: free; 2: debits-limited; 3: credits-limited
    acc["flags"][kind == 2] = AF_DEBITS_MUST_NOT_EXCEED_CREDITS
    acc["flags"][kind == 3] = AF_CREDITS_MUST_NOT_EXCEED_DEBITS
    # Zipf-skewed accounts: a few carry most of the legs, so their balances hover at the limits.
    w = 1.0 / np.arange(1, n_acc + 1) ** 1.1
    w /= w.sum()
    perm = rng.permutation(n_acc)
    dr = perm[rng.choice(n_acc, n_xfer, p=w)]
    cr = perm[rng.choice(n_acc, n_xfer, p=w)]
    clash = dr == cr
    cr[clash] = (cr[clash] + 1) % n_acc
    x = np.zeros(n_xfer, dtype=TRANSFER_DTYPE)
    x["id_lo"] = np.arange(1, n_xfer + 1) + 10**9
    x["debit_account_id_lo"] = dr + 1
    x["credit_account_id_lo"] = cr + 1
    x["amount_lo"] = rng.integers(1, 1000, n_xfer)
    if wide:
        # A third of the amounts between 2^22 and 2^40: the walkers' 64-bit runs and bounded walks
        # (fl_walk_run's wide path, pending credits of 2^28 and more carried across windows).
        big = rng.random(n_xfer) < 0.33
        x["amount_lo"][big] = rng.integers(1 << 22, 1 << 40, int(big.sum()))
    x["ledger"] = 1
    x["code"] = 1
    return acc.view(np.uint8), x.view(np.uint8)


def commit_both(engine, accts, xfers, n_acc, n_xfer, gap_every=0):
    batch = 8190
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=gap_every)
    oracle = OracleEngine(n_acc, n_xfer)
    for e in (oracle, engine):
        assert all(r == b"" for r in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))
    for k, (e, a) in enumerate(zip(expected, actual)):
        assert e == a, "reply of prepare %d differs" % k
    assert_same_state(oracle, engine)
    return expected


@pytest.mark.parametrize("bounds_sweep,walk_merge", [("early", 0), ("auto", 0), ("early", 63), ("auto", 63),
                                                     ("window-early", 0)])
@pytest.mark.parametrize("n_acc,n_xfer,pass_batches", [(64, 200_000, 8), (4096, 300_000, 16)])
def test_mixed_limit_flags(bounds_sweep, walk_merge, n_acc, n_xfer, pass_batches, gpu_engine_factory):
    """walk_merge 0: a wave per heavy segment (the default); 63: heavy segments walked merged."""
    accts, xfers = mixed_limits(n_acc, n_xfer, seed=n_acc)
    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pass_batches * 8190,
                                pass_batches_max=pass_batches, bounds_sweep=bounds_sweep)
    engine.walk_merge_max(walk_merge)
    expected = commit_both(engine, accts, xfers, n_acc, n_xfer)
    codes = np.frombuffer(b"".join(expected), dtype=np.uint32).reshape(-1, 2)[:, 1]
    assert (codes == CreateTransferResult.exceeds_credits).any() and (codes == CreateTransferResult.exceeds_debits).any()
    st = engine.stats()
    assert st["bounds_passes"] == st["flow_passes"] > 0 and st["bounds_abandoned"] == 0
    if bounds_sweep != "auto":
        assert st["bounds_swept"] > 0


@pytest.mark.parametrize("bounds_sweep,walk_merge", [("auto", 0), ("auto", 63), ("window", 0)])
def test_c3_hot_limited(bounds_sweep, walk_merge, gpu_engine_factory):
    n_acc, n_xfer, pb = 1_000_000, 2_000_000, 64
    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * 8190,
                                pass_batches_max=pb, bounds_sweep=bounds_sweep)
    engine.walk_merge_max(walk_merge)
    accts, xfers = generate(engine, "c3h", n_acc, n_xfer, seed=42)
    expected = commit_both(engine, accts, xfers, n_acc, n_xfer, SETTINGS["c3h"]["gap_every"])
    assert sum(len(r) for r in expected) > 0
    st = engine.stats()
    assert st["bounds_passes"] == st["flow_passes"] > 0 and st["bounds_abandoned"] == 0
    assert st["bounds_swept"] > 10_000  # the hot account's checks hover at its limit


@pytest.mark.parametrize("bounds_sweep", ["auto", "early"])
def test_mixed_limit_flags_wide_amounts(bounds_sweep, gpu_engine_factory):
    """Amounts up to 2^40 mixed with small ones: the walkers' 64-bit paths — the in-order walk, the
    bounded walk with pending credits too large for 32 bits, the pending credits a heavy walker
    carries from one window into the next (WalkCarry) — against the oracle."""
    n_acc, n_xfer, pb = 64, 200_000, 8
    accts, xfers = mixed_limits(n_acc, n_xfer, seed=5, wide=True)
    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * 8190,
                                pass_batches_max=pb, bounds_sweep=bounds_sweep)
    engine.walk_merge_max(0)
    expected = commit_both(engine, accts, xfers, n_acc, n_xfer)
    codes = np.frombuffer(b"".join(expected), dtype=np.uint32).reshape(-1, 2)[:, 1]
    assert (codes == CreateTransferResult.exceeds_credits).any() and (codes == CreateTransferResult.exceeds_debits).any()
    st = engine.stats()
    assert st["bounds_passes"] == st["flow_passes"] > 0 and st["bounds_abandoned"] == 0
    if bounds_sweep == "early":
        assert st["bounds_swept"] > 0 and st["walk_heavy"] > 0  # heavy segments (a wave each) walked
