"""GPU vs oracle on the BASELINE.json workload shapes at reduced size (C2 uniform; C3 Zipf s=1.2
with 10% debits_must_not_exceed_credits accounts funded by a bank account; C4 linked chains,
pending transfers with timeouts, post/void of earlier transfers across expiry gaps, balancing).
Inputs come from the engine's device generator; both sides commit identical prepares, through
multi-prepare device passes.  Bit-exact: replies, accounts, transfers, posted groove,
commit_timestamp."""
import numpy as np
import pytest

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.test_gpu_differential import assert_same_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config,n_accounts,n_transfers,pass_batches", [
    ("c2", 20_000, 200_000, 8),
    ("c3", 20_000, 200_000, 8),
    ("c3", 2_000, 100_000, 16),   # hotter: long per-account segments, many exceeds_credits
    ("c4", 20_000, 200_000, 8),
    ("c4", 1_000, 100_000, 16),   # dense two-phase traffic per account
    # BASELINE sizes of accounts, 2M transfers, the bench's 64-prepare passes (4 passes)
    ("c3", 1_000_000, 2_000_000, 64),
    ("c4", 1_000_000, 2_000_000, 64),
    ("c4", 1_000_000, 2_100_000, 128),  # the bench's C4 chunk (bench.py CHUNK_PREPARES)
])
def test_config_parity(config, n_accounts, n_transfers, pass_batches, gpu_engine_factory, bounds_sweep="auto"):
    batch = 8190
    engine = gpu_engine_factory(accounts_max=n_accounts, transfers_max=n_transfers,
                                pass_events_max=pass_batches * batch, pass_batches_max=pass_batches,
                                bounds_sweep=bounds_sweep)
    accts, xfers = generate(engine, config, n_accounts, n_transfers, seed=7)
    a_lens = batches(n_accounts, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_lens = batches(n_transfers, batch)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[config]["gap_every"])

    oracle = OracleEngine(n_accounts, n_transfers)
    for e in (oracle, engine):
        assert all(r == b"" for r in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))
    for k, (e, a) in enumerate(zip(expected, actual)):
        assert e == a, "reply of prepare %d differs" % k
    assert_same_state(oracle, engine)
    if config != "c2":  # the shape really exercises the dependent paths, on the parallel flow path
        st = engine.stats()
        assert st["dependent_events"] > 0 and st["flow_passes"] > 0
        assert st["flow_units"] + st["bounds_units"] > 0
        assert sum(len(r) for r in expected) > 0
    if config == "c3":  # limit checks only: decided by the bounds scans (k_flow.h fl_bounds)
        st = engine.stats()
        if bounds_sweep == "off":
            assert st["bounds_swept"] == 0
        else:  # every pass decided by rounds + sweep, never the ordered run
            assert st["bounds_passes"] == st["flow_passes"] and st["bounds_abandoned"] == 0
        if bounds_sweep == "early":
            assert st["bounds_swept"] > 0


@pytest.mark.parametrize("bounds_sweep", ["early", "off"])
@pytest.mark.parametrize("n_accounts,n_transfers,pass_batches", [(20_000, 200_000, 8), (2_000, 100_000, 16)])
def test_c3_sweep_modes(bounds_sweep, n_accounts, n_transfers, pass_batches, gpu_engine_factory):
    """The limit checks decided by the in-order sweep right after the first scan round, and by
    rounds alone (else the ordered run): the same bytes as the oracle either way."""
    test_config_parity("c3", n_accounts, n_transfers, pass_batches, gpu_engine_factory, bounds_sweep)


def test_c3_sweep_u64_path(gpu_engine_factory):
    """The sweep's u64 X/Y form: one transfer of 2^63 + 12345 in the first prepare pushes the
    certificate's bound past 2^63 (no signed slack), while bound + S stays below 2^64 (the bounds
    still apply); every later pass sweeps in the u64 form.  Same bytes as the oracle."""
    n_accounts, n_transfers, pass_batches, batch = 20_000, 200_000, 8, 8190
    engine = gpu_engine_factory(accounts_max=n_accounts, transfers_max=n_transfers,
                                pass_events_max=pass_batches * batch, pass_batches_max=pass_batches,
                                bounds_sweep="early")
    accts, xfers = generate(engine, "c3", n_accounts, n_transfers, seed=13)
    xfers = xfers.copy()
    xfers[48:56] = np.frombuffer(np.uint64(2**63 + 12345).tobytes(), dtype=np.uint8)  # transfer 0's amount
    xfers[56:64] = 0
    a_lens, x_lens = batches(n_accounts, batch), batches(n_transfers, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_accounts, n_transfers)
    for e in (oracle, engine):
        assert all(r == b"" for r in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))
    assert actual == expected
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["bounds_swept"] > 0 and st["bounds_passes"] > 0 and st["sweep_u64_passes"] > 0
