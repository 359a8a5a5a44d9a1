"""tb_apply_legs with Zipf-heavy buckets split over workgroups (k_apply.h): one account takes 40 %
of the debit legs and another 10 %, so their buckets hold far more than APPLY_SPLIT_MIN (64K) legs
per 64-prepare pass and are summed in 32K-leg parts by their owners and the extra workgroups, with
atomics.  Replies, balances and records must equal the oracle's byte for byte."""
import numpy as np
import pytest

from tests.harness.configs import batches, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.test_gpu_differential import assert_same_state
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

pytestmark = pytest.mark.gpu


def test_heavy_bucket_split(gpu_engine_factory):
    n_acc, n_xfer, batch, pb = 4096, 1_100_000, 8190, 64
    rng = np.random.default_rng(11)
    acc = np.zeros(n_acc, dtype=ACCOUNT_DTYPE)
    acc["id_lo"] = np.arange(1, n_acc + 1)
    acc["ledger"] = 1
    acc["code"] = 1
    x = np.zeros(n_xfer, dtype=TRANSFER_DTYPE)
    x["id_lo"] = np.arange(1, n_xfer + 1) + 10**9
    r = rng.random(n_xfer)
    dr = rng.integers(1, n_acc + 1, n_xfer)
    dr[r < 0.4] = 1
    dr[(r >= 0.4) & (r < 0.5)] = 2
    cr = rng.integers(1, n_acc + 1, n_xfer)
    clash = cr == dr
    cr[clash] = dr[clash] % n_acc + 1
    x["debit_account_id_lo"] = dr
    x["credit_account_id_lo"] = cr
    x["amount_lo"] = rng.integers(1, 1000, n_xfer)
    x["ledger"] = 1
    x["code"] = 1

    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * batch,
                                pass_batches_max=pb, profile=True)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acc, n_xfer)
    accts, xfers = acc.view(np.uint8), x.view(np.uint8)
    for e in (oracle, engine):
        assert all(rep == b"" for rep in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))
    assert actual == expected
    assert all(rep == b"" for rep in expected)  # every transfer commits: all legs on the legs path
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["dependent_events"] == 0 and st["launches_apply"] > 0


def test_bucket_parts_beyond_the_extra_workgroups(gpu_engine_factory):
    """One 512-prepare pass (4.19M transfers) where account 1 is the debit of 55 % of the events and
    account 2 the credit of 50 %: their buckets hold ~2.3M and ~2.1M legs, 70 and 64 parts of
    APPLY_PART, more extra parts (132) than tb_apply_legs has extra workgroups (APPLY_EXTRA = 64).
    So the first split bucket's owner sums part 0 plus the parts left over after the extras, several
    ranges into one LDS table (tb_gather_range's hot-word count trick over each range), and the
    second split bucket's owner gets no extra workgroup at all and sums every part itself."""
    n_acc, batch, pb = 4096, 8190, 512
    n_xfer = pb * batch
    rng = np.random.default_rng(23)
    acc = np.zeros(n_acc, dtype=ACCOUNT_DTYPE)
    acc["id_lo"] = np.arange(1, n_acc + 1)
    acc["ledger"] = 1
    acc["code"] = 1
    x = np.zeros(n_xfer, dtype=TRANSFER_DTYPE)
    x["id_lo"] = np.arange(1, n_xfer + 1) + 10**9
    dr = rng.integers(1, n_acc + 1, n_xfer)
    dr[rng.random(n_xfer) < 0.55] = 1
    cr = rng.integers(1, n_acc + 1, n_xfer)
    cr[rng.random(n_xfer) < 0.50] = 2
    clash = cr == dr
    cr[clash] = dr[clash] % n_acc + 1
    x["debit_account_id_lo"] = dr
    x["credit_account_id_lo"] = cr
    x["amount_lo"] = rng.integers(1, 1 << 20, n_xfer)
    x["ledger"] = 1
    x["code"] = 1

    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * batch,
                                pass_batches_max=pb, profile=True)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acc, n_xfer)
    accts, xfers = acc.view(np.uint8), x.view(np.uint8)
    for e in (oracle, engine):
        assert all(rep == b"" for rep in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))
    assert actual == expected
    assert all(rep == b"" for rep in expected)
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["passes"] >= 1 and st["dependent_events"] == 0 and st["launches_apply"] == st["passes"] - 1
