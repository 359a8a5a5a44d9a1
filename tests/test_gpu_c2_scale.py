"""BASELINE.json configs[1] (C2) at its full size on the GPU, and at the bench's pass size against
the oracle.

* 1M accounts, 100M uniform transfers, 512-prepare device passes (the bench's HBM-resident leg):
  every reply empty, 100M stored transfers, and every account's four balances equal to the sums of
  the amounts of the transfers naming it — computed independently on the GPU with torch (exact
  int64 index_add over the 100M events), compared word for word with the engine's export.  (C2 has
  no failing event, so the sums are the reference's sequential result; size-independent properties
  instead of a 100M-transfer oracle run.)
* 4.19M transfers in 512-prepare passes (the legs path at full pass size), byte for byte against the
  oracle: replies, accounts, transfers, posted groove, commit_timestamp.
"""
import numpy as np
import pytest
import torch

from tests.harness.configs import batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.test_gpu_differential import assert_same_state

pytestmark = pytest.mark.gpu

BATCH = 8190


def _i64(events, off):
    """Column of the 128-B records at byte offset `off` as int64 (little-endian u64 words)."""
    return events[:, off:off + 8].contiguous().view(torch.int64).view(-1)


def test_c2_full_size_balances(gpu_engine_factory):
    n_acct, n_xfer, pb = 1_000_000, 100_000_000, 512
    engine = gpu_engine_factory(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pb * BATCH,
                                pass_batches_max=pb)
    dev = torch.device("cuda", 0)
    accts = torch.empty((n_acct, 128), dtype=torch.uint8, device=dev)
    engine.generate_accounts(accts.data_ptr(), 0, n_acct, seed=5)
    a_lens = batches(n_acct, BATCH)
    a_ts, t = timestamps(a_lens, 10**12)
    res = torch.empty(n_xfer * 8, dtype=torch.uint8, device=dev)  # replies at each prepare's event offset
    rb = torch.empty(len(batches(n_xfer, BATCH)) * 4, dtype=torch.uint8, device=dev)
    engine.commit_device_async(128, a_ts, a_lens, accts.data_ptr(), res.data_ptr(), rb.data_ptr())
    engine.sync()
    assert int(rb[:len(a_lens) * 4].view(torch.int32).sum()) == 0

    events = torch.empty((n_xfer, 128), dtype=torch.uint8, device=dev)
    engine.generate_transfers(events.data_ptr(), 0, n_xfer, n_acct, seed=5, kind=0)
    x_lens = batches(n_xfer, BATCH)
    x_ts, _ = timestamps(x_lens, t + 10)
    engine.commit_device_async(129, x_ts, x_lens, events.data_ptr(), res.data_ptr(), rb.data_ptr())
    engine.sync()
    assert int(rb.view(torch.int32).sum()) == 0, "a C2 transfer failed"
    assert engine.stats()["transfers"] == n_xfer

    # Expected balances, independently: account index of every debit / credit id, int64 sums.
    ids = _i64(accts, 0)
    order = torch.argsort(ids)
    sorted_ids = ids[order]
    assert bool((_i64(accts, 8) == _i64(accts, 8)[0]).all())  # C2 ids differ in the low word only
    amount = _i64(events, 48)
    assert bool((_i64(events, 56) == 0).all()) and bool((amount > 0).all())
    expect = {}
    for name, off in (("debits_posted", 16), ("credits_posted", 32)):
        lo = _i64(events, off)
        k = torch.searchsorted(sorted_ids, lo)
        assert bool((sorted_ids[k.clamp(max=n_acct - 1)] == lo).all())
        assert bool((_i64(events, off + 8) == _i64(accts, 8)[0]).all())
        sums = torch.zeros(n_acct, dtype=torch.int64, device=dev)
        sums.index_add_(0, k, amount)
        expect[name] = sums.cpu().numpy().view(np.uint64)
    del events

    got = engine.export_accounts()
    assert len(got) == n_acct
    g_order = np.argsort(got["id_lo"])
    assert np.array_equal(got["id_lo"][g_order], sorted_ids.cpu().numpy().view(np.uint64))
    for name in ("debits_posted", "credits_posted"):
        assert np.array_equal(got[name + "_lo"][g_order], expect[name]), name
        assert not got[name + "_hi"].any()
    for name in ("debits_pending", "credits_pending"):
        assert not got[name + "_lo"].any() and not got[name + "_hi"].any()


def test_c2_pass_size_oracle(gpu_engine_factory):
    n_acct, pb = 100_000, 512
    n_xfer = pb * BATCH
    engine = gpu_engine_factory(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pb * BATCH,
                                pass_batches_max=pb)
    accts, xfers = generate(engine, "c2", n_acct, n_xfer, seed=9)
    a_lens, x_lens = batches(n_acct, BATCH), batches(n_xfer, BATCH)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acct, n_xfer)
    for e in (oracle, engine):
        assert all(r == b"" for r in e.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    actual = engine.commit_many(129, x_ts, split(xfers, x_lens))  # one 512-prepare pass
    assert actual == expected
    assert_same_state(oracle, engine)
