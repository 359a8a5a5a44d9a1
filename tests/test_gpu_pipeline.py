"""Pipelined host commits (tbgpu_commit_pipelined: chunk c+1's bodies cross PCIe while chunk c
commits, replies land in pinned memory per chunk) against the oracle, bit-exact.

* BASELINE.json configs[0] ("C1", scripts/benchmark.sh / src/benchmark.zig:22-24) at full size:
  10,000 accounts, 1,000,000 transfers, prepares of 8190, bodies in registered host memory.
* The C3 / C4 shapes and the seeded differential workloads with small chunks, so chunk boundaries
  cut through every dependency class (chains never span prepares, so any cut is legal).
"""
import numpy as np
import pytest

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine, OraclePanic
from tests.harness.workload import make_scenario, run_oracle
from tests.test_gpu_differential import CONFIGS, assert_same_state
from tigerbeetle_amd._lib import EnginePanic

pytestmark = pytest.mark.gpu


def replies_of(out_lens, replies, lens):
    got, off = [], 0
    for L, nb in zip(lens, out_lens):
        got.append(bytes(replies[off * 8:off * 8 + int(nb)]))
        off += L
    return got


def test_c1_full_size(gpu_engine_factory):
    n_accounts, n_transfers, batch = 10_000, 1_000_000, 8190
    engine = gpu_engine_factory(accounts_max=n_accounts, transfers_max=n_transfers, pass_events_max=64 * batch,
                                pass_batches_max=64)
    accts, xfers = generate(engine, "c2", n_accounts, n_transfers, seed=42)
    a_lens = batches(n_accounts, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_lens = batches(n_transfers, batch)
    assert len(x_lens) == 123 and x_lens[-1] == 820
    x_ts, _ = timestamps(x_lens, t + 10)

    oracle = OracleEngine(n_accounts, n_transfers)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    assert all(r == b"" for r in expected)  # the reference benchmark panics on any error

    host = np.ascontiguousarray(accts)
    rb, rep, _ = engine.commit_pipelined(128, a_ts, a_lens, host, chunk_batches=1)
    assert int(rb.sum()) == 0
    host = np.ascontiguousarray(xfers)
    engine.register_host(host)
    try:
        rb, rep, lat = engine.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=16, latency=True)
    finally:
        engine.unregister_host(host)
    assert replies_of(rb, rep, x_lens) == expected
    assert np.all(lat > 0)
    assert_same_state(oracle, engine)


@pytest.mark.parametrize("config,chunk", [("c3", 3), ("c4", 5), ("c4", 1)])
def test_config_shapes_pipelined(config, chunk, gpu_engine_factory):
    n_accounts, n_transfers, batch = 5_000, 120_000, 8190
    engine = gpu_engine_factory(accounts_max=n_accounts, transfers_max=n_transfers, pass_events_max=8 * batch,
                                pass_batches_max=8)
    accts, xfers = generate(engine, config, n_accounts, n_transfers, seed=11)
    a_lens = batches(n_accounts, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_lens = batches(n_transfers, batch)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[config]["gap_every"])
    oracle = OracleEngine(n_accounts, n_transfers)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
    assert int(rb.sum()) == 0
    rb, rep, _ = engine.commit_pipelined(129, x_ts, x_lens, np.ascontiguousarray(xfers), chunk_batches=chunk)
    assert replies_of(rb, rep, x_lens) == expected
    assert_same_state(oracle, engine)
    assert sum(len(r) for r in expected) > 0


def run_pipelined(sc, engine, chunk):
    """Replay a scenario, consecutive commits of one operation as one pipelined call."""
    out, group = [], []

    def flush():
        if group:
            lens = [len(g[3]) for g in group]
            body = np.frombuffer(b"".join(b"".join(g[3]) for g in group), dtype=np.uint8).copy()
            rb, rep, _ = engine.commit_pipelined(group[0][1], [g[2] for g in group], lens, body, chunk_batches=chunk)
            out.extend(replies_of(rb, rep, lens))
            group.clear()

    for step in sc.steps:
        if step[0] == "setup":
            flush()
            engine.set_balances(*step[1:])
        else:
            if group and group[0][1] != step[1]:
                flush()
            group.append(step)
    flush()
    return out


@pytest.mark.parametrize("config", ["mixed", "chains", "two_phase", "limits", "hot_ids", "overflow"])
@pytest.mark.parametrize("chunk", [1, 2, 5])
def test_differential_pipelined(config, chunk, gpu_engine_factory):
    sc = make_scenario(4441 + chunk * 31 + sum(map(ord, config)), **CONFIGS[config])
    oracle, engine = OracleEngine(), gpu_engine_factory()
    try:
        expected = run_oracle(sc, oracle)
    except OraclePanic:
        with pytest.raises(EnginePanic):
            run_pipelined(sc, engine, chunk)
        return
    actual = run_pipelined(sc, engine, chunk)
    assert actual == expected
    assert_same_state(oracle, engine)


def test_pipelined_rejects_bad_timestamps(gpu_engine_factory):
    engine = gpu_engine_factory()
    body = np.zeros(128 * 2, dtype=np.uint8)
    with pytest.raises(EnginePanic):  # state_machine.zig:519: timestamp must exceed commit_timestamp
        engine.commit_pipelined(129, [100, 100], [1, 1], body)


def test_pipelined_stops_at_device_panic(gpu_engine_factory):
    """A device panic in an early chunk (the reference traps there: post of a pending transfer whose
    pending balance was set below its amount, state_machine.zig:951-956 checked `-=`) ends the call
    with PANIC; the chunks already enqueued behind it report no replies (out_lens stay 0)."""
    import ctypes

    from tigerbeetle_amd import _lib
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, TransferFlags

    engine = gpu_engine_factory()
    acc = np.zeros(2, dtype=ACCOUNT_DTYPE)
    acc["id_lo"] = [1, 2]
    acc["ledger"] = 1
    acc["code"] = 1
    assert engine.commit(128, 10, acc.tobytes()) == b""
    pend = np.zeros(1, dtype=TRANSFER_DTYPE)
    pend["id_lo"] = 10
    pend["debit_account_id_lo"] = 1
    pend["credit_account_id_lo"] = 2
    pend["amount_lo"] = 100
    pend["ledger"] = 1
    pend["code"] = 1
    pend["flags"] = int(TransferFlags.pending)
    assert engine.commit(129, 20, pend.tobytes()) == b""
    engine.set_balances(1, 0, 0, 0, 0)  # debits_pending 100 -> 0: the post's `-=` traps

    n = 6
    x = np.zeros(n, dtype=TRANSFER_DTYPE)
    x["id_lo"] = [11, 0, 21, 0, 31, 0]  # prepares 1, 3, 5 would reply id_must_not_be_zero
    x["debit_account_id_lo"] = 1
    x["credit_account_id_lo"] = 2
    x["amount_lo"] = 1
    x["ledger"] = 1
    x["code"] = 1
    x["pending_id_lo"][0] = 10
    x["flags"][0] = int(TransferFlags.post_pending_transfer)
    x["debit_account_id_lo"][0] = 0
    x["credit_account_id_lo"][0] = 0
    x["amount_lo"][0] = 0
    body = np.frombuffer(x.tobytes(), dtype=np.uint8).copy()
    replies = np.zeros(n * 8, dtype=np.uint8)
    ts = np.arange(30, 30 + 10 * n, 10, dtype=np.uint64)
    ins = (np.arange(n, dtype=np.uint64) * 128 + np.uint64(body.ctypes.data)).astype(np.uint64)
    outs = (np.arange(n, dtype=np.uint64) * 8 + np.uint64(replies.ctypes.data)).astype(np.uint64)
    in_lens = np.full(n, 128, dtype=np.uint32)
    out_lens = np.full(n, 77, dtype=np.uint32)
    P = ctypes.c_void_p
    st = engine.lib.tbgpu_commit_pipelined(
        engine.h, 129, n, ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ins.ctypes.data_as(ctypes.POINTER(P)),
        in_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), outs.ctypes.data_as(ctypes.POINTER(P)),
        out_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 1, None)
    assert st == _lib.STATUS_PANIC
    assert out_lens.tolist() == [0] * n  # nothing after the panicking chunk is reported
    assert int(engine.lib.tbgpu_commit_timestamp(engine.h)) < int(ts[1])  # no later chunk advanced it
