"""The engine's conventions (include/tbgpu.h): no allocation after tbgpu_init on the commit,
prefetch and write-back entry points; a prefetch-staged body belongs to the very next commit only;
a device panic stops the engine until tbgpu_reset; kernel launch spans on the device clock; and the
asynchronous write-back returns exactly what the synchronous one does, however many commits run
while it is in flight."""
import ctypes

import numpy as np
import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import Scenario, make_scenario, run_many, run_oracle
from tests.test_gpu_differential import CONFIGS
from tigerbeetle_amd import _lib
from tigerbeetle_amd._lib import EnginePanic
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, TransferFlags

pytestmark = pytest.mark.gpu


def allocations():
    return int(_lib.load().tbgpu_debug_allocations())


def _accounts(n, ledger=1):
    a = np.zeros(n, dtype=ACCOUNT_DTYPE)
    a["id_lo"] = np.arange(1, n + 1)
    a["ledger"] = ledger
    a["code"] = 1
    return a


def _transfers(n, first_id, n_accounts, amount=1):
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    t["id_lo"] = np.arange(first_id, first_id + n)
    t["debit_account_id_lo"] = 1 + np.arange(n) % n_accounts
    t["credit_account_id_lo"] = 1 + (np.arange(n) + 1) % n_accounts
    t["amount_lo"] = amount
    t["ledger"] = 1
    t["code"] = 1
    return t


def _prefetch(engine, op, arr):
    _lib.check(engine.lib.tbgpu_prefetch(engine.h, op, arr.ctypes.data, arr.nbytes))


def _commit_raw(engine, op, ts, arr):
    out = np.zeros(max(arr.nbytes // 128 * 8, 8), dtype=np.uint8)
    n = ctypes.c_uint32(0)
    _lib.check(engine.lib.tbgpu_commit(engine.h, op, ts, arr.ctypes.data, arr.nbytes, out.ctypes.data, out.nbytes,
                                       ctypes.byref(n)))
    return out[:n.value].tobytes()


@pytest.mark.parametrize("profile", [False, True])
def test_no_allocation_after_init(profile, gpu_engine_factory):
    engine = gpu_engine_factory(accounts_max=1 << 12, transfers_max=1 << 18, pass_events_max=1 << 14,
                                pass_batches_max=16, profile=profile)
    body = np.zeros(4 * 8190 * 128, dtype=np.uint8)
    engine.register_host(body)
    before = allocations()
    ts = 10**9
    assert engine.commit(128, ts, _accounts(64).tobytes()) == b""
    k = 1
    for rnd in range(3):
        t = _transfers(8190, k, 64)
        k += 8190
        ts += 10**4
        assert engine.commit(129, ts, t.tobytes()) == b""                       # pageable, one prepare
        t = _transfers(8190, k, 64)
        k += 8190
        body[:t.nbytes] = t.view(np.uint8)
        ts += 10**4
        assert _commit_raw(engine, 129, ts, body[:t.nbytes]) == b""             # registered: read through
        t2 = _transfers(8190, k, 64)
        k += 8190
        body[:t2.nbytes] = t2.view(np.uint8)
        _prefetch(engine, 129, body[:t2.nbytes])
        ts += 10**4
        assert _commit_raw(engine, 129, ts, body[:t2.nbytes]) == b""            # staged by prefetch
        many = [_transfers(1000, k + 1000 * j, 64).tobytes() for j in range(3)]
        k += 3000
        assert engine.commit_many(129, [ts + 10**4 * (j + 1) for j in range(3)], many) == [b""] * 3
        ts += 10**5
        t3 = _transfers(3 * 8190, k, 64)
        k += 3 * 8190
        body[:t3.nbytes] = t3.view(np.uint8)
        rb, _, _ = engine.commit_pipelined(129, [ts + 10**4 * (j + 1) for j in range(3)], [8190] * 3, body,
                                           chunk_batches=1)
        assert int(rb.sum()) == 0
        ts += 10**5
        ids = np.zeros((4, 2), dtype=np.uint64)
        ids[:, 0] = [1, 2, 3, 999]
        assert len(engine.commit(130, ts, ids.tobytes())) == 3 * 128              # lookup_accounts
        ts += 10**4
        d = engine.checkpoint_delta(caps=(1 << 16, 1 << 16, 1 << 16))          # synchronous write-back
        assert len(d.transfers) > 0
        ts += 10**4
        assert engine.commit(129, ts, _transfers(100, k, 64).tobytes()) == b""
        k += 100
        engine.checkpoint_delta_async((1 << 16, 1 << 16, 1 << 16))             # asynchronous write-back
        ts += 10**4
        assert engine.commit(129, ts, _transfers(100, k, 64).tobytes()) == b""  # while it is in flight
        k += 100
        assert len(engine.checkpoint_delta_wait().transfers) == 100
        engine.stats()
        if rnd == 0:  # the write-back buffer sets of the mirror are registered by now
            before = allocations()
    assert allocations() == before, "an entry point allocated after tbgpu_init"
    engine.unregister_host(body)


@pytest.mark.parametrize("profile", [False, True])
def test_no_allocation_after_init_node(profile):
    """The same rule on a node engine (two logical shards): every commit entry point (create_accounts
    through the sequencer, create_transfers routed and split, one prepare and many), lookups and the
    synchronous write-back make no device, pinned or event allocation after tbgpu_init."""
    from tigerbeetle_amd.state_machine import Engine, Options
    engine = Engine(Options(accounts_max=1 << 12, transfers_max=1 << 18, pass_events_max=1 << 14, pass_batches_max=16,
                            devices=(0, 0), profile=profile))
    try:
        body = np.zeros(4 * 8190 * 128, dtype=np.uint8)
        engine.register_host(body)
        ts = 10**9
        k = 1
        before = None
        for rnd in range(3):
            a = _accounts(64)
            a["id_lo"] += 64 * rnd
            assert engine.commit(128, ts, a.tobytes()) == b""                   # create_accounts (sequencer)
            n_acc = 64 * (rnd + 1)
            t = _transfers(8190, k, n_acc)
            k += 8190
            ts += 10**4
            assert engine.commit(129, ts, t.tobytes()) == b""                   # one prepare, clean pass
            t = _transfers(8190, k, n_acc)
            t["flags"][::7] = TransferFlags.linked
            t["flags"][-1] = 0
            k += 8190
            ts += 10**4
            assert engine.commit(129, ts, t.tobytes()) == b""                   # dirty pass: split
            many = [_transfers(1000, k + 1000 * j, n_acc).tobytes() for j in range(3)]
            k += 3000
            assert engine.commit_many(129, [ts + 10**4 * (j + 1) for j in range(3)], many) == [b""] * 3
            ts += 10**5
            t3 = _transfers(3 * 8190, k, n_acc)
            k += 3 * 8190
            body[:t3.nbytes] = t3.view(np.uint8)
            rb, _, _ = engine.commit_pipelined(129, [ts + 10**4 * (j + 1) for j in range(3)], [8190] * 3, body,
                                               chunk_batches=1)
            assert int(rb.sum()) == 0
            ts += 10**5
            ids = np.zeros((4, 2), dtype=np.uint64)
            ids[:, 0] = [1, 2, 3, 9999]
            assert len(engine.commit(130, ts, ids.tobytes())) == 3 * 128          # lookup_accounts
            ts += 10**4
            d = engine.checkpoint_delta(caps=(1 << 17, 1 << 17, 1 << 17))      # synchronous write-back
            assert len(d.transfers) > 0
            engine.stats()
            if rnd == 0:  # the mirror's write-back buffers are registered by now
                before = allocations()
        assert allocations() == before, "a node entry point allocated after tbgpu_init"
        engine.unregister_host(body)
    finally:
        engine.close()


def test_prefetch_staging_belongs_to_the_next_commit(gpu_engine_factory):
    """A staged body is taken by the commit right after its prefetch only: any call in between drops
    it, and a re-prefetch restages the current bytes."""
    engine = gpu_engine_factory()
    buf = np.zeros(64 * 128, dtype=np.uint8)
    engine.register_host(buf)
    assert engine.commit(128, 100, _accounts(8).tobytes()) == b""
    good = _transfers(64, 1000, 8)
    bad = good.copy()
    bad["ledger"][::2] = 0  # every other event: ledger_must_not_be_zero (the same ids, never inserted)
    ts = 1000

    def expect_bad(reply):
        r = np.frombuffer(reply, dtype=np.uint32).reshape(-1, 2)
        assert r[:, 0].tolist() == list(range(0, 64, 2))

    # 1. prefetch(good) -> another call -> buffer now holds `bad` -> commit sees `bad`.
    buf[:] = good.view(np.uint8)
    _prefetch(engine, 129, buf)
    engine.stats()
    buf[:] = bad.view(np.uint8)
    ts += 100
    expect_bad(_commit_raw(engine, 129, ts, buf))
    # 2. prefetch(good) -> buffer changes -> prefetch again -> commit sees the new bytes.
    good2 = _transfers(64, 5000, 8)
    bad2 = good2.copy()
    bad2["ledger"][::2] = 0
    buf[:] = good2.view(np.uint8)
    _prefetch(engine, 129, buf)
    buf[:] = bad2.view(np.uint8)
    _prefetch(engine, 129, buf)
    ts += 100
    expect_bad(_commit_raw(engine, 129, ts, buf))
    # 3. a failed commit drops it too: prefetch(good) -> commit with a stale timestamp (PANIC, no
    #    state change) -> buffer changes -> commit sees the new bytes.
    good3 = _transfers(64, 9000, 8)
    bad3 = good3.copy()
    bad3["ledger"][::2] = 0
    buf[:] = good3.view(np.uint8)
    _prefetch(engine, 129, buf)
    with pytest.raises(EnginePanic):
        _commit_raw(engine, 129, 1, buf)
    buf[:] = bad3.view(np.uint8)
    ts += 100
    expect_bad(_commit_raw(engine, 129, ts, buf))
    # 4. a registered body: prefetch stages nothing (the commit reads it through) -> the same bytes.
    good4 = _transfers(64, 20000, 8)
    buf[:] = good4.view(np.uint8)
    _prefetch(engine, 129, buf)
    ts += 100
    assert _commit_raw(engine, 129, ts, buf) == b""
    engine.unregister_host(buf)
    # 5. the staged path itself (a pageable body): prefetch -> commit of the same bytes; and a
    #    re-prefetch after the bytes changed restages them.
    page = np.zeros(64 * 128, dtype=np.uint8)
    page[:] = _transfers(64, 30000, 8).view(np.uint8)
    _prefetch(engine, 129, page)
    ts += 100
    assert _commit_raw(engine, 129, ts, page) == b""
    good6 = _transfers(64, 40000, 8)
    bad6 = good6.copy()
    bad6["ledger"][::2] = 0
    page[:] = good6.view(np.uint8)
    _prefetch(engine, 129, page)
    page[:] = bad6.view(np.uint8)
    _prefetch(engine, 129, page)
    ts += 100
    expect_bad(_commit_raw(engine, 129, ts, page))


def test_device_panic_stops_the_engine_until_reset(gpu_engine_factory):
    engine = gpu_engine_factory()
    assert engine.commit(128, 10, _accounts(2).tobytes()) == b""
    pend = _transfers(1, 10, 2, amount=100)
    pend["flags"] = int(TransferFlags.pending)
    assert engine.commit(129, 20, pend.tobytes()) == b""
    engine.set_balances(1, 0, 0, 0, 0)  # debits_pending 100 -> 0: the post's checked `-=` traps
    post = np.zeros(1, dtype=TRANSFER_DTYPE)
    post["id_lo"] = 11
    post["pending_id_lo"] = 10
    post["flags"] = int(TransferFlags.post_pending_transfer)
    with pytest.raises(EnginePanic):
        engine.commit(129, 30, post.tobytes())
    with pytest.raises(EnginePanic, match="stopped"):
        engine.commit(129, 40, _transfers(1, 50, 2).tobytes())
    engine.export_accounts()  # reads still work
    engine.reset()
    assert engine.commit(128, 10, _accounts(2).tobytes()) == b""
    assert engine.commit(129, 20, _transfers(4, 1, 2).tobytes()) == b""


def test_kernel_spans_on_the_device_clock(gpu_engine_factory):
    """Launch spans on the device clock: one per pass for validate and resolve, each no longer than the
    HIP-event pair around the same launch (which also holds its dispatch) — validate's span measured
    with no event pair inside it (between tb_pass_clear and tb_resolve, pass.h)."""
    engine = gpu_engine_factory(accounts_max=1 << 12, transfers_max=1 << 18, pass_events_max=1 << 15,
                                pass_batches_max=8, profile=True)
    assert engine.commit(128, 10**9, _accounts(256).tobytes()) == b""

    def run(first, mask):
        engine.reset_stats()
        engine.profile_mask(mask)
        bodies = [_transfers(8190, first + 8190 * j, 256).tobytes() for j in range(4)]
        assert engine.commit_many(129, [10**10 * first + 10**5 * j for j in range(4)], bodies) == [b""] * 4
        return engine.stats()

    hip = run(1, engine.PROF_ALL)
    st = run(1 + 4 * 8190, engine.PROF_APPLY)
    assert st["span_launches"][0] == st["passes"] > 0 and st["span_launches"][1] == st["passes"]
    for k, key, launches in ((0, "ms_validate", "launches_validate"), (1, "ms_resolve", "launches_resolve")):
        per_span = st["span_ms"][k] / st["span_launches"][k]
        per_hip = hip[key] / hip[launches]
        assert 0 < per_span <= per_hip * 1.25 + 0.005, (k, per_span, per_hip)


@pytest.mark.parametrize("devices", [None, (0, 0)], ids=["single", "node2"])
@pytest.mark.parametrize("config", ["mixed", "two_phase", "chains"])
def test_async_write_back_equals_sync(config, devices, gpu_engine_factory):
    """Each segment's write-back through tbgpu_checkpoint_delta_async, waited for only after the
    next segment committed, equals the synchronous write-back of an engine committing the same
    (node2: a two-shard node, whose asynchronous write-back merges the shards at the call)."""
    sc = make_scenario(707 + sum(map(ord, config)), **CONFIGS[config])
    cut = np.linspace(0, len(sc.steps), 5).astype(int)
    segs = []
    for a, b in zip(cut[:-1], cut[1:]):
        s = Scenario()
        s.steps = sc.steps[a:b]
        segs.append(s)
    kw = dict(devices=devices) if devices else {}
    e_sync, e_async = gpu_engine_factory(**kw), gpu_engine_factory(**kw)
    caps = (1 << 14, 1 << 14, 1 << 14)

    def rows(arr):
        return sorted(bytes(r) for r in np.asarray(arr).view(np.uint8).reshape(len(arr), -1))

    expected, got = [], []
    for i, seg in enumerate(segs):
        run_many(seg, e_sync)
        expected.append(e_sync.checkpoint_delta(caps=caps))
        run_many(seg, e_async)
        if i:
            got.append(e_async.checkpoint_delta_wait())  # the previous segment's, after this one committed
        e_async.checkpoint_delta_async(caps)
    got.append(e_async.checkpoint_delta_wait())
    for d_s, d_a in zip(expected, got):
        assert np.array_equal(d_s.transfers, d_a.transfers)  # by timestamp on both
        assert np.array_equal(d_s.posted, d_a.posted)
        assert d_s.created_after == d_a.created_after
        assert rows(d_s.accounts) == rows(d_a.accounts)
        assert sorted(zip(map(bytes, d_s.accounts.view(np.uint8).reshape(-1, 128)), map(bytes, d_s.accounts_before))) == \
            sorted(zip(map(bytes, d_a.accounts.view(np.uint8).reshape(-1, 128)), map(bytes, d_a.accounts_before)))
    oracle = OracleEngine()
    run_oracle(sc, oracle)
    assert e_async.export_accounts().tobytes() == oracle.export_accounts().tobytes()


def _chunk_ops(rng, n_acc, per_op, ops, first_id):
    """`ops` create_transfers bodies of `per_op` events over `n_acc` accounts: an eighth pending,
    and from the second op on a sixteenth posting or voiding a pending transfer of an earlier op."""
    bodies, pending, next_id = [], [], first_id
    for k in range(ops):
        t = np.zeros(per_op, dtype=TRANSFER_DTYPE)
        t["id_lo"] = np.arange(next_id, next_id + per_op)
        next_id += per_op
        dr = rng.integers(1, n_acc + 1, per_op)
        cr = 1 + (dr + rng.integers(0, n_acc - 1, per_op)) % n_acc
        t["debit_account_id_lo"], t["credit_account_id_lo"] = dr, cr
        t["amount_lo"] = rng.integers(1, 100, per_op)
        t["ledger"], t["code"] = 1, 1
        pend = rng.random(per_op) < 1 / 8
        t["flags"][pend] = int(TransferFlags.pending)
        if pending:
            for i in rng.choice(per_op, per_op // 16, replace=False):
                if not pending or pend[i]:
                    continue
                p = pending.pop(int(rng.integers(0, len(pending))))
                t["flags"][i] = int(TransferFlags.post_pending_transfer if i % 2 else TransferFlags.void_pending_transfer)
                t["pending_id_lo"][i] = p["id_lo"]
                for f in ("debit_account_id_lo", "credit_account_id_lo", "amount_lo"):
                    t[f][i] = p[f]
        pending.extend(t[pend])
        bodies.append(t)
    return bodies


@pytest.mark.parametrize("stage", [False, True], ids=["read_through", "staged"])
def test_chunked_write_back_bound_copy_out(stage, gpu_engine_factory):
    """A write-back every two one-prepare commits, as a replica writing back every few ops does.
    Once a write-back's objects fill their bounds, the next copy-outs are sent at their bounds from
    the first commit after (`write_backs_bound`); with prefetch staging the bodies while a copy-out
    is in flight (`staged`) no slice waits for a commit's reads.  Every delta equals the synchronous
    write-back of an engine committing the same prepares, the posted pairs (which cross at the wait)
    included, and the replies and balances equal the oracle's."""
    n_acc, per_op, ops = 1 << 16, 512, 24
    kw = dict(accounts_max=n_acc, transfers_max=1 << 16, pass_events_max=1 << 13, pass_batches_max=8)
    e_sync, e_async = gpu_engine_factory(**kw), gpu_engine_factory(**kw)
    oracle = OracleEngine(n_acc, ops * per_op)
    ts = 10**9
    for a0 in range(0, n_acc, 8190):
        body = _accounts(min(8190, n_acc - a0))
        body["id_lo"] += a0
        ts += 10**6
        for e in (e_sync, e_async, oracle):
            assert e.commit(128, ts, body.tobytes()) == b""
    caps = (1 << 14, 1 << 14, 1 << 14)
    e_sync.checkpoint_delta(caps=caps)
    e_async.checkpoint_delta(caps=caps)
    buf = np.zeros(per_op * 128, dtype=np.uint8)
    e_async.register_host(buf)
    expected, got = [], []
    for k, t in enumerate(_chunk_ops(np.random.default_rng(5), n_acc, per_op, ops, 1 << 20)):
        ts += 10**6
        buf[:] = t.view(np.uint8)
        if stage:
            _prefetch(e_async, 129, buf)
        reply = _commit_raw(e_async, 129, ts, buf)
        assert reply == e_sync.commit(129, ts, t.tobytes()) == oracle.commit(129, ts, t.tobytes())
        if k % 2 == 1:
            expected.append(e_sync.checkpoint_delta(caps=caps))
            if k > 1:
                got.append(e_async.checkpoint_delta_wait())
            e_async.checkpoint_delta_async(caps)
    got.append(e_async.checkpoint_delta_wait())
    st = e_async.stats()
    assert st["write_backs_async"] == ops // 2 and st["write_backs_bound"] == ops // 2 - 1, st
    assert sum(len(d.posted) for d in expected[1:]) > 0
    for d_s, d_a in zip(expected, got, strict=True):
        assert np.array_equal(d_s.transfers, d_a.transfers)
        assert np.array_equal(d_s.posted, d_a.posted)
        assert d_s.created_after == d_a.created_after
        assert sorted(zip(map(bytes, d_s.accounts.view(np.uint8).reshape(-1, 128)), map(bytes, d_s.accounts_before))) == \
            sorted(zip(map(bytes, d_a.accounts.view(np.uint8).reshape(-1, 128)), map(bytes, d_a.accounts_before)))
    e_async.unregister_host(buf)
    assert e_async.export_accounts().tobytes() == oracle.export_accounts().tobytes()
