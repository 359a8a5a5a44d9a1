"""The node engine: one tbgpu handle over N shards (include/tbgpu.h tbgpu_config.devices, csrc/node.h)
driven through the same C ABI as a single-device engine, against the oracle byte for byte.

The box has one GPU, so the shards are LOGICAL shards sharing cuda:0 (devices = (0, 0) or
(0, 0, 0)): the routing, the gathers from the sources' send buffers, the owner legs, the replies
built from the homes' codes and the sequencer of dirty passes all run exactly as across GPUs; only
the peer reads stay inside one HBM instead of crossing xGMI."""
import numpy as np
import pytest

from tests.harness import known_answers, table
from tests.harness.configs import batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.harness.workload import make_scenario
from tests.test_gpu_differential import CONFIGS, _run, assert_same_state
from tests.test_gpu_tables import TABLES
from tigerbeetle_amd._lib import EngineError
from tigerbeetle_amd.types import TRANSFER_DTYPE

pytestmark = pytest.mark.gpu


@pytest.fixture
def node_factory():
    from tigerbeetle_amd.state_machine import Engine, Options

    made = []

    def make(devices=(0, 0), **kw):
        opts = dict(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64,
                    devices=tuple(devices))
        opts.update(kw)
        e = Engine(Options(**opts))
        made.append(e)
        return e

    yield make
    for e in made:
        e.close()


@pytest.mark.parametrize("name,text", TABLES, ids=[n for n, _ in TABLES])
def test_node_reproduces_reference_table(name, text, node_factory):
    table.check(text, node_factory())


@pytest.mark.parametrize("config", ["mixed", "chains", "two_phase", "limits", "hot_ids", "clean", "overflow",
                                    "big_batches"])
@pytest.mark.parametrize("many", [False, True], ids=["commit", "commit_many"])
def test_node_differential(config, many, node_factory):
    sc = make_scenario(5003 + sum(map(ord, config)), **CONFIGS[config])
    _run(sc, OracleEngine(), node_factory(devices=(0, 0, 0) if many else (0, 0)), many)


@pytest.mark.parametrize("scenario", known_answers.load(), ids=lambda s: s["name"])
def test_node_client_answers(scenario, node_factory):
    known_answers.run(scenario, node_factory())


@pytest.mark.parametrize("shards", [2, 3])
def test_node_imports_persist_until_accounts_change(shards, node_factory):
    """A home keeps the foreign accounts it imported for the next passes (k_node.h tb_node_import),
    the tombstones of ids no owner held included, and flushes them before any account is inserted:
    transfers naming missing accounts, then those accounts created, then transfers naming them again
    (and passes re-reading the kept imports) answer as the oracle does; the ledger summary, read with
    the imports still in the tables, counts each account once and finds no stray balance."""
    from tigerbeetle_amd.types import ACCOUNT_DTYPE
    engine = node_factory(devices=(0,) * shards)
    oracle = OracleEngine(4096, 1 << 14)
    rng = np.random.default_rng(11 + shards)

    def accounts(ids, ledger=1):
        a = np.zeros(len(ids), dtype=ACCOUNT_DTYPE)
        a["id_lo"] = ids
        a["ledger"], a["code"] = ledger, 7
        return a.tobytes()

    next_id = [1]

    def transfers(n, dr_ids, cr_ids, ledger=1):
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        t["id_lo"] = np.arange(next_id[0], next_id[0] + n)
        next_id[0] += n
        t["debit_account_id_lo"] = rng.choice(dr_ids, n)
        t["credit_account_id_lo"] = rng.choice(cr_ids, n)
        t["credit_account_id_lo"] = np.where(t["credit_account_id_lo"] == t["debit_account_id_lo"],
                                             t["credit_account_id_lo"] + 1000, t["credit_account_id_lo"])
        t["amount_lo"] = rng.integers(1, 50, n)
        t["ledger"], t["code"] = ledger, 1
        return t.tobytes()

    ts = [10**9]

    def both(op, body):
        ts[0] += 10**6
        got, want = engine.commit(op, ts[0], body), oracle.commit(op, ts[0], body)
        assert got == want
        return got

    old, late = np.arange(1, 201), np.arange(500, 541)
    both(128, accounts(old))
    both(128, accounts(old + 1000))
    for _ in range(3):  # the late accounts do not exist yet: account_not_found, their tombstones kept
        assert both(129, transfers(2000, np.concatenate([old, late]), old)) != b""
    led = engine.ledger_summary()
    assert led["accounts"] == 400 and led["stray"] == 0, led
    both(128, accounts(late))            # flushes every import first
    both(128, accounts(late + 1000, 2))  # a second ledger: exists checks against kept imports would differ
    for k in range(4):
        body = transfers(2000, np.concatenate([old, late]), np.concatenate([old, late]), ledger=1 + (k == 3))
        both(129, body)
    led = engine.ledger_summary()
    assert led["accounts"] == 482 and led["stray"] == 0, led
    assert_same_state(oracle, engine)


@pytest.mark.parametrize("shards", [2, 3, 4])
def test_node_clean_passes_pipelined(shards, node_factory):
    """C2-shaped passes from registered host memory (the headline's call), routed across the shards,
    with the failures a clean pass can hold: duplicate ids inside a pass and across passes (exists,
    exists_with_different_*), a non-zero timestamp field (answered at the source, never routed), a
    missing account — every reply, account, transfer and the commit timestamp equal the oracle's."""
    n_acc, n_xfer, batch, chunk = 6000, 300_000, 8190, 3
    engine = node_factory(devices=(0,) * shards, accounts_max=n_acc, transfers_max=n_xfer,
                          pass_events_max=chunk * batch, pass_batches_max=chunk)
    accts, xfers = generate(engine, "c2", n_acc, n_xfer, seed=5 + shards)
    x = xfers.view(TRANSFER_DTYPE).copy()
    rng = np.random.default_rng(shards)
    dup = rng.choice(np.arange(1000, n_xfer), 600, replace=False)
    src = rng.integers(0, 900, 600)
    x["id_lo"][dup] = x["id_lo"][src]
    x["id_hi"][dup] = x["id_hi"][src]
    x["amount_lo"][dup[:300]] += 1  # exists_with_different_amount for half of them
    x["timestamp"][rng.choice(n_xfer, 200, replace=False)] = 7
    x["debit_account_id_lo"][rng.choice(n_xfer, 200, replace=False)] ^= 0x5A5A
    xfers = x.view(np.uint8).reshape(-1)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
    assert int(rb.sum()) == 0
    host = np.ascontiguousarray(xfers)
    engine.register_host(host)
    try:
        rb, rep, lat = engine.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=chunk, latency=True)
    finally:
        engine.unregister_host(host)
    got, off = [], 0
    for L, nb in zip(x_lens, rb):
        got.append(bytes(rep[off * 8:off * 8 + int(nb)]))
        off += L
    assert got == expected
    assert sum(len(r) for r in expected) > 0
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["transfers"] == len(oracle.export_transfers())


def test_node_checkpoint_and_lookups(node_factory):
    """Write-back of a node equals the oracle's state diff (merged over the shards: each account's
    owner copy, each transfer from its home), and lookups read each object where it lives."""
    from tests.test_gpu_checkpoint import test_checkpoint_deltas
    test_checkpoint_deltas("two_phase", None, lambda **kw: node_factory(devices=(0, 0, 0), **kw))


def test_node_refuses_device_resident(node_factory):
    engine = node_factory()
    with pytest.raises(EngineError):
        engine.commit_device_async(129, [10], [1], 0, 0, 0)


def _commit_generated(config, shards, chunk, n_acc, n_xfer, seed, node_factory):
    """Commit a BASELINE shape (the device generator's accounts, then its transfers from registered
    host memory in `chunk`-prepare blocks) on a node of `shards` logical shards and the oracle; every
    reply, account, transfer and posted entry must be equal. Returns the node's stats."""
    from tests.harness.configs import SETTINGS
    batch = 8190
    engine = node_factory(devices=(0,) * shards, accounts_max=n_acc, transfers_max=n_xfer,
                          pass_events_max=chunk * batch, pass_batches_max=chunk)
    accts, xfers = generate(engine, config, n_acc, n_xfer, seed=seed)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[config]["gap_every"])
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
    assert int(rb.sum()) == 0
    engine.reset_stats()
    host = np.ascontiguousarray(xfers)
    engine.register_host(host)
    try:
        rb, rep, _ = engine.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=chunk)
    finally:
        engine.unregister_host(host)
    got, off = [], 0
    for L, nb in zip(x_lens, rb):
        got.append(bytes(rep[off * 8:off * 8 + int(nb)]))
        off += L
    for k, (e, a) in enumerate(zip(expected, got)):
        assert e == a, "reply of prepare %d differs" % k
    assert_same_state(oracle, engine)
    st = engine.stats()
    led = engine.ledger_summary()
    assert led["stray"] == 0, led
    return expected, st


@pytest.mark.parametrize("config,shards", [("c3", 2), ("c3", 4), ("c4", 2), ("c4", 4)])
def test_node_dirty_passes_split(config, shards, node_factory):
    """BASELINE C3 / C4 shapes at 1M accounts and 2M transfers, through 2 and 4 shards in
    64-prepare blocks: every dirty pass is SPLIT — the dependent subsequence committed in order by
    the sequencer, the rest routed — never sequenced whole (no host code walks the events); every
    reply, account, transfer and posted entry equals the oracle's."""
    n_xfer = 2_000_000
    expected, st = _commit_generated(config, shards, 64, 1_000_000, n_xfer, 11 + shards, node_factory)
    assert sum(len(r) for r in expected) > 0
    assert st["node_passes_whole"] == 0 and st["node_passes_split"] > 0, st
    assert 0 < st["node_sequenced_events"] < n_xfer, st  # only the dependent subsequence is sequenced


def test_node_hw_queues_env():
    """The suite runs the node with every stream on its own hardware queue (tests/conftest.py), the
    concurrency of N real devices; GPU_MAX_HW_QUEUES=4 (HIP's default) is the case that hid round 5's
    sequencer race."""
    import os
    print("GPU_MAX_HW_QUEUES=%s" % os.environ.get("GPU_MAX_HW_QUEUES"))
    assert int(os.environ.get("GPU_MAX_HW_QUEUES", "0")) >= 8


@pytest.mark.parametrize("config", ["c2", "c3", "c4"])
def test_node_eight_shards(config, node_factory):
    """BASELINE configs[4]'s shard count: eight logical shards (devices = (0,) * 8), 16-prepare
    blocks so that every pass has all eight sources busy (128 prepares, 1.05M transfers a pass).
    c2 is C5's clean shape (uniform accounts, 7/8 of the legs cross shards), c3 / c4 its dirty
    shapes (limit accounts under Zipf; chains and two-phase): byte-exact against the oracle, the
    ledger's stray balance zero, and every dirty pass split, never sequenced whole."""
    n_xfer = 2_500_000
    expected, st = _commit_generated(config, 8, 16, 1_000_000, n_xfer, 31, node_factory)
    if config == "c2":
        assert st["node_passes_split"] == 0 and st["node_passes_whole"] == 0, st
    else:
        assert sum(len(r) for r in expected) > 0
        assert st["node_passes_whole"] == 0 and st["node_passes_split"] > 0, st
        assert 0 < st["node_sequenced_events"] < n_xfer, st


@pytest.mark.parametrize("shards", [2, 3])
def test_node_device_resident_blocks(shards, node_factory):
    """The node's device-resident commit (bench.py's `value` at N > 1): every source's prepares sit
    back to back in its own HBM in pass-block order and its route kernels read them in place; the
    same prepares from host memory, and from device memory in another block layout (copied), give the
    oracle's bytes too."""
    n_acc, n_xfer, batch, chunk = 5000, 200_000, 8190, 2
    engine = node_factory(devices=(0,) * shards, accounts_max=n_acc, transfers_max=n_xfer,
                          pass_events_max=chunk * batch, pass_batches_max=chunk)
    accts, xfers = generate(engine, "c2", n_acc, n_xfer, seed=17 + shards)
    x = xfers.view(TRANSFER_DTYPE).copy()
    rng = np.random.default_rng(shards)
    dup = rng.choice(np.arange(1000, n_xfer), 300, replace=False)
    x["id_lo"][dup] = x["id_lo"][rng.integers(0, 900, 300)]
    x["id_hi"][dup] = x["id_hi"][0]
    xfers = x.view(np.uint8).reshape(-1)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
    assert int(rb.sum()) == 0
    n_prep = len(x_lens)
    starts = np.concatenate([[0], np.cumsum(x_lens)]).astype(np.int64)
    src_of = (np.arange(n_prep) % (shards * chunk)) // chunk
    ptrs = np.zeros(n_prep, dtype=np.uint64)
    bufs = []
    for d in range(shards):
        sh = engine.shard(d)
        mine = np.nonzero(src_of == d)[0]
        body = np.concatenate([xfers[starts[k] * 128:starts[k + 1] * 128] for k in mine]) if len(mine) else np.zeros(128, np.uint8)
        dev = sh.alloc(body.nbytes)
        sh.to_device(dev, body)
        bufs.append((sh, dev))
        off = 0
        for k in mine:
            ptrs[k] = dev + off * 128
            off += x_lens[k]
    replies = np.empty(n_xfer * 8, dtype=np.uint8)

    def run(ptr_list, chunk_batches, t0):
        engine.reset_transfers()
        ts, _ = timestamps(x_lens, t0)
        rb, _ = engine.commit_pipelined_ptrs(129, ts, x_lens, ptr_list, replies, chunk_batches=chunk_batches)
        got, off = [], 0
        for L, nb in zip(x_lens, rb):
            got.append(bytes(replies[off * 8:off * 8 + int(nb)]))
            off += L
        return ts, got

    try:
        t0 = t + 10
        ts, got = run(ptrs, chunk, t0)  # resident: every block read in place
        o2 = OracleEngine(n_acc, n_xfer)
        assert all(r == b"" for r in o2.commit_many(128, a_ts, split(accts, a_lens)))
        expected = o2.commit_many(129, ts, split(xfers, x_lens))
        assert got == expected and sum(len(r) for r in expected) > 0
        assert_same_state(o2, engine)
        t0 = ts[-1] + 10
        ts, got = run(ptrs, chunk + 1, t0)  # other blocks: device bodies copied to the sources
        o3 = OracleEngine(n_acc, n_xfer)
        assert all(r == b"" for r in o3.commit_many(128, a_ts, split(accts, a_lens)))
        assert got == o3.commit_many(129, ts, split(xfers, x_lens))
        assert_same_state(o3, engine)
    finally:
        for sh, dev in bufs:
            sh.free(dev)


@pytest.mark.parametrize("config", ["mixed", "two_phase", "limits"])
def test_node_without_issue_pool(config, node_factory, monkeypatch):
    """TBGPU_NODE_THREADS=0: every phase issued shard after shard on the calling thread (no issue
    pool) — the same bytes as the oracle, as with the pool (test_node_differential)."""
    monkeypatch.setenv("TBGPU_NODE_THREADS", "0")
    sc = make_scenario(5003 + sum(map(ord, config)), **CONFIGS[config])
    _run(sc, OracleEngine(), node_factory(devices=(0, 0, 0)), True)


@pytest.mark.parametrize("shards,spin_us", [(2, None), (3, None), (3, "0")], ids=["2", "3", "3-pool-sleeps"])
def test_node_one_prepare_calls(shards, spin_us, node_factory, monkeypatch):
    """The replica's call on a node: one prepare per call from registered host memory (a one-pass
    call: the body's copy on the route stream, the block's metadata from the classification's
    arguments, the plan words and the reply arena read once their completion words flip), clean
    calls with duplicate ids, non-zero timestamps and missing accounts, interleaved with dirty
    calls (a linked chain: a split pass, whose classification rewrites the plan words) — every
    reply, account and transfer equals the oracle's.  TBGPU_NODE_SPIN_US=0: the issue pool's
    threads sleep between every phase (each phase's job reaches them through the condition
    variable)."""
    if spin_us is not None:
        monkeypatch.setenv("TBGPU_NODE_SPIN_US", spin_us)
    n_acc, batch, n_prep = 6000, 8190, 16
    n_xfer = batch * n_prep
    engine = node_factory(devices=(0,) * shards, accounts_max=n_acc, transfers_max=n_xfer,
                          pass_events_max=4 * batch, pass_batches_max=4)
    accts, xfers = generate(engine, "c2", n_acc, n_xfer, seed=23 + shards)
    x = xfers.view(TRANSFER_DTYPE).copy()
    rng = np.random.default_rng(40 + shards)
    dup = rng.choice(np.arange(batch, n_xfer), 400, replace=False)
    src = rng.integers(0, batch, 400)
    x["id_lo"][dup] = x["id_lo"][src]
    x["id_hi"][dup] = x["id_hi"][src]
    x["timestamp"][rng.choice(n_xfer, 100, replace=False)] = 9
    x["debit_account_id_lo"][rng.choice(n_xfer, 100, replace=False)] ^= 0x5A5A
    for k in (3, 4, 9):  # dirty calls: a 6-event linked chain inside the prepare
        x["flags"][k * batch + 100:k * batch + 105] |= 1
    xfers = x.view(np.uint8).reshape(-1)
    a_lens, x_lens = batches(n_acc, batch), [batch] * n_prep
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=4)
    assert int(rb.sum()) == 0
    host = np.ascontiguousarray(xfers)
    engine.register_host(host)
    try:
        got = []
        for k in range(n_prep):
            body = host[k * batch * 128:(k + 1) * batch * 128]
            nb, rep, _ = engine.commit_pipelined(129, [x_ts[k]], [batch], body)
            got.append(bytes(rep[:int(nb[0])]))
    finally:
        engine.unregister_host(host)
    for k, (e, a) in enumerate(zip(expected, got)):
        assert e == a, "reply of prepare %d differs" % k
    assert sum(len(r) for r in expected) > 0
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["node_passes_split"] >= 3, st
