"""Groove write-back (tbgpu_checkpoint_delta, the durable replica's checkpoint / compact:
src/state_machine.zig:542-582 over src/lsm/groove.zig:902-963 insert / upsert).  A scenario is
committed in segments with a write-back after each; each delta must hold exactly the objects the
oracle's state changed in that segment, and replaying the deltas into an empty host "forest" must
rebuild the oracle's final grooves byte for byte."""
import numpy as np
import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import Scenario, make_scenario, run_oracle
from tests.test_gpu_differential import CONFIGS
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

pytestmark = pytest.mark.gpu


def _segments(sc, k):
    """Split a scenario's steps into k consecutive sub-scenarios."""
    cut = np.linspace(0, len(sc.steps), k + 1).astype(int)
    out = []
    for a, b in zip(cut[:-1], cut[1:]):
        s = Scenario()
        s.steps = sc.steps[a:b]
        out.append(s)
    return out


def _rows(arr):
    return {bytes(r[:16]): bytes(r) for r in arr.view(np.uint8).reshape(-1, 128)}


def _changed(before, after):
    """Records of `after` that are new or differ from `before` (keyed by id)."""
    b, a = _rows(before), _rows(after)
    return {k: v for k, v in a.items() if b.get(k) != v}


def _posted(arr):
    return {int(ts): int(f) for ts, f in np.asarray(arr, dtype=np.uint64).reshape(-1, 2)}


@pytest.mark.parametrize("devices", [None, (0, 0)], ids=["single", "node2"])
@pytest.mark.parametrize("config", ["mixed", "two_phase", "chains", "limits"])
def test_checkpoint_deltas(config, devices, gpu_engine_factory):
    sc = make_scenario(99 + sum(map(ord, config)), **CONFIGS[config])
    oracle, engine = OracleEngine(), gpu_engine_factory(**(dict(devices=devices) if devices else {}))
    forest_a, forest_t, forest_p = {}, {}, {}
    prev = (oracle.export_accounts(), oracle.export_transfers(), oracle.export_posted())
    for seg in _segments(sc, 3):
        run_oracle(seg, oracle)
        run_oracle(seg, engine)
        d = engine.checkpoint_delta()
        now = (oracle.export_accounts(), oracle.export_transfers(), oracle.export_posted())
        # Exactly the changed objects, in the documented order.
        assert _rows(d.accounts) == _changed(prev[0], now[0])
        assert _rows(d.transfers) == _changed(prev[1], now[1])
        p_prev, p_now = _posted(prev[2]), _posted(now[2])
        assert _posted(d.posted) == {k: v for k, v in p_now.items() if p_prev.get(k) != v}
        # The forest's previous balances of every re-balanced account (zero for new ones): what a
        # groove upsert diffs its balance index trees against.
        old_rows = _rows(prev[0])
        for rec, before in zip(d.accounts.view(np.uint8).reshape(-1, 128), d.accounts_before):
            old = old_rows.get(bytes(rec[:16]))
            want = np.frombuffer(old[16:80], dtype=np.uint64) if old else np.zeros(8, dtype=np.uint64)
            assert np.array_equal(before, want)
        ids = [bytes(r[:16]) for r in d.accounts.view(np.uint8).reshape(-1, 128)]
        assert len(ids) == len(set(ids))  # each account once (no particular order: the groove sorts)
        ts = d.transfers["timestamp"] if len(d.transfers) else np.array([], dtype=np.uint64)
        assert np.all(np.diff(ts.astype(np.int64)) > 0)
        # Replay into the host forest (insert / upsert).
        forest_a.update(_rows(d.accounts))
        forest_t.update(_rows(d.transfers))
        forest_p.update(_posted(d.posted))
        prev = now
    assert forest_a == _rows(prev[0])
    assert forest_t == _rows(prev[1])
    assert forest_p == _posted(prev[2])
    # Nothing committed since: an empty write-back.
    d = engine.checkpoint_delta()
    assert len(d.accounts) == len(d.transfers) == len(d.posted) == 0


def test_checkpoint_after_reset(gpu_engine_factory):
    sc = make_scenario(5, **CONFIGS["mixed"])
    engine = gpu_engine_factory()
    run_oracle(sc, engine)
    engine.checkpoint_delta()
    engine.reset()
    run_oracle(sc, engine)
    d = engine.checkpoint_delta()  # everything again: the reset state is the empty state
    assert _rows(d.accounts) == _rows(engine.export_accounts())
    assert _rows(d.transfers) == _rows(engine.export_transfers())


def _warm(engine, op, events, forest_a, forest_t, forest_p):
    """The restart path of the reference-side wrapper (zig/state_machine_gpu.zig prefetch): load the
    objects a prepare reads that the forest holds (src/state_machine.zig:419-467: the event ids, the
    pending transfer and its posted entry, the debit / credit accounts); the engine keeps the ones
    it already has."""
    from tigerbeetle_amd.types import TransferFlags as TF
    acc_ids, xfer_ids = set(), set()
    for ev in events:
        ev = bytes(ev)
        if op == 128:
            acc_ids.add(ev[:16])
            continue
        xfer_ids.add(ev[:16])
        flags = int.from_bytes(ev[118:120], "little")
        acc_ids.update((ev[16:32], ev[32:48]))
        if flags & (TF.post_pending_transfer | TF.void_pending_transfer):
            xfer_ids.add(ev[64:80])
            p = forest_t.get(ev[64:80])
            if p is not None:
                acc_ids.update((p[16:32], p[32:48]))
    accts = [forest_a[k] for k in sorted(acc_ids) if k in forest_a]
    xfers = [forest_t[k] for k in sorted(xfer_ids) if k in forest_t]
    states = [1 + forest_p[int.from_bytes(x[120:128], "little")] if int.from_bytes(x[120:128], "little") in forest_p
              else 0 for x in xfers]
    if accts:
        engine.load_accounts(np.frombuffer(b"".join(accts), dtype=np.uint8).view(ACCOUNT_DTYPE))
    if xfers:
        engine.load_transfers(np.frombuffer(b"".join(xfers), dtype=np.uint8).view(TRANSFER_DTYPE), states)


@pytest.mark.parametrize("config", ["mixed", "two_phase", "chains", "limits"])
def test_restart_from_forest(config, gpu_engine_factory):
    """A replica restart: the engine's objects reach the forest by write-back, the process dies, a
    new engine starts empty (commit_timestamp from the checkpoint) and the rest of the history is
    committed with prefetch loading what each prepare reads from the forest.  Every reply equals
    the oracle's (which never restarted), and forest + the new engine's objects equal its grooves."""
    sc = make_scenario(313 + sum(map(ord, config)), **CONFIGS[config])
    assert all(step[0] == "commit" for step in sc.steps)
    first, second = _segments(sc, 2)
    oracle, engine = OracleEngine(), gpu_engine_factory()
    assert run_oracle(first, oracle) == run_oracle(first, engine)
    d = engine.checkpoint_delta()
    forest_a, forest_t, forest_p = _rows(d.accounts), _rows(d.transfers), _posted(d.posted)
    checkpoint_ts = engine.commit_timestamp
    engine.close()

    engine = gpu_engine_factory()
    engine.set_commit_timestamp(checkpoint_ts)
    for _, op, ts, events in second.steps:
        _warm(engine, op, events, forest_a, forest_t, forest_p)
        body = b"".join(events)
        assert engine.commit(op, ts, body) == oracle.commit(op, ts, body)
    accounts = dict(forest_a)
    accounts.update(_rows(engine.export_accounts()))
    transfers = dict(forest_t)
    transfers.update(_rows(engine.export_transfers()))
    posted = dict(forest_p)
    posted.update(_posted(engine.export_posted()))
    assert accounts == _rows(oracle.export_accounts())
    assert transfers == _rows(oracle.export_transfers())
    assert posted == _posted(oracle.export_posted())
    assert engine.commit_timestamp == oracle.commit_timestamp

    # The restarted engine's next write-back: loaded objects are not new, re-balanced ones carry
    # the forest's balances as `before`, and applying it (insert / upsert) rebuilds the oracle.
    d = engine.checkpoint_delta()
    for rec, before in zip(d.accounts.view(np.uint8).reshape(-1, 128), d.accounts_before):
        key = bytes(rec[:16])
        if int.from_bytes(bytes(rec[120:128]), "little") > d.created_after:
            assert key not in forest_a and not before.any()  # groove insert
        else:
            assert np.array_equal(before, np.frombuffer(forest_a[key][16:80], dtype=np.uint64))  # upsert
    new_t = _rows(d.transfers)
    assert not set(new_t) & set(forest_t)  # every transfer in the delta is a groove insert
    forest_a.update(_rows(d.accounts))
    forest_t.update(new_t)
    forest_p.update(_posted(d.posted))
    assert forest_a == _rows(oracle.export_accounts())
    assert forest_t == _rows(oracle.export_transfers())
    assert forest_p == _posted(oracle.export_posted())
