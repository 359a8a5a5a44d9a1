"""Bounded HBM residency (include/tbgpu.h tbgpu_evict_transfers / tbgpu_transfers_maybe_cold,
csrc/k_evict.h): a replica that commits several times the transfer log's capacity, writing each bar
back to its forest (tbgpu_checkpoint_delta), evicting what the forest holds, and loading back what
a prepare names (its prefetch: the reference's groove prefetch, src/state_machine.zig:419-467) —
every reply byte equal to the oracle's, which never evicts anything.  The workload names evicted
transfers on purpose: duplicate ids (exists, exists_with_different_*), posts and voids of old
pending transfers (and again: already_posted / already_voided), expiry."""
import numpy as np
import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import make_scenario
from tigerbeetle_amd.types import TRANSFER_DTYPE, TransferFlags

pytestmark = pytest.mark.gpu


def _ids(body):
    t = np.frombuffer(body, dtype=TRANSFER_DTYPE)
    ids = [(int(x["id_lo"]), int(x["id_hi"])) for x in t]
    pv = (t["flags"] & (TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)) != 0
    ids += [(int(x["pending_id_lo"]), int(x["pending_id_hi"])) for x in t[pv]]
    return list(dict.fromkeys(ids))


@pytest.mark.parametrize("devices", [None, (0, 0)], ids=["single", "node2"])
@pytest.mark.parametrize("behind", [False, True], ids=["sync", "behind"])
def test_commit_past_the_log_with_eviction(behind, devices, gpu_engine_factory):
    """behind: the Zig wrapper's engine_write_back_behind shape — each bar's delta captured
    asynchronously and delivered to the forest while the next bar commits (its posts and voids of
    the previous bars' pending transfers included); eviction is refused while a delta is in flight
    and while any commit is unwritten, so the wrapper writes a bar back synchronously when the log
    is three-quarters full and evicts then (an eviction one bar behind could drop a
    pending transfer the bar in flight posts).

    node2: a node of two logical shards (include/tbgpu.h: every home shard evicts from its own log and
    answers the cold queries of the ids it homes; the node's write-back merges the shards)."""
    from tigerbeetle_amd._lib import EngineError
    if devices:
        engine = gpu_engine_factory(accounts_max=4096, transfers_max=1 << 14, pass_events_max=2048, pass_batches_max=16,
                                    devices=devices)
        n_batches = 520
    else:
        engine = gpu_engine_factory(accounts_max=4096, transfers_max=1 << 14, pass_events_max=8192, pass_batches_max=16)
        n_batches = 320
    cap = engine.stats()["log_capacity"]
    sc = make_scenario(2024, n_accounts=64, n_transfer_batches=n_batches, batch_len=(100, 400), p_pending=0.3,
                       p_post_void=0.25, p_dup=0.08, p_linked=0.05, p_limit=0.05, p_balancing=0.02, p_invalid=0.03,
                       id_space=1 << 40)
    oracle = OracleEngine(4096, 1 << 18)
    forest, forest_posted = {}, {}  # the durable copy, built from the write-backs only
    loads = evictions = committed = refused = 0
    codes = set()
    bar = 16
    inflight = False

    def apply(d):
        for rec in d.transfers:
            key = (int(rec["id_lo"]), int(rec["id_hi"]))
            forest[key] = rec.tobytes()
        for pts, voided in d.posted:
            forest_posted[int(pts)] = 2 if voided else 1

    for k, (_, op, ts, events) in enumerate(sc.steps):
        body = b"".join(events)
        if op == 129:
            ids = _ids(body)
            arr = np.array([[lo, hi] for lo, hi in ids], dtype=np.uint64).reshape(-1, 2)
            cold = engine.transfers_maybe_cold(arr)
            recs = [forest[i] for i, c in zip(ids, cold) if c and i in forest]
            if recs:
                r = np.frombuffer(b"".join(recs), dtype=TRANSFER_DTYPE)
                states = np.array([forest_posted.get(int(t), 0) for t in r["timestamp"]], dtype=np.uint8)
                engine.load_transfers(r, states)
                loads += len(recs)
        expected = oracle.commit(op, ts, body)
        assert engine.commit(op, ts, body) == expected, "prepare %d differs" % k
        if op == 129:
            committed += len(events)
            codes.update(np.frombuffer(expected, dtype=np.uint32)[1::2].tolist())
        if k % bar == bar - 1:
            full = engine.stats()["log_used"] > cap // 2
            if behind and inflight:
                with pytest.raises(EngineError):  # a delta in flight
                    engine.evict_transfers(cap // 4)
                apply(engine.checkpoint_delta_wait())
                inflight = False
                with pytest.raises(EngineError):  # this bar's commits are not written back
                    engine.evict_transfers(cap // 4)
                refused += 2
            if behind and not full:
                engine.checkpoint_delta_async((1 << 14, 1 << 14, 1 << 14))
                inflight = True
                continue
            apply(engine.checkpoint_delta())
            if full:
                evictions += engine.evict_transfers(cap // 4)
    if inflight:
        apply(engine.checkpoint_delta_wait())
    st = engine.stats()
    assert committed > 3 * cap and st["log_capacity"] == cap
    if devices:
        assert st["node_passes_split"] > 0  # the sequencer's passes ran against evicted homes too
    assert evictions > 0 and st["transfers_evicted"] == evictions and loads > 0
    assert refused > 0 or not behind
    # The evicted transfers were named again: duplicates and two-phase results against them.
    assert 46 in codes or any(c in codes for c in range(36, 46)), codes  # exists / exists_with_different_*
    assert 33 in codes or 34 in codes, codes  # already posted / voided
    assert engine.commit_timestamp == oracle.commit_timestamp
