"""Multi-rank sharding at world_size 2 over gloo on CPU: the collective protocol
of tigerbeetle_amd.sharded (routed clean passes, dirty-pass prefetch -> scratch commit ->
write-back, replicated create_accounts, merged exports) with the oracle-backed test double of the
per-rank backend, checked against one oracle committing the concatenated prepares."""
import json
import socket
import time

import pytest
import torch.multiprocessing as mp

from tests.harness.shard_runner import run_rank


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(tmp_path, kind, world, scenario_kw, max_prepares=4, timeout=300, dist_backend="gloo"):
    """Run the scenario on `world` ranks; a rank that dies or hangs fails the test (all ranks are
    killed at the deadline, never left waiting in a collective)."""
    out = tmp_path / "verdict.json"
    ctx = mp.spawn(run_rank, args=(world, free_port(), kind, scenario_kw, max_prepares, str(out), dist_backend),
                   nprocs=world, join=False)
    deadline = time.monotonic() + timeout
    try:
        while not ctx.join(timeout=1.0):
            if time.monotonic() > deadline:
                raise TimeoutError("sharded run exceeded %d s" % timeout)
    finally:
        for p in ctx.processes:
            if p.is_alive():
                p.kill()
    return json.loads(out.read_text())


CLEAN = dict(p_limit=0.0, p_linked=0.0, p_pending=0.0, p_post_void=0.0, p_balancing=0.0)


@pytest.mark.parametrize("seed", [1, 2])
def test_sharded_clean_passes(tmp_path, seed):
    v = run_world(tmp_path, "oracle", 2, dict(seed=seed, n_accounts=48, n_transfer_batches=8, **CLEAN))
    assert v["ok"], v["problems"]
    assert v["clean"] > 0 and v["dirty"] == 0 and v["split"] == 0


@pytest.mark.parametrize("seed", [3, 4])
def test_sharded_mixed_passes(tmp_path, seed):
    v = run_world(tmp_path, "oracle", 2, dict(seed=seed, n_accounts=48, n_transfer_batches=10))
    assert v["ok"], v["problems"]
    assert v["split"] > 0 and v["dirty"] == 0  # dependent subsequences sequenced, no whole-pass gather


def test_sharded_clean_then_dirty_interleaved(tmp_path):
    # Single-prepare passes: some clean, some dirty; effects of dirty passes (new transfers at their
    # homes, posted states, collected balances) must be visible to later clean passes.
    v = run_world(tmp_path, "oracle", 2, dict(seed=11, n_accounts=32, n_transfer_batches=14, p_linked=0.02,
                                              p_pending=0.3, p_post_void=0.1, p_balancing=0.0, p_limit=0.0),
                  max_prepares=1)
    assert v["ok"], v["problems"]
    assert v["clean"] > 0 and v["split"] > 0


@pytest.mark.parametrize("seed", [31, 32])
def test_sharded_dependent_kinds(tmp_path, seed):
    # Every dependency class in split passes: chains (with chain-breaking and open chains), limit
    # accounts, balancing (its accounts marked pass-wide), two-phase in the same and later passes,
    # duplicate ids across ranks (demoted to the sequencer), invalid events.
    v = run_world(tmp_path, "oracle", 2, dict(seed=seed, n_accounts=24, n_transfer_batches=12, p_linked=0.25,
                                              p_limit=0.3, p_balancing=0.1, p_pending=0.4, p_post_void=0.3,
                                              p_dup=0.15, id_space=400))
    assert v["ok"], v["problems"]
    assert v["split"] > 0 and v["demoted"] > 0


def test_sharded_three_ranks_split(tmp_path):
    v = run_world(tmp_path, "oracle", 3, dict(seed=33, n_accounts=32, n_transfer_batches=9, p_linked=0.15,
                                              p_post_void=0.2, p_pending=0.3), max_prepares=3)
    assert v["ok"], v["problems"]
    assert v["split"] > 0


def test_sharded_near_overflow_balances(tmp_path):
    v = run_world(tmp_path, "oracle", 2, dict(seed=5, n_accounts=32, n_transfer_batches=6, near_overflow=True,
                                              **CLEAN))
    assert v["ok"], v["problems"]


def test_sharded_huge_amounts_fresh_balances(tmp_path):
    # Amounts near 2^127 on zero balances: a rank's saturated S must make the pass dirty (no
    # certificate), so the overflow checks run in order on the scratch engine.
    v = run_world(tmp_path, "oracle", 2, dict(seed=9, n_accounts=16, n_transfer_batches=6, p_huge=0.08, **CLEAN))
    assert v["ok"], v["problems"]
