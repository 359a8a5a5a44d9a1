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


@pytest.mark.parametrize("config", ["mixed", "two_phase", "chains", "limits"])
def test_checkpoint_deltas(config, gpu_engine_factory):
    sc = make_scenario(99 + sum(map(ord, config)), **CONFIGS[config])
    oracle, engine = OracleEngine(), gpu_engine_factory()
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
        ids = [bytes(r[:16])[::-1] for r in d.accounts.view(np.uint8).reshape(-1, 128)]
        assert ids == sorted(ids)
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
