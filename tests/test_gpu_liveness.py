"""tb_flow whose launch the device cannot hold at once (include/tbgpu.h "Device exclusivity",
k_flow.h fl_admit).

tb_flow separates its phases with a grid barrier, so its workgroups must run together. They used to
be the whole launch: a workgroup kept off the device (a co-tenant holding its CU) left the others
waiting at the first barrier, and the pass ended in PANIC_FLOW_STALL. Now the workgroups that
entered within the first one's admission window are the grid, and the later ones exit at once.
`tbgpu_bench_flow_launch` launches tb_flow with eight times as many workgroups as the device holds
together (one per CU), so most of every launch starts only after others finished: the old barrier
waited for all of them and stalled; admission must complete the pass with the ones it admitted."""
import time

import numpy as np
import pytest

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps
from tests.harness.oracle import OracleEngine
from tests.test_gpu_differential import assert_same_state
from tigerbeetle_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["c3", "c4"])
def test_flow_admits_the_workgroups_that_run(kind, gpu_engine_factory, monkeypatch):
    """C3 (limit accounts: bounds, sweep, walkers) and C4 (chains, two-phase: the ordered run)
    passes with tb_flow launched 8x over what the device holds, every wait bounded at 1 s: no
    stall, tb_flow ran, and replies and state equal the oracle's."""
    monkeypatch.setenv("TBGPU_STALL_MS", "1000")  # read by tbgpu_init
    n_acc, n_xfer, batch, chunk = 20_000, 160_000, 8190, 4
    engine = gpu_engine_factory(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=chunk * batch,
                                pass_batches_max=chunk)
    accts, xfers = generate(engine, kind, n_acc, n_xfer, seed=31)
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[kind]["gap_every"])
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    rb, _, _ = engine.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
    assert int(rb.sum()) == 0
    # tb_flow holds a CU per workgroup: 2048 workgroups are 8x the MI355X's 256 CUs
    _lib.check(engine.lib.tbgpu_bench_flow_launch(engine.h, 2048))
    host = np.ascontiguousarray(xfers)
    engine.register_host(host)
    t0 = time.perf_counter()
    try:
        rb, rep, _ = engine.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=chunk)
    finally:
        engine.unregister_host(host)
    dt = time.perf_counter() - t0
    off = 0
    for k, (L, nb) in enumerate(zip(x_lens, rb)):
        assert bytes(rep[off * 8:off * 8 + int(nb)]) == expected[k], "reply of prepare %d differs" % k
        off += L
    assert_same_state(oracle, engine)
    st = engine.stats()
    assert st["dependent_events"] > 0 and st["flow_passes"] > 0, st
    assert dt < 10, dt
