"""Zero-copy commits (include/tbgpu.h tbgpu_log_window): prepares placed at the engine's next
transfer-log positions and committed there (PassArgs.inplace: a committed create's record is its
event with the timestamp written; a post / void's is composed over it; the ordered path stores its
own).  Every dependency class of the differential workloads, several prepares per call, against
the oracle byte for byte — replies, accounts, transfers, the posted groove, commit_timestamp — and
a C2-sized call (the legs path) against the same call committed from a separate buffer."""
import numpy as np
import pytest

from tests.harness.configs import KINDS, batches, timestamps
from tests.harness.oracle import OracleEngine, OraclePanic
from tests.harness.workload import make_scenario, run_oracle
from tests.test_gpu_differential import CONFIGS, assert_same_state
from tigerbeetle_amd._lib import EnginePanic

pytestmark = pytest.mark.gpu


def run_inplace(sc, engine, per_call=4):
    """The scenario with its create_transfers prepares committed in place, up to `per_call` a call."""
    cap = sum(sum(len(e) for e in s[3]) // 128 for s in sc.steps if s[0] != "setup" and s[1] == 129) + 1
    res_dev = engine.alloc(max(cap, 1) * 8)
    rb_dev = engine.alloc(per_call * 4)
    replies, group = [], []

    def flush():
        if not group:
            return
        bodies = [b"".join(g[3]) for g in group]
        lens = [len(b) // 128 for b in bodies]
        n = sum(lens)
        if n == 0:
            for _ in group:
                replies.append(b"")
            group.clear()
            return
        window = engine.log_window(n)
        engine.to_device(window, np.frombuffer(b"".join(bodies), dtype=np.uint8))
        engine.commit_device_async(129, [g[2] for g in group], lens, window, res_dev, rb_dev)
        engine.sync()
        rb = engine.to_host(rb_dev, len(group) * 4).view(np.uint32)
        res = engine.to_host(res_dev, n * 8)
        off = 0
        for L, nb in zip(lens, rb):
            replies.append(bytes(res[off * 8:off * 8 + int(nb)]))
            off += L
        group.clear()

    try:
        for step in sc.steps:
            if step[0] == "setup":
                flush()
                engine.set_balances(*step[1:])
            elif step[1] == 129:
                group.append(step)
                if len(group) == per_call:
                    flush()
            else:
                flush()
                replies.append(engine.commit(step[1], step[2], b"".join(step[3])))
        flush()
    finally:
        engine.free(res_dev)
        engine.free(rb_dev)
    return replies


@pytest.mark.parametrize("config", sorted(CONFIGS))
def test_inplace_matches_oracle(config, gpu_engine_factory):
    cfg = dict(CONFIGS[config])
    cfg.setdefault("n_transfer_batches", 12)
    sc = make_scenario(7100 + sorted(CONFIGS).index(config), **cfg)
    oracle = OracleEngine(4096, 1 << 17)
    engine = gpu_engine_factory(pass_events_max=8192, pass_batches_max=4)
    try:
        expected = run_oracle(sc, oracle)
    except OraclePanic:
        with pytest.raises(EnginePanic):
            run_inplace(sc, engine)
        return
    actual = run_inplace(sc, engine)
    assert len(actual) == len(expected)
    for k, (e, a) in enumerate(zip(expected, actual)):
        assert e == a, "reply of prepare %d differs" % k
    assert_same_state(oracle, engine)


def test_log_window_bounds(gpu_engine_factory):
    engine = gpu_engine_factory(transfers_max=1 << 12)
    w0 = engine.log_window(16)
    assert w0 == engine.log_window(1 << 12)  # the whole log, from the next position
    with pytest.raises(Exception):
        engine.log_window((1 << 12) + 1)


@pytest.mark.parametrize("kind", ["c2", "c4"])
def test_inplace_pass_equals_copy(kind, gpu_engine_factory):
    """A 64-prepare C2 / C4 call (C2: the balance-legs path) in place and from a separate buffer:
    the same replies, accounts, transfers and posted groove."""
    n_acc, batch, nb = 50_000, 8190, 64
    n = batch * nb
    out = []
    for inplace in (False, True):
        e = gpu_engine_factory(accounts_max=n_acc, transfers_max=n + 1024, pass_events_max=n, pass_batches_max=nb)
        acct = e.alloc(n_acc * 128)
        e.generate_accounts(acct, 0, n_acc, seed=3)
        a_lens = batches(n_acc, batch)
        a_ts, t = timestamps(a_lens, 10**12)
        a_res, a_rb = e.alloc(n_acc * 8), e.alloc(len(a_lens) * 4)
        e.commit_device_async(128, a_ts, a_lens, acct, a_res, a_rb)
        e.sync()
        lens = [batch] * nb
        ts, _ = timestamps(lens, t + 10)
        dst = e.log_window(n) if inplace else e.alloc(n * 128)
        e.generate_transfers(dst, 0, n, n_acc, seed=5, kind=KINDS[kind])
        res, rb = e.alloc(n * 8), e.alloc(nb * 4)
        e.commit_device_async(129, ts, lens, dst, res, rb)
        e.sync()
        r = e.to_host(rb, nb * 4).view(np.uint32).copy()
        replies = [bytes(x) for x in np.split(e.to_host(res, n * 8), nb)]
        replies = [rep[:int(b)] for rep, b in zip(replies, r)]
        out.append((replies, e.export_accounts().tobytes(), e.export_transfers().tobytes(), e.export_posted().tobytes(),
                    e.commit_timestamp, e.stats()["transfers"]))
    assert out[0] == out[1]
    assert out[0][5] > 0
