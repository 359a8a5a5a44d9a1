"""The replica's call shape on a node engine (VERDICT r3 What's weak #8): one C2 prepare of 8190
transfers per tbgpu_commit, from registered host memory, on N logical shards of one GPU (the same
kernels and peer reads as N devices, inside one HBM) and on a single engine for comparison.  Prints
one JSON line per engine: transfers/s and per-call latency percentiles (host clock).

usage: python tools/gpu/node_one_prepare.py [prepares] [shards]
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

from tests.harness.configs import KINDS, batches, timestamps  # noqa: E402
from tigerbeetle_amd import _lib  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

n_prep = int(sys.argv[1]) if len(sys.argv) > 1 else 400
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n_acct, batch = 1_000_000, 8190
n_xfer = n_prep * batch


def run(devices):
    e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer + 1024, pass_events_max=64 * batch,
                       pass_batches_max=64, devices=devices))
    acct = e.alloc(n_acct * 128)
    e.generate_accounts(acct, 0, n_acct, seed=42)
    a_host = e.to_host(acct, n_acct * 128)
    e.free(acct)
    a_lens = batches(n_acct, batch)
    a_ts, t = timestamps(a_lens, 1_000_000_000)
    rb, _, _ = e.commit_pipelined(128, a_ts, a_lens, a_host, chunk_batches=64)
    assert int(rb.sum()) == 0
    ev = e.alloc(n_xfer * 128)
    e.generate_transfers(ev, 0, n_xfer, n_acct, seed=42, kind=KINDS["c2"])
    body = e.to_host(ev, n_xfer * 128)
    e.free(ev)
    e.register_host(body)
    lat = []
    out = np.zeros(batch * 8, dtype=np.uint8)
    n = ctypes.c_uint32(0)
    ts = t + 10
    warm = 20
    for k in range(n_prep):
        ts += batch
        view = body[k * batch * 128:(k + 1) * batch * 128]
        if k == warm:
            t0 = time.perf_counter()
        c0 = time.perf_counter()
        # the body straight from the registered buffer, as the replica's message pool
        _lib.check(e.lib.tbgpu_commit(e.h, 129, ts, view.ctypes.data, view.nbytes, out.ctypes.data, out.nbytes,
                                      ctypes.byref(n)))
        lat.append(time.perf_counter() - c0)
        assert n.value == 0, "C2 transfers all succeed"
    total = time.perf_counter() - t0
    e.unregister_host(body)
    st = e.stats()
    e.close()
    ms = np.sort(np.array(lat[warm:]) * 1e3)
    return {"engine": "node, %d logical shards" % len(devices) if len(devices) > 1 else "single",
            "prepares": n_prep - warm, "transfers_per_s": round((n_prep - warm) * batch / total, 1),
            "p50_ms": round(float(ms[len(ms) // 2]), 4), "p99_ms": round(float(ms[int(len(ms) * 0.99)]), 4),
            "passes_clean": st.get("node_passes_clean"), "passes_split": st.get("node_passes_split")}


for devs in ((0,), tuple([0] * shards)):
    print(json.dumps(run(devs)), flush=True)
