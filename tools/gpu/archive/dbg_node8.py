"""Diagnose node parity at many shards: commit a generated BASELINE shape on nodes of several
(shards, chunk) shapes and report, per shape, whether replies / accounts / transfers equal the
oracle's, and for extra or missing transfers: their reply codes, home shard and flags.
Usage: python tools/gpu/dbg_node8.py c3 1000000 8:16 4:16 8:64"""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DBG_Q", "8")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from tests.harness.configs import SETTINGS, batches, generate, split, timestamps  # noqa: E402
from tests.harness.oracle import OracleEngine  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402


def main():
    config, n_xfer = sys.argv[1], int(sys.argv[2])
    shapes = [tuple(map(int, a.split(":"))) for a in sys.argv[3:]]
    n_acc, batch = 1_000_000, 8190
    gen_engine = Engine(Options(accounts_max=n_acc, transfers_max=1 << 16, pass_events_max=8192, pass_batches_max=1))
    accts, xfers = generate(gen_engine, config, n_acc, n_xfer, seed=31)
    gen_engine.close()
    a_lens, x_lens = batches(n_acc, batch), batches(n_xfer, batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[config]["gap_every"])
    oracle = OracleEngine(n_acc, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, x_ts, split(xfers, x_lens))
    t_o = oracle.export_transfers()
    ids_o = set(zip(t_o["id_lo"].tolist(), t_o["id_hi"].tolist()))
    x = xfers.view(np.dtype([("id_lo", "<u8"), ("id_hi", "<u8"), ("rest", "V112")]))
    code_of = {}
    off = 0
    for L, r in zip(x_lens, expected):
        rr = np.frombuffer(r, dtype=np.uint32).reshape(-1, 2)
        for i, c in rr:
            code_of[off + int(i)] = int(c)
        off += L
    for shards, chunk in shapes:
        e = Engine(Options(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=chunk * batch,
                           pass_batches_max=chunk, devices=(0,) * shards))
        rb, _, _ = e.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=chunk)
        assert int(rb.sum()) == 0
        host = np.ascontiguousarray(xfers)
        e.register_host(host)
        rb, rep, _ = e.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=chunk)
        e.unregister_host(host)
        got, off = [], 0
        for L, nb in zip(x_lens, rb):
            got.append(bytes(rep[off * 8:off * 8 + int(nb)]))
            off += L
        bad = [k for k, (a, b) in enumerate(zip(expected, got)) if a != b]
        t_g = e.export_transfers()
        ids_g = list(zip(t_g["id_lo"].tolist(), t_g["id_hi"].tolist()))
        extra = [i for i in ids_g if i not in ids_o]
        dup = len(ids_g) - len(set(ids_g))
        missing = len(ids_o - set(ids_g))
        st = e.stats()
        led = e.ledger_summary()
        accs_eq = e.export_accounts().tobytes() == oracle.export_accounts().tobytes()
        print("shape %d:%d replies_bad=%d first=%s transfers o=%d g=%d extra=%d dup=%d missing=%d accounts_eq=%s "
              "split=%d whole=%d seq=%d stray=%d" % (shards, chunk, len(bad), bad[:5], len(t_o), len(t_g), len(extra),
                                                     dup, missing, accs_eq, st["node_passes_split"],
                                                     st["node_passes_whole"], st["node_sequenced_events"],
                                                     led["stray"]), flush=True)
        if extra:
            pos = {(int(a), int(b)): k for k, (a, b) in enumerate(zip(x["id_lo"], x["id_hi"]))}
            ev = [pos.get(i, -1) for i in extra[:2000]]
            codes = {}
            for k in ev:
                c = code_of.get(k, 0)
                codes[c] = codes.get(c, 0) + 1
            passes = {}
            per = shards * chunk * batch
            for k in ev:
                passes[k // per] = passes.get(k // per, 0) + 1
            print("  extra events: codes %s, by pass %s, first events %s" % (codes, sorted(passes.items())[:20], ev[:10]),
                  flush=True)
        e.close()


if __name__ == "__main__":
    main()
