"""BASELINE.json configs[4] ("C5": 100M accounts hash-partitioned, uniform transfers, cross-shard
legs) at its full account count, on the GPU box's one GPU.

* The node engine (include/tbgpu.h tbgpu_config.devices, csrc/node.h) with two logical shards on
  cuda:0: 100M accounts created through the C ABI (each on its owner shard only: every shard's account
  table is half of a single engine's), then a sample
  of 64 prepares compared byte for byte with the oracle — the oracle holds exactly the accounts the
  sample touches, built from the generator's records and the create timestamps, not from the GPU —
  then two full passes of 2 x 256 prepares (every source block full: 512 prepares, 4.19M transfers
  per pass) with the size-independent properties: every reply empty, every transfer stored once,
  debits == credits (pending and posted), no balance on a shard that does not own its account.
* The per-process protocol over RCCL at one rank (bench.py --engine ranks --sharded, backend nccl)
  at the same account count and one full 512-prepare pass, with the same properties."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.harness.configs import batches, split, timestamps
from tests.harness.oracle import OracleEngine
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_ACCOUNTS = 100_000_000
BATCH = 8190


def test_c5_node_full_size():
    from tigerbeetle_amd.state_machine import Engine, Options

    chunk, sample_prepares, passes = 256, 64, 2
    n_xfer = sample_prepares * BATCH + passes * 2 * chunk * BATCH
    engine = Engine(Options(accounts_max=N_ACCOUNTS, transfers_max=n_xfer, pass_events_max=chunk * BATCH,
                            pass_batches_max=chunk, devices=(0, 0)))
    try:
        # Transfers first (the generator needs only the account count): the sample's accounts.
        gen = engine.alloc(n_xfer * 128)
        engine.generate_transfers(gen, 0, n_xfer, N_ACCOUNTS, seed=5)
        xfers = engine.to_host(gen, n_xfer * 128)
        engine.free(gen)
        x = xfers.view(TRANSFER_DTYPE)
        n_sample = sample_prepares * BATCH
        # Account ids are IdPermutation.inversion (maxInt(u128) - (index + 1)): one common high word.
        H = x["debit_account_id_hi"][0]
        assert (x["debit_account_id_hi"][:n_sample] == H).all() and (x["credit_account_id_hi"][:n_sample] == H).all()
        ref = np.unique(np.concatenate([x["debit_account_id_lo"][:n_sample], x["credit_account_id_lo"][:n_sample]]))

        # 100M accounts through the node (sequenced create_accounts, each to its owner), in chunks of 2048
        # prepares;
        # the oracle gets the sample's accounts as created (generator record + create timestamp).
        a_lens = batches(N_ACCOUNTS, BATCH)
        a_ts, t = timestamps(a_lens, 10**9)
        oracle_accts = []
        a_chunk = 2048 * BATCH
        dev = engine.alloc(a_chunk * 128)
        for a0 in range(0, N_ACCOUNTS, a_chunk):
            n_a = min(a_chunk, N_ACCOUNTS - a0)
            engine.generate_accounts(dev, a0, n_a, seed=5)
            host = engine.to_host(dev, n_a * 128)
            k0 = a0 // BATCH
            lens = batches(n_a, BATCH)
            rb, _, _ = engine.commit_pipelined(128, a_ts[k0:k0 + len(lens)], lens, host, chunk_batches=chunk)
            assert int(rb.sum()) == 0
            recs = host.view(ACCOUNT_DTYPE).copy()
            hit = np.isin(recs["id_lo"], ref) & (recs["id_hi"] == H)
            idx = np.nonzero(hit)[0]
            k = k0 + idx // BATCH
            j = idx % BATCH
            L = np.asarray(a_lens, dtype=np.uint64)[k]
            recs["timestamp"][idx] = np.asarray(a_ts, dtype=np.uint64)[k] - L + 1 + j.astype(np.uint64)
            oracle_accts.append(recs[idx])
        engine.free(dev)
        oracle_accts = np.concatenate(oracle_accts)
        assert len(oracle_accts) == len(ref)

        # The sample: byte for byte against the oracle.
        x_lens = batches(n_xfer, BATCH)
        x_ts, _ = timestamps(x_lens, t + 10)
        oracle = OracleEngine(len(ref) + 16, n_sample)
        oracle.upsert_accounts(oracle_accts)
        s_lens, s_ts = x_lens[:sample_prepares], x_ts[:sample_prepares]
        expected = oracle.commit_many(129, s_ts, split(xfers[:n_sample * 128], s_lens))
        host = np.ascontiguousarray(xfers)
        engine.register_host(host)
        rb, rep, _ = engine.commit_pipelined(129, s_ts, s_lens, host[:n_sample * 128], chunk_batches=chunk)
        got, off = [], 0
        for Ls, nb in zip(s_lens, rb):
            got.append(bytes(rep[off * 8:off * 8 + int(nb)]))
            off += Ls
        assert got == expected
        ids = np.stack([oracle_accts["id_lo"], oracle_accts["id_hi"]], axis=1)
        mine, found = engine.fetch_accounts(ids)
        theirs, _ = oracle.fetch_accounts(ids)
        assert found.all() and mine.tobytes() == theirs.tobytes()
        assert engine.export_transfers().tobytes() == oracle.export_transfers().tobytes()

        # Two full passes of 2 x 256 prepares: size-independent properties.
        rest_lens, rest_ts = x_lens[sample_prepares:], x_ts[sample_prepares:]
        rb, _, _ = engine.commit_pipelined(129, rest_ts, rest_lens, host[n_sample * 128:], chunk_batches=chunk)
        engine.unregister_host(host)
        assert int(rb.sum()) == 0
        st = engine.stats()
        assert st["transfers"] == n_xfer and st["dependent_events"] == 0
        # Partitioned records: each shard's account table holds its own half of the ledger (plus one
        # routed sub-pass's imports), half of what one engine holding all 100M accounts allocates.
        single = (1 << 28) * (32 + 64 + 32 + 4)  # pow2(2 x 100M) slots x (hot, balances, cold, mark)
        shard_bytes = st["node_shard_account_bytes"][:2]
        assert all(0 < b <= single // 2 for b in shard_bytes), (shard_bytes, single)
        assert st["accounts"] == N_ACCOUNTS
        s = engine.ledger_summary()
        assert s["accounts"] == N_ACCOUNTS and s["stray"] == 0
        assert (x["amount_hi"] == 0).all()
        assert s["debits_posted"] == s["credits_posted"] == int(x["amount_lo"].sum(dtype=np.uint64))
        assert s["debits_pending"] == s["credits_pending"] == 0
    finally:
        engine.close()


def test_c5_rccl_one_rank_full_size():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--engine", "ranks", "--sharded", "--dist-backend", "nccl", "--accounts", str(N_ACCOUNTS),
           "--transfers", str(512 * BATCH), "--steps", "1", "--warmup", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["parity"]["full_run_properties"] is True
    assert line["passes"]["clean"] == 1 and line["passes"]["dirty"] == 0
