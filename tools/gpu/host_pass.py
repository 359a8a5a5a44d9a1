"""C2 commits from registered host memory (the bench's `host_path` leg: tbgpu_commit_pipelined,
64-prepare chunks, three in flight), for the PMC passes of that leg (tools/gpu/profile.sh
hkt|hfetch|hwrite) without the device-resident leg's kernels in the same trace.

usage: python tools/gpu/host_pass.py [transfers] [chunk_prepares]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

from tests.harness.configs import KINDS, batches, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

n_xfer = int(sys.argv[1]) if len(sys.argv) > 1 else 20_962_400
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n_acct, batch = 1_000_000, 8190
# Tables sized as the headline engine (100M transfers: a 2-GB index), whatever this run commits.
e = Engine(Options(accounts_max=n_acct, transfers_max=max(n_xfer, 100_000_000), pass_events_max=chunk * batch,
                   pass_batches_max=chunk))
a_lens = batches(n_acct, batch)
a_ts, t = timestamps(a_lens, 1_000_000_000)
acct = e.alloc(n_acct * 128)
e.generate_accounts(acct, 0, n_acct, seed=42)
res = e.alloc(n_acct * 8)
rb = e.alloc((n_acct // batch + 2) * 4)
e.commit_device_async(128, a_ts, a_lens, acct, res, rb)
e.sync()
ev = e.alloc(n_xfer * 128)
e.generate_transfers(ev, 0, n_xfer, n_acct, seed=42, kind=KINDS["c2"])
host = e.to_host(ev, n_xfer * 128)
e.free(ev)
e.register_host(host)
x_lens = batches(n_xfer, batch)
x_ts, _ = timestamps(x_lens, t + 10)
out_lens, _, _ = e.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=chunk)
e.unregister_host(host)
print("host passes of %d prepares: %d transfers, reply bytes %d" % (chunk, n_xfer, int(np.asarray(out_lens).sum())))
e.close()
