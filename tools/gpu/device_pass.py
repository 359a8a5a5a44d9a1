"""C2 commits with the prepares already resident in HBM (no host copies in flight), for PMC passes
that must see the pass kernels' own HBM traffic only (tools/gpu/profile.sh dfetch|dwrite): under
rocprofv3 the runtime copies host prepares with a blit kernel whose writes to the staging buffer
are evicted from L2 during the next kernel and counted there.

usage: python tools/gpu/device_pass.py [transfers] [pass_prepares] [inplace]
  inplace 1 (default): the prepares are generated at their transfer-log positions and committed in
  place (tbgpu_log_window: the headline's path); 0: from a separate HBM buffer (the copy commit).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

from tests.harness.configs import KINDS, batches, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

n_xfer = int(sys.argv[1]) if len(sys.argv) > 1 else 20_971_200
pb = int(sys.argv[2]) if len(sys.argv) > 2 else 512
inplace = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n_acct, batch = 1_000_000, 8190
# Tables sized as the headline engine (100M transfers: a 2-GB index), whatever this run commits.
e = Engine(Options(accounts_max=n_acct, transfers_max=max(n_xfer, 100_000_000), pass_events_max=pb * batch,
                   pass_batches_max=pb))
a_lens = batches(n_acct, batch)
a_ts, t = timestamps(a_lens, 1_000_000_000)
acct = e.alloc(n_acct * 128)
e.generate_accounts(acct, 0, n_acct, seed=42)
res = e.alloc(max(n_acct, n_xfer) * 8)
rb = e.alloc((n_xfer // batch + 2) * 4)
e.commit_device_async(128, a_ts, a_lens, acct, res, rb)
e.sync()
ev = e.log_window(n_xfer) if inplace else e.alloc(n_xfer * 128)
e.generate_transfers(ev, 0, n_xfer, n_acct, seed=42, kind=KINDS["c2"])
e.sync()
x_lens = batches(n_xfer, batch)
x_ts, _ = timestamps(x_lens, t + 10)
e.commit_device_async(129, x_ts, x_lens, ev, res, rb)
e.sync()
replies = e.to_host(rb, len(x_lens) * 4).view(np.uint32)
print("device passes of %d prepares%s: %d transfers, reply bytes %d" % (pb, " in place" if inplace else "", n_xfer,
                                                                      int(replies.sum())))
e.close()
