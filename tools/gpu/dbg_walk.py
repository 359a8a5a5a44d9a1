import os, sys
sys.path.insert(0, ".")
os.environ["TBGPU_STALL_MS"] = "3000"
import numpy as np
from tests.test_gpu_walk import mixed_limits
from tests.harness.configs import batches, split, timestamps
from tigerbeetle_amd.state_machine import Engine, Options
for n_acc, n_xfer, pb, mode, merge in [(64, 200_000, 8, "early", 0), (64, 200_000, 8, "auto", 0), (4096, 300_000, 16, "early", 0)]:
    accts, xfers = mixed_limits(n_acc, n_xfer, seed=n_acc)
    e = Engine(Options(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * 8190, pass_batches_max=pb, bounds_sweep=mode))
    e.walk_merge_max(merge)
    a_lens, x_lens = batches(n_acc, 8190), batches(n_xfer, 8190)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    e.commit_many(128, a_ts, split(accts, a_lens))
    try:
        e.commit_many(129, x_ts, split(xfers, x_lens))
        print(n_acc, mode, "ok", {k: v for k, v in e.stats().items() if k.startswith("walk")}, flush=True)
    except Exception as ex:
        st = e.stats()
        print(n_acc, mode, "FAIL", ex, {k: v for k, v in st.items() if k.startswith("walk")}, flush=True)
    e.close()
