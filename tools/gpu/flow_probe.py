"""Print flow-path statistics for a BASELINE workload shape (debug aid): passes, dependent
events, passes that ran on the parallel flow path, units, and the replay kernel time."""
import sys
import time

sys.path.insert(0, ".")
from tests.harness.configs import SETTINGS, batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

config, n_acc, n_xfer, pb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
e = Engine(Options(accounts_max=n_acc, transfers_max=n_xfer, pass_events_max=pb * 8190, pass_batches_max=pb,
                   profile=True))
accts, xfers = generate(e, config, n_acc, n_xfer, seed=7)
a_lens = batches(n_acc, 8190)
a_ts, t = timestamps(a_lens, 10**12)
e.commit_many(128, a_ts, split(accts, a_lens))
x_lens = batches(n_xfer, 8190)
x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[config]["gap_every"])
e.reset_stats()
t0 = time.time()
e.commit_many(129, x_ts, split(xfers, x_lens))
dt = time.time() - t0
s = e.stats()
print(config, "wall %.3fs" % dt, {k: s[k] for k in ("passes", "dependent_events", "flow_passes", "flow_units", "flow_runs", "flow_run_units",
                                                   "ms_replay", "launches_replay", "ms_validate", "ms_resolve")})
