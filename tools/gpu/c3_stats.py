"""Debug aid (GPU box): commit a C3 shape and print the engine's flow/bounds counters."""
import sys

sys.path.insert(0, ".")
from tests.harness.configs import SETTINGS, batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

cfg, n_acct, n_xfer, pb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pb * 8190, pass_batches_max=pb))
accts, xfers = generate(e, cfg, n_acct, n_xfer, seed=7)
a_lens, x_lens = batches(n_acct, 8190), batches(n_xfer, 8190)
a_ts, t = timestamps(a_lens, 10**12)
x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[cfg]["gap_every"])
e.commit_many(128, a_ts, split(accts, a_lens))
before = e.stats()
e.commit_many(129, x_ts, split(xfers, x_lens))
st = e.stats()
print({k: st[k] - before.get(k, 0) if isinstance(st[k], int) else st[k] for k in st})
names = ("plan", "sort", "link", "bounds_setup", "bounds_rounds", "sweep", "run_or_apply", "replies_wg0")
print({n: round(a - b, 3) for n, a, b in zip(names, st["flow_phase_ms"], before["flow_phase_ms"])})
