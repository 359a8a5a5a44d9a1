"""Debug aid (GPU box): C3 at 10M transfers through 64-prepare pipelined chunks and through
512-prepare device passes; compares failures, transfer counts and balance totals."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.harness.configs import SETTINGS, batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402


def run(cfg, seed, n_acct, n_xfer, pb, pipelined):
    e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pb * 8190, pass_batches_max=pb))
    accts, xfers = generate(e, cfg, n_acct, n_xfer, seed=seed)
    a_lens, x_lens = batches(n_acct, 8190), batches(n_xfer, 8190)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10, gap_every=SETTINGS[cfg]["gap_every"])
    e.commit_many(128, a_ts, split(accts, a_lens))
    if pipelined:
        rb, rep, _ = e.commit_pipelined(129, x_ts, x_lens, np.ascontiguousarray(xfers), chunk_batches=pb)
        replies, off = [], 0
        for L, nb in zip(x_lens, rb):
            replies.append(bytes(rep[off * 8:off * 8 + int(nb)]))
            off += L
    else:
        replies = e.commit_many(129, x_ts, split(xfers, x_lens))
    st = e.stats()
    acc = e.export_accounts()
    tot = {f: int(acc[f + "_lo"].astype(object).sum()) for f in ("debits_posted", "credits_posted")}
    return replies, st, tot


cfg, seed = sys.argv[1], int(sys.argv[2])
n_acct, n_xfer = 1_000_000, int(sys.argv[3]) if len(sys.argv) > 3 else 10_000_000
ra, sa, ta = run(cfg, seed, n_acct, n_xfer, 64, True)
rb_, sb, tb = run(cfg, seed, n_acct, n_xfer, 512, False)
fa = sum(len(r) // 8 for r in ra)
fb = sum(len(r) // 8 for r in rb_)
diff = [k for k, (x, y) in enumerate(zip(ra, rb_)) if x != y]
print("64-chunk: failed %d transfers %d totals %s" % (fa, sa["transfers"], ta))
print("512-pass: failed %d transfers %d totals %s" % (fb, sb["transfers"], tb))
print("prepares whose replies differ: %d %s" % (len(diff), diff[:10]))
