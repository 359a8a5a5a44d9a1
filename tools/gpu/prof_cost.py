"""What the bench's in-step profiling costs the headline: C2, 100M transfers committed in place in
512-prepare passes (bench.py's headline leg), timed with each profile mask in turn, alternating.

usage: python tools/gpu/prof_cost.py [rounds]
Prints one JSON line per (mask, round) and a summary line: ms per step for each mask.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

from tests.harness.configs import KINDS, batches, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n_acct, n_xfer, batch, pb = 1_000_000, 100_000_000, 8190, 512
e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer + 6 * 64 * batch, pass_events_max=pb * batch,
                   pass_batches_max=pb, profile=True))
a_lens = batches(n_acct, batch)
a_ts, t = timestamps(a_lens, 1_000_000_000)
acct = e.alloc(n_acct * 128)
e.generate_accounts(acct, 0, n_acct, seed=42)
res = e.alloc(n_xfer * 8)
rb = e.alloc((n_xfer // batch + 2) * 4)
e.commit_device_async(128, a_ts, a_lens, acct, res, rb)
e.sync()
x_lens = batches(n_xfer, batch)
MASKS = {"bench (apply|pass|replay)": e.PROF_APPLY | e.PROF_PASS | e.PROF_REPLAY, "none": 0,
         "pass only": e.PROF_PASS, "spans only (the timed steps since round 6)": e.PROF_SPANS}
out = {k: [] for k in MASKS}
for r in range(rounds + 1):
    for name, mask in MASKS.items():
        e.reset_transfers()
        win = e.log_window(n_xfer)
        e.generate_transfers(win, 0, n_xfer, n_acct, seed=42, kind=KINDS["c2"])
        e.sync()
        ts, t = timestamps(x_lens, t + 10)
        e.profile_mask(mask)
        e.reset_stats()
        t0 = time.perf_counter()
        e.commit_device_async(129, ts, x_lens, win, res, rb)
        t_issue = time.perf_counter()
        e.sync()
        ms = (time.perf_counter() - t0) * 1e3
        issue_ms = (t_issue - t0) * 1e3
        fails = int(e.to_host(rb, len(x_lens) * 4).view(np.uint32).sum())
        st = e.stats()
        val_ms = st["span_ms"][0] / st["span_launches"][0] if st.get("span_launches") and st["span_launches"][0] else None
        if r:  # round 0 warms up every mask
            out[name].append(ms)
            print(json.dumps({"mask": name, "round": r, "ms": round(ms, 3), "issue_ms": round(issue_ms, 3), "validate_span_ms": round(val_ms, 4) if val_ms else None,
                              "reply_bytes": fails}), flush=True)
print(json.dumps({"summary_ms_per_step": {k: [round(min(v), 3), round(float(np.median(v)), 3)] for k, v in out.items()},
                  "transfers": n_xfer}), flush=True)
e.close()
