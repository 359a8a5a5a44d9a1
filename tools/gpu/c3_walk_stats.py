"""Analysis (not product code): the shape of what the bounds rounds leave to the sweep's walkers in
the adversarial C3 (configs "c3h"), per 64-prepare pass: segments (per limit account, its undecided
positions), heavy segments (>= WALK_HEAVY), and how the undecided units couple them — a unit whose
check is on a light segment and whose other leg is on a heavy one makes the heavy walk wait.

usage (GPU box): python tools/gpu/c3_walk_stats.py [config] [accounts] [transfers] [rounds] [heavy]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.harness.configs import batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3h"
    n_acct = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    n_xfer = int(sys.argv[3]) if len(sys.argv) > 3 else 3_144_960
    n_rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    heavy_min = int(sys.argv[5]) if len(sys.argv) > 5 else 256
    pass_events = 64 * 8190
    e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pass_events, pass_batches_max=64))
    accts, xfers = generate(e, cfg, n_acct, n_xfer, seed=42)
    a_lens, x_lens = batches(n_acct, 8190), batches(n_xfer, 8190)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    e.commit_many(128, a_ts, split(accts, a_lens))
    replies = e.commit_many(129, x_ts, split(xfers, x_lens))
    ok = np.ones(n_xfer, dtype=bool)
    off = 0
    for L, r in zip(x_lens, replies):
        p = np.frombuffer(r, dtype=np.uint32).reshape(-1, 2)
        ok[off + p[:, 0].astype(np.int64)] = False
        off += L
    a = accts.view(ACCOUNT_DTYPE)
    x = xfers.view(TRANSFER_DTYPE)
    order = np.argsort(a["id_lo"])
    idx_of = lambda lo: order[np.searchsorted(a["id_lo"][order], lo)]  # noqa: E731
    dr, cr = idx_of(x["debit_account_id_lo"]), idx_of(x["credit_account_id_lo"])
    amt = x["amount_lo"].astype(np.int64)
    limited = (a["flags"] & 2) != 0
    debits = np.zeros(n_acct, dtype=np.int64)
    credits = np.zeros(n_acct, dtype=np.int64)
    for p0 in range(0, n_xfer, pass_events):
        p1 = min(n_xfer, p0 + pass_events)
        ev = np.arange(p0, p1)
        dep = limited[dr[ev]] | limited[cr[ev]]
        status = np.where(dep & limited[dr[ev]], -1, 1).astype(np.int8)
        lm_d, lm_c = limited[dr[ev]], limited[cr[ev]]
        legs_acct = np.concatenate([dr[ev][lm_d], cr[ev][lm_c]])
        legs_ev = np.concatenate([np.nonzero(lm_d)[0], np.nonzero(lm_c)[0]])
        legs_deb = np.concatenate([np.ones(lm_d.sum(), bool), np.zeros(lm_c.sum(), bool)])
        o = np.lexsort((legs_ev, legs_acct))
        legs_acct, legs_ev, legs_deb = legs_acct[o], legs_ev[o], legs_deb[o]
        seg_start = np.r_[True, legs_acct[1:] != legs_acct[:-1]]
        seg_id = np.cumsum(seg_start) - 1
        starts = np.nonzero(seg_start)[0]
        la = amt[ev][legs_ev]

        def excl(v):
            c = np.cumsum(v)
            return c - v - (c[starts] - v[starts])[seg_id]

        x0, y0 = debits[legs_acct], credits[legs_acct]
        for _ in range(n_rounds):
            st = status[legs_ev]
            dmin = excl(np.where(legs_deb & (st == 1), la, 0))
            dmax = excl(np.where(legs_deb & (st != 0), la, 0))
            cmin = excl(np.where(~legs_deb & (st == 1), la, 0))
            cmax = excl(np.where(~legs_deb & (st != 0), la, 0))
            und = legs_deb & (st < 0)
            status[legs_ev[und & (x0 + dmax + la <= y0 + cmin)]] = 1
            status[legs_ev[und & (x0 + dmin + la > y0 + cmax)]] = 0
        und_unit = status < 0
        # undecided positions: legs of undecided units on limited accounts
        upos = und_unit[legs_ev]
        ua, ue, ud = legs_acct[upos], legs_ev[upos], legs_deb[upos]
        accs, cnt = np.unique(ua, return_counts=True)
        heavy_set = set(accs[cnt >= heavy_min].tolist())
        is_heavy = np.zeros(n_acct, dtype=bool)
        is_heavy[list(heavy_set)] = True
        uu = np.nonzero(und_unit)[0]
        d_, c_ = dr[ev][uu], cr[ev][uu]
        c_lim = limited[c_]
        hd, hc = is_heavy[d_], is_heavy[c_] & c_lim
        heavy_units = hd | hc
        hl = ~hd & hc             # check on a light account, credit on a heavy one: the heavy walk waits
        lh = hd & c_lim & ~hc     # check on a heavy account, credit on a light limited one
        hh = hd & hc
        # longest chain of alternations in the heavy stream that needs a light verdict
        print("pass %d: undecided units %d, positions %d, segments %d, heavy %d (positions %d, longest %d); "
              "heavy-stream units %d: heavy-heavy %d, light check -> heavy credit %d, heavy check -> light credit %d; "
              "light-only units %d" % (
                  p0 // pass_events, len(uu), len(ua), len(accs), len(heavy_set), int(cnt[cnt >= heavy_min].sum()),
                  int(cnt.max()) if len(cnt) else 0, int(heavy_units.sum()), int(hh.sum()), int(hl.sum()),
                  int(lh.sum()), int((~heavy_units).sum())), flush=True)
        okp = ok[ev]
        np.add.at(debits, dr[ev][okp], amt[ev][okp])
        np.add.at(credits, cr[ev][okp], amt[ev][okp])


if __name__ == "__main__":
    main()
