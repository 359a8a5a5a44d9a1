"""Analysis (not product code): after a few bounds rounds, how do the undecided limit checks of a C3
pass split into independent groups?  Two undecided units interact only through a limit account they
both touch, so connected components of (unit -- its limit accounts) could be swept in parallel.

Per 64-prepare pass: the balances at the pass start come from the engine's true results (every
earlier ok transfer applied), then the bounds rounds of k_flow.h are simulated on the host (as
tools/gpu/c3_bounds.py does for one big pass) and the undecided units are grouped.

usage (GPU box): python tools/gpu/c3_components.py [seed] [accounts] [transfers] [rounds]
"""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.harness.configs import batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE  # noqa: E402


def components(n, edges_a, edges_b):
    parent = np.arange(n)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for a, b in zip(edges_a, edges_b):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    return np.array([find(x) for x in range(n)])


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 42
    n_acct = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    n_xfer = int(sys.argv[3]) if len(sys.argv) > 3 else 2_096_640
    n_rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    pass_events = 64 * 8190
    e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=pass_events, pass_batches_max=64))
    accts, xfers = generate(e, "c3", n_acct, n_xfer, seed=seed)
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
        status = np.where(dep & limited[dr[ev]], -1, 1).astype(np.int8)  # only debits of limited accounts check
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
        undec = np.nonzero(status < 0)[0]
        if len(undec):
            uacc = np.unique(np.concatenate([dr[ev][undec][lm_d[undec]], cr[ev][undec][lm_c[undec]]]))
            pos = {v: i for i, v in enumerate(uacc)}
            both = undec[lm_d[undec] & lm_c[undec]]
            comp = components(len(uacc), [pos[v] for v in dr[ev][both]], [pos[v] for v in cr[ev][both]])
            unit_comp = np.array([comp[pos[dr[ev][u]]] if lm_d[u] else comp[pos[cr[ev][u]]] for u in undec])
            sizes = np.sort(np.bincount(unit_comp))[::-1]
            sizes = sizes[sizes > 0]
            print("pass %d: dependent %d, undecided after %d rounds %d, accounts %d, components %d, "
                  "largest %s (%.0f%% of the undecided)" % (p0 // pass_events, dep.sum(), n_rounds, len(undec),
                                                           len(uacc), len(sizes), sizes[:5].tolist(),
                                                           100.0 * sizes[0] / len(undec)))
        # true effects of the pass
        okp = ok[ev]
        np.add.at(debits, dr[ev][okp], amt[ev][okp])
        np.add.at(credits, cr[ev][okp], amt[ev][okp])


if __name__ == "__main__":
    main()
