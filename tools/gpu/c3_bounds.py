"""Analysis (not product code): how much of the C3 ordered work can interval bounds decide in
parallel?  Generates a C3 workload on the GPU, commits it on the engine for the true results, then
simulates on the host the round-based bounds certification of limit checks
(state_machine.zig:863-864, tigerbeetle.zig:31-39): a debit on a debits_must_not_exceed_credits
account is certainly ok if dp + dpost + amount <= cpost holds with every undecided earlier debit
counted and every undecided earlier credit left out, certainly failing if it fails with the
opposite choices; each round re-scans every limit account's events with the decided ones.

usage (GPU box): python tools/gpu/c3_bounds.py [accounts] [transfers]
"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from tests.harness.configs import batches, generate, split, timestamps  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402
from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE  # noqa: E402


def main():
    n_acct = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    n_xfer = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
    e = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=64 * 8190, pass_batches_max=64))
    accts, xfers = generate(e, "c3", n_acct, n_xfer, seed=42)
    a_lens, x_lens = batches(n_acct, 8190), batches(n_xfer, 8190)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    e.commit_many(128, a_ts, split(accts, a_lens))
    replies = e.commit_many(129, x_ts, split(xfers, x_lens))
    codes = np.zeros(n_xfer, dtype=np.int64)
    off = 0
    for L, r in zip(x_lens, replies):
        p = np.frombuffer(r, dtype=np.uint32).reshape(-1, 2)
        codes[off + p[:, 0].astype(np.int64)] = p[:, 1]
        off += L
    a = accts.view(ACCOUNT_DTYPE)
    x = xfers.view(TRANSFER_DTYPE)
    ids = a["id_lo"]  # ids differ in the low word (IdPermutation.inversion)
    order = np.argsort(ids)
    idx_of = lambda lo: order[np.searchsorted(ids[order], lo)]  # noqa: E731
    dr, cr = idx_of(x["debit_account_id_lo"]), idx_of(x["credit_account_id_lo"])
    amt = x["amount_lo"].astype(np.int64)
    limited = (a["flags"] & 2) != 0
    print("accounts %d (limited %d), transfers %d, failed %d (codes %s)" % (
        n_acct, limited.sum(), n_xfer, (codes != 0).sum(), np.unique(codes[codes != 0]).tolist()))

    dep = limited[dr] | limited[cr]
    status = np.where(limited[dr], -1, 1).astype(np.int8)  # only debits of limited accounts can fail
    print("events touching a limited account: %d (%.1f%%), undecided at start: %d" % (
        dep.sum(), 100 * dep.mean(), (status < 0).sum()))
    # Legs of limited accounts, by (account, event).
    ev = np.arange(n_xfer)
    legs_acct = np.concatenate([dr[limited[dr]], cr[limited[cr]]])
    legs_ev = np.concatenate([ev[limited[dr]], ev[limited[cr]]])
    legs_deb = np.concatenate([np.ones(limited[dr].sum(), bool), np.zeros(limited[cr].sum(), bool)])
    o = np.lexsort((legs_ev, legs_acct))
    legs_acct, legs_ev, legs_deb = legs_acct[o], legs_ev[o], legs_deb[o]
    seg_start = np.r_[True, legs_acct[1:] != legs_acct[:-1]]
    seg_id = np.cumsum(seg_start) - 1
    la = amt[legs_ev]

    def seg_excl_cumsum(v):
        c = np.cumsum(v)
        starts = np.nonzero(seg_start)[0]
        base = c[starts] - v[starts]
        return c - v - base[seg_id]

    rounds, t0 = 0, time.time()
    hist = []
    while True:
        st = status[legs_ev]
        dmin = seg_excl_cumsum(np.where(legs_deb & (st == 1), la, 0))
        dmax = seg_excl_cumsum(np.where(legs_deb & (st != 0), la, 0))
        cmin = seg_excl_cumsum(np.where(~legs_deb & (st == 1), la, 0))
        cmax = seg_excl_cumsum(np.where(~legs_deb & (st != 0), la, 0))
        und = legs_deb & (st < 0)
        ok = und & (dmax + la <= cmin)
        bad = und & (dmin + la > cmax)
        status[legs_ev[ok]] = 1
        status[legs_ev[bad]] = 0
        rounds += 1
        left = int((status < 0).sum())
        hist.append(left)
        if left == 0 or rounds >= 5000 or (not ok.any() and not bad.any()):
            break
    truth_fail = codes != 0
    print("rounds %d (%.1f s); undecided after rounds 1,2,4,8,16,32,64,128: %s" % (
        rounds, time.time() - t0, [hist[k - 1] if k <= len(hist) else 0 for k in (1, 2, 4, 8, 16, 32, 64, 128)]))
    print("matches the engine: %s (fail %d vs %d)" % (
        bool(np.array_equal(status == 0, truth_fail)), (status == 0).sum(), truth_fail.sum()))


if __name__ == "__main__":
    main()
