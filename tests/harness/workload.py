"""Seeded random workloads for differential tests (engine vs oracle), in the spirit of the
reference's auditor-driven workload (src/state_machine/workload.zig, auditor.zig): every
dependency class of SURVEY.md §7 "hard parts" is exercised — limit accounts, balancing transfers,
duplicate ids inside and across batches, two-phase pending/post/void in the same and in later
batches, expiry, linked chains (including open chains at batch end), invalid events, and u128
near-overflow balances.
"""
import random

from tigerbeetle_amd.types import (AccountFlags as AF, TransferFlags as TF, U128_MAX, pack_account,
                                   pack_transfer)

NS = 1_000_000_000


class Scenario:
    """A sequence of (operation, timestamp, [event bytes]) prepares plus optional setup actions."""

    def __init__(self):
        self.steps = []  # ("commit", op, ts, body) | ("setup", id, dp, dpost, cp, cpost)


def account_id(i):
    return U128_MAX - (i + 1)  # IdPermutation.inversion (testing/id.zig:31)


def make_scenario(seed, *, n_accounts=64, n_account_batches=2, n_transfer_batches=8, batch_len=(1, 200),
                  p_limit=0.1, p_linked=0.1, p_pending=0.2, p_post_void=0.2, p_balancing=0.05,
                  p_dup=0.05, p_invalid=0.05, p_timeout=0.5, id_space=None, near_overflow=False, p_huge=0.0,
                  ledgers=(1, 2), start_ts=10**12):
    rng = random.Random(seed)
    sc = Scenario()
    ts = start_ts

    # -- accounts ----------------------------------------------------------------------------
    acct_idx = list(range(n_accounts))
    created = []
    for b in range(n_account_batches):
        events = []
        chunk = acct_idx[b::n_account_batches]
        for i in chunk:
            flags = 0
            r = rng.random()
            if r < p_limit:
                flags |= AF.debits_must_not_exceed_credits if rng.random() < 0.5 else AF.credits_must_not_exceed_debits
            if rng.random() < p_linked:
                flags |= AF.linked
            ledger = ledgers[i % len(ledgers)]
            ev = dict(id=account_id(i), ledger=ledger, code=1 + (i % 7), flags=int(flags),
                      user_data_128=rng.getrandbits(8), user_data_64=rng.getrandbits(8), user_data_32=rng.getrandbits(4))
            if rng.random() < p_invalid:
                kind = rng.randrange(5)
                if kind == 0:
                    ev["ledger"] = 0
                elif kind == 1:
                    ev["code"] = 0
                elif kind == 2:
                    ev["reserved"] = 1
                elif kind == 3:
                    ev["flags"] |= 0x8
                else:
                    ev["timestamp"] = 5
            events.append(pack_account(**ev))
            if rng.random() < p_dup:  # duplicate (maybe with different fields)
                ev2 = dict(ev)
                if rng.random() < 0.5:
                    ev2["code"] = ev["code"] + 1
                events.append(pack_account(**ev2))
            created.append((i, ev["ledger"]))
        if not events:
            continue
        ts += 1 + len(events)
        sc.steps.append(("commit", 128, ts, events))

    if near_overflow:
        for i in rng.sample(range(n_accounts), k=max(1, n_accounts // 8)):
            big = U128_MAX - rng.randrange(0, 1 << 20)
            dp = rng.choice([0, rng.randrange(1 << 10)])
            sc.steps.append(("setup", account_id(i), dp, big - dp - rng.randrange(1 << 10),
                             0, rng.randrange(1 << 30)))

    # -- transfers ---------------------------------------------------------------------------
    id_space = id_space or (n_transfer_batches * batch_len[1] * 2)
    pendings = []  # (id, dr, cr, amount, ledger) of pending transfers attempted so far
    all_ids = []
    for b in range(n_transfer_batches):
        L = rng.randint(*batch_len)
        events = []
        for k in range(L):
            flags = 0
            if pendings and rng.random() < p_post_void:
                pid, pdr, pcr, pamt, pled = rng.choice(pendings)
                flags = TF.post_pending_transfer if rng.random() < 0.6 else TF.void_pending_transfer
                amount = rng.choice([0, 0, pamt, max(1, pamt - 1), min(pamt + 1, U128_MAX)])
                ev = dict(id=rng.randrange(1, id_space), pending_id=pid, amount=amount, flags=int(flags),
                          debit_account_id=rng.choice([0, 0, pdr, account_id(rng.randrange(n_accounts))]),
                          credit_account_id=rng.choice([0, 0, pcr]), ledger=rng.choice([0, 0, pled]),
                          code=rng.choice([0, 0, 1]), user_data_64=rng.choice([0, 5]))
                if rng.random() < 0.05:
                    ev["flags"] |= TF.pending
            else:
                dr = rng.randrange(n_accounts)
                cr = rng.randrange(n_accounts)
                if dr == cr:
                    cr = (cr + 1) % n_accounts
                ledger = ledgers[dr % len(ledgers)]
                amount = rng.choice([1, 2, 3, 10, 100, rng.randrange(1, 1000), rng.randrange(1, 1 << 40)])
                if p_huge and rng.random() < p_huge:  # (no draw at 0: keeps older seeds' streams) sums past 2^128 on fresh balances (saturated certificate)
                    amount = rng.choice([U128_MAX, 1 << 127, (1 << 126) + rng.randrange(1 << 20)])
                if rng.random() < p_pending:
                    flags |= TF.pending
                if rng.random() < p_balancing:
                    flags |= rng.choice([TF.balancing_debit, TF.balancing_credit,
                                         TF.balancing_debit | TF.balancing_credit])
                    if rng.random() < 0.3:
                        amount = 0
                timeout = 0
                if flags & TF.pending and rng.random() < p_timeout:
                    timeout = rng.choice([1, 2, 5, 50, 1000])
                tid = rng.randrange(1, id_space)
                if all_ids and rng.random() < p_dup:
                    tid = rng.choice(all_ids)
                ev = dict(id=tid, debit_account_id=account_id(dr), credit_account_id=account_id(cr),
                          amount=amount, ledger=ledger, code=1 + rng.randrange(3), flags=int(flags),
                          timeout=timeout, user_data_128=rng.getrandbits(4))
                if flags & TF.pending:
                    pendings.append((tid, account_id(dr), account_id(cr), amount, ledger))
            if rng.random() < p_linked:
                ev["flags"] |= TF.linked
            if rng.random() < p_invalid:
                kind = rng.randrange(6)
                if kind == 0:
                    ev["ledger"] = 0 if not (ev["flags"] & (TF.post_pending_transfer | TF.void_pending_transfer)) else 9
                elif kind == 1:
                    ev["code"] = 0
                elif kind == 2:
                    ev["flags"] |= 1 << 7
                elif kind == 3:
                    ev["timestamp"] = 1
                elif kind == 4:
                    ev["debit_account_id"] = account_id(n_accounts + 5)
                else:
                    ev["id"] = 0
            all_ids.append(ev["id"])
            events.append(pack_transfer(**ev))
        gap = rng.choice([0, 0, 0, NS, 3 * NS, 60 * NS])
        ts += 1 + gap + len(events)
        sc.steps.append(("commit", 129, ts, events))
    return sc


def run_oracle(sc, oracle):
    """Replay a scenario through an engine with the reference's commit-per-prepare interface;
    returns the list of reply bytes (one per commit)."""
    replies = []
    for step in sc.steps:
        if step[0] == "setup":
            oracle.set_balances(*step[1:])
        else:
            _, op, ts, events = step
            replies.append(oracle.commit(op, ts, b"".join(events)))
    return replies


def run_many(sc, engine):
    """Replay a scenario grouping consecutive commits of one operation into commit_many calls
    (multi-batch device passes)."""
    replies = []
    group = []

    def flush():
        if group:
            op = group[0][1]
            out = engine.commit_many(op, [g[2] for g in group], [b"".join(g[3]) for g in group])
            replies.extend(out)
            group.clear()

    for step in sc.steps:
        if step[0] == "setup":
            flush()
            engine.set_balances(*step[1:])
        else:
            if group and group[0][1] != step[1]:
                flush()
            group.append(step)
    flush()
    return replies
