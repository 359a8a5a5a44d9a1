"""Host model of the engine's dependence classification (which events of a create_transfers pass the
ordered fallback commits): a restatement of the rules of tigerbeetle_amd/csrc/k_validate.h (hazard
bits) and k_resolve.h (tb_classify, chain propagation), for one pass over a known pre-pass state.

It is not the reference's logic — the reference has no notion of dependence — but the engine's own
rule, written independently, so a GPU test can assert that `stats["dependent_events"]` is exactly
this count (VERDICT r3 What's weak #1: the classification must not depend on scheduling).

Model limits: the pass's global overflow certificate must hold (bound + S < 2^128; true of every
workload without near-overflow balances), balances must never have been set directly (no `setup`
steps), and 32-bit fingerprint collisions of distinct ids are ignored.
"""
from tigerbeetle_amd.types import TRANSFER_DTYPE, AccountFlags as AF, TransferFlags as TF, U128_MAX

import numpy as np

LIMITS = int(AF.debits_must_not_exceed_credits) | int(AF.credits_must_not_exceed_debits)
PADDING = 0xFFC0  # TransferFlags bits 6..15


def _u128(lo, hi):
    return int(lo) | (int(hi) << 64)


def dependent_count(prepares, accounts, existing_ids=frozenset()):
    """prepares: list of transfer bodies (bytes) of ONE device pass, in order; accounts: {id: (flags,
    ledger)} live before the pass; existing_ids: transfer ids stored before the pass (a post / void
    of such a pending transfer is not modelled: the pass must hold every pending it names).
    Returns the number of events the engine classifies dependent."""
    evs = []  # per event: dict
    for p, body in enumerate(prepares):
        rec = np.frombuffer(body, dtype=TRANSFER_DTYPE)
        L = len(rec)
        for j in range(L):
            r = rec[j]
            evs.append(dict(p=p, j=j, L=L, id=_u128(r["id_lo"], r["id_hi"]),
                            dr=_u128(r["debit_account_id_lo"], r["debit_account_id_hi"]),
                            cr=_u128(r["credit_account_id_lo"], r["credit_account_id_hi"]),
                            amount=_u128(r["amount_lo"], r["amount_hi"]),
                            pid=_u128(r["pending_id_lo"], r["pending_id_hi"]), timeout=int(r["timeout"]),
                            ledger=int(r["ledger"]), code=int(r["code"]), flags=int(r["flags"]),
                            ts=int(r["timestamp"])))
    # -- kernel 1 (k_validate.h): who claims its id, pv keys, hazard bits ---------------------------
    for e in evs:
        f = e["flags"]
        e.update(claims=False, pv_key=False, accts=False, limit=False, bal=False, ok=False, selfdep=False)
        if (f & TF.linked) and e["j"] == e["L"] - 1:
            continue  # linked_event_chain_open
        if e["ts"] != 0:
            continue  # timestamp_must_be_zero
        if f & PADDING or e["id"] in (0, U128_MAX):
            continue
        if f & (TF.post_pending_transfer | TF.void_pending_transfer):
            if (f & TF.post_pending_transfer) and (f & TF.void_pending_transfer):
                continue
            if f & (TF.pending | TF.balancing_debit | TF.balancing_credit):
                continue
            if e["pid"] in (0, U128_MAX) or e["pid"] == e["id"] or e["timeout"] != 0:
                continue
            e["pv"] = True
            e["pv_key"] = True
            e["claims"] = True
            continue
        if e["dr"] in (0, U128_MAX) or e["cr"] in (0, U128_MAX) or e["dr"] == e["cr"] or e["pid"] != 0:
            continue
        if not (f & TF.pending) and e["timeout"] != 0:
            continue
        if not (f & (TF.balancing_debit | TF.balancing_credit)) and e["amount"] == 0:
            continue
        if e["ledger"] == 0 or e["code"] == 0:
            continue
        e["claims"] = True  # the id's home entry is claimed with the account probes (:211-232)
        da, ca = accounts.get(e["dr"]), accounts.get(e["cr"])
        if da is None or ca is None or da[1] != ca[1] or e["ledger"] != da[1]:
            continue
        e["accts"] = True
        e["limit"] = bool((da[0] | ca[0]) & LIMITS)
        e["bal"] = bool(f & (TF.balancing_debit | TF.balancing_credit))
    # Claims: an id claimed by two or more events of the pass, and stored before by none, collides.
    claimers = {}
    for e in evs:
        if e["claims"]:
            claimers.setdefault(e["id"], []).append(e)
    collided = {i for i, c in claimers.items() if len(c) >= 2 and i not in existing_ids}
    claimed_in_pass = {i for i in claimers if i not in existing_ids}
    pv_keys = {}
    for e in evs:
        if e["pv_key"]:
            pv_keys[e["pid"]] = pv_keys.get(e["pid"], 0) + 1
    any_dup = bool(collided) or any(n >= 2 for n in pv_keys.values())
    any_pv = bool(pv_keys)
    marked = set()
    # Intrinsic ok-ness of an event that reached the account checks (create_transfer): the exists
    # check (id stored before) and the timeout overflow are the failures left after them.
    for e in evs:
        if e.get("pv"):
            e["selfdep"] = e["id"] in collided
            continue
        if not e["accts"]:
            continue
        if e["bal"]:  # marks before the id check (k_validate.h: balancing accounts marked up front)
            if e["flags"] & TF.balancing_debit:
                marked.add(e["dr"])
            if e["flags"] & TF.balancing_credit:
                marked.add(e["cr"])
        exists = e["id"] in existing_ids
        e["selfdep"] = e["id"] in collided
        e["ok"] = not exists  # timeouts in workloads never overflow u64 nanoseconds
    any_bal = bool(marked)
    # -- kernel 2 (k_resolve.h tb_classify) ----------------------------------------------------------
    for e in evs:
        dep = e["selfdep"]
        if not dep and any_dup:
            if e["claims"] and not e.get("pv") and e["id"] in collided:
                dep = True
            if e["pv_key"] and pv_keys.get(e["pid"], 0) >= 2:
                dep = True
        if not dep and any_pv:
            if (e["accts"] or e["pv_key"]) and e["id"] in pv_keys:
                dep = True
            if e["pv_key"] and e["pid"] in claimed_in_pass:
                dep = True
        if not dep and e["accts"] and e["ok"]:
            if e["bal"] or e["limit"]:
                dep = True
            elif any_bal and (e["dr"] in marked or e["cr"] in marked):
                dep = True
        e["dep"] = dep
    # Linked chains: a chain with a dependent member is dependent as a whole (execute :628-692).
    total = 0
    i = 0
    while i < len(evs):
        j = i
        while j + 1 < len(evs) and evs[j + 1]["p"] == evs[i]["p"] and (evs[j]["flags"] & TF.linked):
            j += 1
        members = evs[i:j + 1]
        if evs[i]["flags"] & TF.linked and len(members) >= 1:
            if any(m["dep"] for m in members):
                total += len(members)
        else:
            total += sum(1 for m in members if m["dep"])
        i = j + 1
    return total
