// k_replay.h — kernel 3 of a pass: the ordered fallback.
//
// One workgroup.  Lane 0 replays the dependent events of the pass in batch order with the
// reference's sequential logic (execute state_machine.zig:612-698, create_transfer :779-884,
// post_or_void_pending_transfer :907-1014, create_account :738-765) directly on the HBM tables.
// Linked-chain scopes keep an undo log and roll back LIFO on discard (cache_map.zig:266-309).
// Every event that can observe a dependent event's effect is itself dependent (see k_resolve.h),
// so replaying only this subsequence reproduces the sequential results exactly.  Afterwards the
// workgroup writes the replies of the batches that had dependent events.
#pragma once

#include "k_resolve.h"

enum : u32 {
    UNDO_ACCOUNT_INSERT = 1, UNDO_BALANCE_UPDATE = 2, UNDO_TRANSFER_INSERT = 3, UNDO_POSTED = 4,
    UNDO_FREE_DELTA = 5,  // flow path: the four balance deltas added (atomically) to a free account
};

struct alignas(16) UndoEntry {
    u32 kind;
    u32 slot;  // account slot / index entry / log position
    u64 pad;
    AccountBal before;  // UNDO_FREE_DELTA: the deltas
};

// Replay state of one lane.  FLOW = false: the sequential replay (one lane of one workgroup owns
// every table it touches).  FLOW = true: one of many lanes of the parallel flow path (k_flow.h):
// every read of state another lane may have written goes through L1-bypassing agent-scope loads,
// and balances of FREE accounts (no limit flag, not balancing-marked, under the global overflow
// certificate: no check reads them) are changed only by atomic deltas, since lanes that do not
// share a resource run concurrently.
struct Replay {
    Tables T;
    UndoEntry* undo;
    u32 undo_len;
    u32 undo_cap;
    u64 log_base;
    bool scope;
    bool failed;  // a panic was raised: stop
    // flow path
    u32 epoch;
    bool cert_global;
    bool cert64;  // no balance word can carry this pass: free-account deltas are low-word adds
    // Flow path: this lane's change to transfer_count (mod 2^64), added once per wave when the run
    // ends — one atomic per unit on that single word serialised the run.
    u64 xcount = 0;
};

// Flow path: lookups kernel 1 already did exactly (k_flow.h).  The account slots of an event it
// validated through the account checks (HZ_ACCTS; accounts never change in a create_transfers
// pass), and — for a single-event unit — the id's absence (its speculative claim was a new entry,
// and no other dependent event of the pass names this id): the insert then revives that entry
// instead of claiming a new one.  entry == TB_NOT_FOUND: the slots only (chain members).
// rec: kernel 1 wrote this event's record at its log position under `entry` (HZ_REC; the record a
// successful create writes, as it is not balancing): an insert revives `entry`, storing nothing.
struct FastHint {
    u32 drs, crs;
    u32 entry;  // index entry claimed by kernel 1 (tombstoned by kernel 2), or TB_NOT_FOUND
    bool known_new = false;  // the id is absent: skip the find, revive `entry`
    bool rec = false;
};

__device__ static inline u64 fl_ld64(const void* p) {
    return __hip_atomic_load((const u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ static inline u128 fl_ld128(const void* p) {
    const u64* w = (const u64*)p;
    return tb_u128(fl_ld64(w), fl_ld64(w + 1));
}
template <bool FLOW, typename R>
__device__ static inline R rp_load(const R* p) {
    static_assert(sizeof(R) % 8 == 0, "8-byte words");
    if (!FLOW) return *p;
    R r;
    u64* d = (u64*)&r;
#pragma unroll
    for (u32 k = 0; k < sizeof(R) / 8; k++) d[k] = fl_ld64((const u64*)p + k);
    return r;
}
template <bool FLOW>
__device__ static inline u8 rp_load_posted(const Tables& T, u32 pos) {
    if (!FLOW) return T.xposted[pos];
    const u32 w = __hip_atomic_load((const u32*)(T.xposted + (pos & ~3u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (u8)(w >> (8 * (pos & 3)));
}
// Flow-path stores: lanes of other workgroups (other XCDs, whose L2s are not coherent with this
// one) read what a unit writes once its successors are released, so every word is stored
// write-through at agent scope (sc1) and drained before the release (fl_run_unit).
template <bool FLOW, typename R>
__device__ static inline void rp_store(R* p, const R& v) {
    static_assert(sizeof(R) % 8 == 0, "8-byte words");
    if (!FLOW) {
        *p = v;
        return;
    }
    const u64* s = (const u64*)&v;
#pragma unroll
    for (u32 k = 0; k < sizeof(R) / 8; k++) {
        __hip_atomic_store((u64*)p + k, s[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// An account's balances (both planes, tb_device.h BalView) with the same rules.
template <bool FLOW>
__device__ static inline AccountBal rp_bal_load(const BalView& V, u64 slot) {
    if (!FLOW) return tb_bal_load(V, slot);
    const u64* l = V.lo + 4 * slot;
    const u64* h = V.hi + 4 * slot;
    AccountBal b;
    b.debits_pending = tb_u128(fl_ld64(l), fl_ld64(h));
    b.debits_posted = tb_u128(fl_ld64(l + 1), fl_ld64(h + 1));
    b.credits_pending = tb_u128(fl_ld64(l + 2), fl_ld64(h + 2));
    b.credits_posted = tb_u128(fl_ld64(l + 3), fl_ld64(h + 3));
    return b;
}
template <bool FLOW>
__device__ static inline void rp_bal_store(const BalView& V, u64 slot, const AccountBal& b) {
    if (!FLOW) {
        tb_bal_store(V, slot, b);
        return;
    }
    u64* l = V.lo + 4 * slot;
    u64* h = V.hi + 4 * slot;
    const u128 f[4] = {b.debits_pending, b.debits_posted, b.credits_pending, b.credits_posted};
#pragma unroll
    for (u32 k = 0; k < 4; k++) {
        __hip_atomic_store(l + k, tb_lo(f[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(h + k, tb_hi(f[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <bool FLOW>
__device__ static inline void rp_store_posted(const Tables& T, u32 pos, u8 v) {
    if (!FLOW) {
        T.xposted[pos] = v;
        return;
    }
    u32* w = (u32*)(T.xposted + (pos & ~3u));
    const u32 sh = 8 * (pos & 3);
    __hip_atomic_fetch_and(w, ~(0xFFu << sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v) __hip_atomic_fetch_or(w, (u32)v << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Flow path: is this account's balance an ordering resource (k_flow.h)?  Must agree with the
// planner's choice.
__device__ static inline bool fl_account_is_resource(const Tables& T, u32 slot, u32 epoch, bool cert_global) {
    return !cert_global || (T.acct_hot[slot].flags & AF_LIMITS) || T.account_mark[slot] == epoch;
}

// tb_transfer_find with agent-scope loads (entries and records may be new from another lane).
template <bool FLOW>
__device__ static inline u32 rp_transfer_find(const Tables& T, u64 lo, u64 hi) {
    if (!FLOW) return tb_transfer_find(T, lo, hi);
    if (tb_id_reserved(lo, hi)) return TB_NOT_FOUND;
    const u64 fp = tb_fp32(lo, hi);
    u64 pos = tb_hash_id(lo, hi) & T.xidx_mask;
    for (u64 n = 0; n <= T.xidx_mask; n++) {
        const u64 e = fl_ld64(&T.xidx[pos]);
        if (e == 0) return TB_NOT_FOUND;
        if ((e >> 32) == fp && !(e & XI_TOMB)) {
            const u32 lp = tb_xi_pos(e);
            const u64* idw = (const u64*)&T.xlog[lp];
            if (fl_ld64(idw) == lo && fl_ld64(idw + 1) == hi) return lp;
        }
        pos = (pos + 1) & T.xidx_mask;
    }
    return TB_NOT_FOUND;
}

__device__ static inline void rp_panic(Replay& R, u32 code) {
    tb_panic(R.T.g, code);
    R.failed = true;
}

__device__ static inline void rp_push(Replay& R, u32 kind, u32 slot, const AccountBal* before) {
    if (!R.scope) return;
    if (R.undo_len == R.undo_cap) {
        rp_panic(R, PANIC_UNDO_FULL);
        return;
    }
    UndoEntry& e = R.undo[R.undo_len++];
    e.kind = kind;
    e.slot = slot;
    if (before) e.before = *before;
}

__device__ static inline void rp_add_free_delta(Replay& R, u32 slot, const AccountBal& d) {
    const u128 f[4] = {d.debits_pending, d.debits_posted, d.credits_pending, d.credits_posted};
    if (R.cert64) {  // every balance stays below 2^64: the low word alone is exact, no carry to wait for
#pragma unroll
        for (u32 k = 0; k < 4; k++) {
            if (f[k]) tb_bal_add_lo(R.T.bal, slot, k, tb_lo(f[k]));
        }
        return;
    }
#pragma unroll
    for (u32 k = 0; k < 4; k++) {
        if (f[k]) tb_bal_add(R.T.bal, slot, k, f[k]);
    }
}

template <bool FLOW>
__device__ static inline void rp_scope_close(Replay& R, bool persist) {
    if (!persist) {
        while (R.undo_len > 0) {
            const UndoEntry& e = R.undo[--R.undo_len];
            switch (e.kind) {
            case UNDO_ACCOUNT_INSERT:  // tombstone (id = maxInt), timestamp kept
                tb_account_tombstone(R.T, e.slot);
                R.T.g->account_count--;
                break;
            case UNDO_BALANCE_UPDATE: rp_bal_store<FLOW>(R.T.bal, e.slot, e.before); break;
            case UNDO_FREE_DELTA: {
                AccountBal neg;
                neg.debits_pending = (u128)0 - e.before.debits_pending;
                neg.debits_posted = (u128)0 - e.before.debits_posted;
                neg.credits_pending = (u128)0 - e.before.credits_pending;
                neg.credits_posted = (u128)0 - e.before.credits_posted;
                rp_add_free_delta(R, e.slot, neg);
                break;
            }
            case UNDO_TRANSFER_INSERT:
                tb_xindex_tombstone(R.T, e.slot);
                if (FLOW) R.xcount--;
                else R.T.g->transfer_count--;
                break;
            case UNDO_POSTED: rp_store_posted<FLOW>(R.T, e.slot, POSTED_NONE); break;
            }
        }
    }
    R.undo_len = 0;
    R.scope = false;
}

// Checked `+` (ReleaseSafe trap).
__device__ static inline u128 rp_add(Replay& R, u128 a, u128 b) {
    u128 r;
    if (tb_add_overflows(a, b, &r)) rp_panic(R, PANIC_OVERFLOW);
    return r;
}

// A free account on the flow path is not read at all (zeros, *free = true): under the global
// certificate no check its value feeds can fire (overflows :848-861), and the others read only
// constrained accounts (balancing :826-846, limits :863-868); rp_balance_update then applies the
// difference as a delta.
template <bool FLOW>
__device__ static inline AccountBal rp_balance_load(Replay& R, u32 slot, bool* free) {
    *free = FLOW && !fl_account_is_resource(R.T, slot, R.epoch, R.cert_global);
    if (*free) return AccountBal{};
    return rp_bal_load<FLOW>(R.T.bal, slot);
}

// Write an account's balances (`before` = what rp_balance_load returned).  A free account on the
// flow path gets the difference as atomic deltas: other lanes may be adding to it concurrently,
// and its value is read by no check (see Replay).
template <bool FLOW>
__device__ static inline void rp_balance_update(Replay& R, u32 slot, const AccountBal& before, const AccountBal& next) {
    if (FLOW && !fl_account_is_resource(R.T, slot, R.epoch, R.cert_global)) {
        AccountBal d;
        d.debits_pending = next.debits_pending - before.debits_pending;
        d.debits_posted = next.debits_posted - before.debits_posted;
        d.credits_pending = next.credits_pending - before.credits_pending;
        d.credits_posted = next.credits_posted - before.credits_posted;
        rp_push(R, UNDO_FREE_DELTA, slot, &d);
        rp_add_free_delta(R, slot, d);
        return;
    }
    rp_push(R, UNDO_BALANCE_UPDATE, slot, &before);
    rp_bal_store<FLOW>(R.T.bal, slot, next);
}

// Insert a transfer record at the event's own log position (after an exact find said "absent").
template <bool FLOW>
__device__ static inline void rp_transfer_insert(Replay& R, const Transfer& t, u32 log_pos) {
    rp_store<FLOW>(&R.T.xlog[log_pos], t);
    if (FLOW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the record before its index entry
    const u32 entry = tb_transfer_claim_new(R.T, tb_lo(t.id), tb_hi(t.id), log_pos);
    if (entry == TB_NOT_FOUND) {
        R.failed = true;
        return;
    }
    if (FLOW) R.xcount++;
    else R.T.g->transfer_count++;
    rp_push(R, UNDO_TRANSFER_INSERT, entry, nullptr);
}

template <bool FLOW>
__device__ static inline u32 rp_post_or_void(Replay& R, const Transfer& t, u32 log_pos, const FastHint* hint = nullptr) {
    const Tables& T = R.T;
    const u16 f = t.flags;
    if ((f & TF_POST) && (f & TF_VOID)) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_PENDING) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_DEBIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_CREDIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (t.pending_id == 0) return CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (t.pending_id == TB_U128_MAX) return CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (t.pending_id == t.id) return CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t.timeout != 0) return CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    const u32 pslot = rp_transfer_find<FLOW>(T, tb_lo(t.pending_id), tb_hi(t.pending_id));
    if (pslot == TB_NOT_FOUND) return CT_PENDING_TRANSFER_NOT_FOUND;
    const Transfer p = rp_load<FLOW>(&T.xlog[pslot]);
    if (!(p.flags & TF_PENDING)) return CT_PENDING_TRANSFER_NOT_PENDING;
    // hint: the pending transfer's account slots, from kernel 1 (it found the same record: an
    // earlier pass's, whose id no event of this pass can re-create).
    const u32 drs = hint ? hint->drs : tb_account_find(T, tb_lo(p.debit_account_id), tb_hi(p.debit_account_id));
    const u32 crs = hint ? hint->crs : tb_account_find(T, tb_lo(p.credit_account_id), tb_hi(p.credit_account_id));
    if (drs == TB_NOT_FOUND || crs == TB_NOT_FOUND) {
        rp_panic(R, PANIC_ASSERT);
        return R_OK;
    }
    if (t.debit_account_id > 0 && t.debit_account_id != p.debit_account_id) {
        return CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    }
    if (t.credit_account_id > 0 && t.credit_account_id != p.credit_account_id) {
        return CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    }
    if (t.ledger > 0 && t.ledger != p.ledger) return CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t.code > 0 && t.code != p.code) return CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;
    const u128 amount = t.amount > 0 ? t.amount : p.amount;
    if (amount > p.amount) return CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if ((f & TF_VOID) && amount < p.amount) return CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    const u32 es = rp_transfer_find<FLOW>(T, tb_lo(t.id), tb_hi(t.id));
    if (es != TB_NOT_FOUND) return tb_post_void_exists(t, rp_load<FLOW>(&T.xlog[es]), p);
    const u8 posted = rp_load_posted<FLOW>(T, pslot);
    if (posted == POSTED_POSTED) return CT_PENDING_TRANSFER_ALREADY_POSTED;
    if (posted == POSTED_VOIDED) return CT_PENDING_TRANSFER_ALREADY_VOIDED;
    if (!(p.timestamp < t.timestamp)) {
        rp_panic(R, PANIC_ASSERT);
        return R_OK;
    }
    if (p.timeout > 0) {
        const u64 timeout_ns = (u64)p.timeout * 1000000000ULL;
        const u64 expiry = p.timestamp + timeout_ns;
        if (expiry < p.timestamp) {
            rp_panic(R, PANIC_OVERFLOW);
            return R_OK;
        }
        if (t.timestamp >= expiry) return CT_PENDING_TRANSFER_EXPIRED;
    }

    Transfer r;
    r.id = t.id;
    r.debit_account_id = p.debit_account_id;
    r.credit_account_id = p.credit_account_id;
    r.user_data_128 = t.user_data_128 > 0 ? t.user_data_128 : p.user_data_128;
    r.user_data_64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
    r.user_data_32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
    r.ledger = p.ledger;
    r.code = p.code;
    r.pending_id = t.pending_id;
    r.timeout = 0;
    r.timestamp = t.timestamp;
    r.flags = t.flags;
    r.amount = amount;
    rp_transfer_insert<FLOW>(R, r, log_pos);
    if (R.failed) return R_OK;

    rp_push(R, UNDO_POSTED, pslot, nullptr);
    rp_store_posted<FLOW>(T, pslot, (f & TF_POST) ? POSTED_POSTED : POSTED_VOIDED);

    bool dfree, cfree;
    const AccountBal dr0 = rp_balance_load<FLOW>(R, drs, &dfree);
    const AccountBal cr0 = rp_balance_load<FLOW>(R, crs, &cfree);
    AccountBal dr = dr0, cr = cr0;
    // The `-=` asserts (:991-992).  A free account on the flow path is not read: its pending
    // balance covers every outstanding pending transfer (the engine runs the flow path only while
    // no balance was set directly), this one included.
    if ((!dfree && dr.debits_pending < p.amount) || (!cfree && cr.credits_pending < p.amount)) {
        rp_panic(R, PANIC_OVERFLOW);
        return R_OK;
    }
    dr.debits_pending -= p.amount;
    cr.credits_pending -= p.amount;
    if (f & TF_POST) {
        dr.debits_posted = rp_add(R, dr.debits_posted, amount);
        cr.credits_posted = rp_add(R, cr.credits_posted, amount);
    }
    rp_balance_update<FLOW>(R, drs, dr0, dr);
    rp_balance_update<FLOW>(R, crs, cr0, cr);
    return R_OK;
}

template <bool FLOW>
__device__ static inline u32 rp_create_transfer(Replay& R, const Transfer& t, u32 log_pos,
                                                const FastHint* hint = nullptr) {
    const Tables& T = R.T;
    const u16 f = t.flags;
    if (f & TF_PADDING) return CT_RESERVED_FLAG;
    if (t.id == 0) return CT_ID_MUST_NOT_BE_ZERO;
    if (t.id == TB_U128_MAX) return CT_ID_MUST_NOT_BE_INT_MAX;
    if (f & (TF_POST | TF_VOID)) return rp_post_or_void<FLOW>(R, t, log_pos, hint);

    if (t.debit_account_id == 0) return CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.debit_account_id == TB_U128_MAX) return CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == 0) return CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t.credit_account_id == TB_U128_MAX) return CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t.credit_account_id == t.debit_account_id) return CT_ACCOUNTS_MUST_BE_DIFFERENT;
    if (t.pending_id != 0) return CT_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TF_PENDING)) {
        if (t.timeout != 0) return CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    }
    if (!(f & (TF_BAL_DEBIT | TF_BAL_CREDIT))) {
        if (t.amount == 0) return CT_AMOUNT_MUST_NOT_BE_ZERO;
    }
    if (t.ledger == 0) return CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t.code == 0) return CT_CODE_MUST_NOT_BE_ZERO;

    const u32 drs = hint ? hint->drs : tb_account_find(T, tb_lo(t.debit_account_id), tb_hi(t.debit_account_id));
    if (drs == TB_NOT_FOUND) return CT_DEBIT_ACCOUNT_NOT_FOUND;
    const u32 crs = hint ? hint->crs : tb_account_find(T, tb_lo(t.credit_account_id), tb_hi(t.credit_account_id));
    if (crs == TB_NOT_FOUND) return CT_CREDIT_ACCOUNT_NOT_FOUND;
    const AccountHot dh = T.acct_hot[drs];
    const AccountHot ch = T.acct_hot[crs];
    bool dfree, cfree;
    const AccountBal dr0 = rp_balance_load<FLOW>(R, drs, &dfree);
    const AccountBal cr0 = rp_balance_load<FLOW>(R, crs, &cfree);
    AccountBal dr = dr0, cr = cr0;
    if (!(t.timestamp > dh.timestamp) || !(t.timestamp > ch.timestamp)) {
        rp_panic(R, PANIC_ASSERT);
        return R_OK;
    }
    if (dh.ledger != ch.ledger) return CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t.ledger != dh.ledger) return CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    const bool revive = hint && hint->known_new;
    const u32 es = revive ? TB_NOT_FOUND : rp_transfer_find<FLOW>(T, tb_lo(t.id), tb_hi(t.id));
    if (es != TB_NOT_FOUND) return tb_transfer_exists(t, rp_load<FLOW>(&T.xlog[es]));

    u128 amount = t.amount;
    if (f & (TF_BAL_DEBIT | TF_BAL_CREDIT)) {
        if (amount == 0) amount = (u128)UINT64_MAX;  // maxInt(u64) (:829)
    }
    if (f & TF_BAL_DEBIT) {
        const u128 bal = rp_add(R, dr.debits_posted, dr.debits_pending);
        const u128 room = dr.credits_posted > bal ? dr.credits_posted - bal : 0;  // -|
        if (room < amount) amount = room;
        if (amount == 0) return CT_EXCEEDS_CREDITS;
    }
    if (f & TF_BAL_CREDIT) {
        const u128 bal = rp_add(R, cr.credits_posted, cr.credits_pending);
        const u128 room = cr.debits_posted > bal ? cr.debits_posted - bal : 0;
        if (room < amount) amount = room;
        if (amount == 0) return CT_EXCEEDS_DEBITS;
    }
    if (R.failed) return R_OK;

    // Overflow checks (:848-861).  A free account on the flow path reads as zero here; the global
    // certificate holds, so none of these could fire for its real value either.
    u128 r;
    if (f & TF_PENDING) {
        if (tb_add_overflows(amount, dr.debits_pending, &r)) return CT_OVERFLOWS_DEBITS_PENDING;
        if (tb_add_overflows(amount, cr.credits_pending, &r)) return CT_OVERFLOWS_CREDITS_PENDING;
    }
    if (tb_add_overflows(amount, dr.debits_posted, &r)) return CT_OVERFLOWS_DEBITS_POSTED;
    if (tb_add_overflows(amount, cr.credits_posted, &r)) return CT_OVERFLOWS_CREDITS_POSTED;
    if (tb_add_overflows(amount, rp_add(R, dr.debits_pending, dr.debits_posted), &r)) return CT_OVERFLOWS_DEBITS;
    if (tb_add_overflows(amount, rp_add(R, cr.credits_pending, cr.credits_posted), &r)) return CT_OVERFLOWS_CREDITS;
    if (R.failed) return R_OK;
    const u64 timeout_ns = (u64)t.timeout * 1000000000ULL;
    if (t.timestamp + timeout_ns < t.timestamp) return CT_OVERFLOWS_TIMEOUT;
    // debits_exceed_credits / credits_exceed_debits (tigerbeetle.zig:31-39).
    if ((dh.flags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        rp_add(R, rp_add(R, dr.debits_pending, dr.debits_posted), amount) > dr.credits_posted) {
        return CT_EXCEEDS_CREDITS;
    }
    if ((ch.flags & AF_CREDITS_MUST_NOT_EXCEED_DEBITS) &&
        rp_add(R, rp_add(R, cr.credits_pending, cr.credits_posted), amount) > cr.debits_posted) {
        return CT_EXCEEDS_DEBITS;
    }
    if (R.failed) return R_OK;

    Transfer t2 = t;
    t2.amount = amount;
    if (hint && hint->rec) {  // the record is in place: revive kernel 1's entry (undone by a tombstone)
        atomicAnd((unsigned long long*)&R.T.xidx[hint->entry], ~(unsigned long long)XI_TOMB);
        R.xcount++;  // only the flow path passes a hint
        rp_push(R, UNDO_TRANSFER_INSERT, hint->entry, nullptr);
    } else if (revive) {  // the id is new: store the record, revive kernel 1's entry
        rp_store<FLOW>(&R.T.xlog[log_pos], t2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the record before its index entry
        atomicAnd((unsigned long long*)&R.T.xidx[hint->entry], ~(unsigned long long)XI_TOMB);
        R.xcount++;  // only the flow path passes a hint
        rp_push(R, UNDO_TRANSFER_INSERT, hint->entry, nullptr);
    } else {
        rp_transfer_insert<FLOW>(R, t2, log_pos);
    }
    if (R.failed) return R_OK;
    if (f & TF_PENDING) {
        dr.debits_pending = rp_add(R, dr.debits_pending, amount);
        cr.credits_pending = rp_add(R, cr.credits_pending, amount);
    } else {
        dr.debits_posted = rp_add(R, dr.debits_posted, amount);
        cr.credits_posted = rp_add(R, cr.credits_posted, amount);
    }
    rp_balance_update<FLOW>(R, drs, dr0, dr);
    rp_balance_update<FLOW>(R, crs, cr0, cr);
    return R_OK;
}

__device__ static inline u32 rp_create_account(Replay& R, const Account& a) {
    const u32 code = tb_account_stateless(a);
    if (code != R_OK) return code;
    const u32 es = tb_account_find(R.T, tb_lo(a.id), tb_hi(a.id));
    if (es != TB_NOT_FOUND) return tb_account_exists(a, tb_account_load(R.T, es));
    const u32 slot = tb_account_claim(R.T, tb_lo(a.id), tb_hi(a.id), a.timestamp);
    if (slot == TB_NOT_FOUND) {
        R.failed = true;
        return R_OK;
    }
    tb_account_store_new(R.T, slot, a);
    R.T.g->account_count++;
    rp_push(R, UNDO_ACCOUNT_INSERT, slot, nullptr);
    return R_OK;
}

// Replay the dependent events of batch b (lane 0 only).  Returns the max ok timestamp.
template <u8 OP>
__device__ static inline u64 rp_batch(const PassArgs& P, Replay& R, u32 b) {
    const u64 boff = P.batch_off[b];
    const u32 L = (u32)(P.batch_off[b + 1] - boff);
    const u32 pbase = (u32)(boff - P.e0);
    const u32 nd = P.dep_count[b - P.b0];
    const u32* list = P.dep_list + pbase;
    u64 tsmax = 0;
    bool in_chain = false, broken = false;
    u32 chain_k = 0;
    for (u32 k = 0; k < nd && !R.failed; k++) {
        const u32 i = list[k];
        const u8* ev = P.events + (boff + i) * 128;
        const u16 flags = P.eflags[pbase + i];
        const u64 evts = (P.routed || (P.info[pbase + i] & HZ_INPLACE)) ? 0 : *(const u64*)(ev + 120);  // stamped in place
        const bool linked = flags & 1;
        u32 result;
        if (linked && !in_chain) {
            in_chain = true;
            chain_k = k;
            R.scope = true;
            R.undo_len = 0;
        }
        if (linked && i == L - 1) {
            result = R_LINKED_EVENT_CHAIN_OPEN;
        } else if (broken) {
            result = R_LINKED_EVENT_FAILED;
        } else if (evts != 0) {
            result = R_TIMESTAMP_MUST_BE_ZERO;
        } else {
            const u64 ts = tb_event_ts(P, b, boff, L, i);
            if (OP == OP_CREATE_TRANSFERS) {
                Transfer t = *(const Transfer*)ev;
                t.timestamp = ts;
                result = rp_create_transfer<false>(R, t, (u32)(R.log_base + pbase + i));
            } else {
                Account a = *(const Account*)ev;
                a.timestamp = ts;
                result = rp_create_account(R, a);
            }
            if (result == R_OK && !R.failed) tsmax = ts;
        }
        if (R.failed) break;
        if (result != R_OK && in_chain && !broken) {
            broken = true;
            rp_scope_close<false>(R, false);
            for (u32 kk = chain_k; kk < k; kk++) {
                u32* w = &P.info[pbase + list[kk]];
                *w = (*w & 0xFFFFFF00u) | R_LINKED_EVENT_FAILED;
            }
        }
        u32* w = &P.info[pbase + i];
        *w = (*w & 0xFFFFFF00u) | result;
        if (in_chain && (!linked || result == R_LINKED_EVENT_CHAIN_OPEN)) {
            if (!broken) rp_scope_close<false>(R, true);
            in_chain = false;
            broken = false;
        }
    }
    return tsmax;
}

template <u8 OP>
__global__ __launch_bounds__(REPLAY_THREADS) void tb_replay(PassArgs P, UndoEntry* undo, u32 undo_cap) {
    __shared__ u8 s_code[BATCH_LDS];
    __shared__ u32 s_wave[REPLAY_THREADS / 64];
    __shared__ u32 s_list[REPLAY_THREADS];
    __shared__ u32 s_nlist;
    __shared__ u32 s_failed;
    Globals* g = P.T.g;
    const u32 nb = P.b1 - P.b0;
    if (threadIdx.x == 0) s_failed = 0;
    __syncthreads();
    const bool any = *(volatile u64*)&g->dependent_total != 0;
    if (any) {
        Replay R;
        R.T = P.T;
        R.undo = undo;
        R.undo_len = 0;
        R.undo_cap = undo_cap;
        R.scope = false;
        R.failed = false;
        R.log_base = P.log_base;
        u64 tsmax = 0;
        for (u32 c = 0; c < nb; c += REPLAY_THREADS) {
            const u32 k = c + threadIdx.x;
            const bool has = k < nb && P.dep_count[k] > 0;
            u32 total;
            const u32 r = tb_block_rank(has, s_wave, total);
            if (has) s_list[r] = k;
            if (threadIdx.x == 0) s_nlist = total;
            __syncthreads();
            const u32 nl = s_nlist;
            for (u32 q = 0; q < nl; q++) {
                const u32 b = P.b0 + s_list[q];
                if (threadIdx.x == 0) {
                    if (!s_failed) {
                        const u64 m = rp_batch<OP>(P, R, b);
                        tsmax = max(tsmax, m);
                        if (R.failed) s_failed = 1;
                    }
                }
                __syncthreads();
                // The batch's final codes are in P.info now; write its reply.
                const u64 boff = P.batch_off[b];
                const u32 L = (u32)(P.batch_off[b + 1] - boff);
                const u32 pbase = (u32)(boff - P.e0);
                for (u32 i = threadIdx.x; i < L; i += REPLAY_THREADS) s_code[i] = (u8)(P.info[pbase + i] & 0xFF);
                __syncthreads();
                tb_write_replies(P, b, L, s_code, s_wave);
                __syncthreads();
            }
            __syncthreads();
        }
        if (threadIdx.x == 0 && tsmax > g->commit_timestamp) g->commit_timestamp = tsmax;
    }
    if (threadIdx.x == 0) {
        // Close the pass: bound += S, reset the dependent counter.
        if (P.op == OP_CREATE_TRANSFERS) {
            const u128 S = tb_sum_total(P.sum_shards);
            const u128 nb2 = tb_sat_add(tb_u128(g->bound_lo, g->bound_hi), S);
            g->bound_lo = tb_lo(nb2);
            g->bound_hi = tb_hi(nb2);
        }
        g->dependent_all += g->dependent_total;
        g->dependent_total = 0;
    }
}
