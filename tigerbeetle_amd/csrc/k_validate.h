// k_validate.h — kernel 1 of a pass: one event per lane.
//
// Computes each event's *intrinsic* result against the pre-pass HBM state, in the reference's code
// order (create_transfer state_machine.zig:779-884, post_or_void_pending_transfer :907-1014,
// create_account :738-765), plus the hazard bits the resolve kernel needs to decide whether that
// result can be trusted (see DESIGN.md "Dependence").
#pragma once

#include "pass.h"

#define TB_CODE_PANIC 63u  // the reference would trap if this event were evaluated in sequence

struct TransferScratch {
    u32 hz = 0;
    u32 dr = TB_NOT_FOUND, cr = TB_NOT_FOUND;
    u32 ps = TB_NOT_FOUND;  // log position of the pending transfer (post/void)
    u32 rs = TB_NOT_FOUND;  // index entry claimed by the speculative insert
    u128 amount = 0;        // amount applied by an independent ok event (post: posted amount)
    u128 contrib = 0;       // contribution to S (overflow certificate)
    u64 kid = 0, kpid = 0;  // dedup keys of id / pending_id
    u64 rec_ts = 0;         // != 0: the event's record is the event with this timestamp (written
                            // from the LDS stage by the whole workgroup, coalesced)
};

// create_transfer_exists (state_machine.zig:886-905).
__device__ static inline u32 tb_transfer_exists(const Transfer& t, const Transfer& e) {
    if (t.flags != e.flags) return CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t.debit_account_id != e.debit_account_id) return CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (t.credit_account_id != e.credit_account_id) return CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t.amount != e.amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    if (t.user_data_128 != e.user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t.user_data_64 != e.user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t.user_data_32 != e.user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t.timeout != e.timeout) return CT_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t.code != e.code) return CT_EXISTS_WITH_DIFFERENT_CODE;
    return CT_EXISTS;
}

// post_or_void_pending_transfer_exists (state_machine.zig:1016-1077).
__device__ static inline u32 tb_post_void_exists(const Transfer& t, const Transfer& e, const Transfer& p) {
    if (t.flags != e.flags) return CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t.amount == 0) {
        if (e.amount != p.amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (t.amount != e.amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (t.pending_id != e.pending_id) return CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (t.user_data_128 == 0) {
        if (e.user_data_128 != p.user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else {
        if (t.user_data_128 != e.user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t.user_data_64 == 0) {
        if (e.user_data_64 != p.user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else {
        if (t.user_data_64 != e.user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t.user_data_32 == 0) {
        if (e.user_data_32 != p.user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else {
        if (t.user_data_32 != e.user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    return CT_EXISTS;
}

// The record of a post / void (post_or_void_pending_transfer :971-985): the event's fields where it
// gives them, the pending transfer's otherwise.
__device__ static inline Transfer tb_compose_post_void(const Transfer& t, const Transfer& p, u64 ts) {
    Transfer r;
    r.id = t.id;
    r.debit_account_id = p.debit_account_id;
    r.credit_account_id = p.credit_account_id;
    r.amount = t.amount > 0 ? t.amount : p.amount;
    r.pending_id = t.pending_id;
    r.user_data_128 = t.user_data_128 > 0 ? t.user_data_128 : p.user_data_128;
    r.user_data_64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
    r.user_data_32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
    r.timeout = 0;
    r.ledger = p.ledger;
    r.code = p.code;
    r.flags = t.flags;
    r.timestamp = ts;
    return r;
}

// The `id` existence check of create_transfer (:824) / post_or_void (:954) fused with the
// speculative index claim.  Returns R_OK (claimed, record to be written by the caller),
// a pseudo "exists" marker via *exists_pos, or CLAIM_COLLIDED (dependent).
__device__ static inline u32 tb_claim_id(const PassArgs& P, const Transfer& t, u32 pe, TransferScratch& s,
                                         u32* exists_pos, u64 first = ~0ULL) {
    s.kid = tb_dedup_key(tb_lo(t.id), tb_hi(t.id));
    if (TB_ABL(P, ABL_SPEC)) return CLAIM_NEW;
    u32 entry = TB_NOT_FOUND;
    if (TB_ABL(P, ABL_CAS)) {  // timing only: no atomic claim
        s.rs = (u32)(tb_hash_id(tb_lo(t.id), tb_hi(t.id)) & P.T.xidx_mask);
        s.hz |= HZ_SPEC;
        return CLAIM_NEW;
    }
    const u32 r = tb_transfer_claim(P.T, tb_lo(t.id), tb_hi(t.id), P.log_base + pe, P.log_base, exists_pos, &entry,
                                    first);
    if (r == CLAIM_NEW) {
        s.rs = entry;
        s.hz |= HZ_SPEC;
    } else if (r == CLAIM_COLLIDED) {
        s.hz |= HZ_SELFDEP;
        P.pass_words[PW_DUP] = 1;
    }
    return r;
}

// Claims are never withdrawn here: an entry claimed by an event that then fails stays claimed
// until kernel 2 tombstones it, so it keeps detecting same-pass collisions on its id (a later
// same-id event collides with it and both are replayed in order).
__device__ static inline u32 tb_validate_post_void(const PassArgs& P, const Transfer& t, u64 ts, u32 pe,
                                                   TransferScratch& s) {
    const Tables& T = P.T;
    const u16 f = t.flags;
    if ((f & TF_POST) && (f & TF_VOID)) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_PENDING) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_DEBIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_CREDIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (t.pending_id == 0) return CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (t.pending_id == TB_U128_MAX) return CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (t.pending_id == t.id) return CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t.timeout != 0) return CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    // From here the result reads the state of pending_id and of id.  Register both now (the
    // pending-dependent checks below may change under the replay): pending_id in the pass pending
    // set, id by claiming its index entry.
    s.hz |= HZ_POSTVOID | HZ_PV_KEY;
    P.pass_words[PW_PV] = 1;
    s.kpid = tb_dedup_key(tb_lo(t.pending_id), tb_hi(t.pending_id));
    tb_dedup_mark(P);
    if (tb_dedup_insert(P.dedup, P.dedup_mask, s.kpid)) P.pass_words[PW_DUP] = 1;
    u32 es = TB_NOT_FOUND;
    const u32 claim = tb_claim_id(P, t, pe, s, &es);
    if (claim == CLAIM_COLLIDED) return R_OK;  // dependent: the replay decides

    const u32 pslot = tb_transfer_find(T, tb_lo(t.pending_id), tb_hi(t.pending_id));
    if (pslot != TB_NOT_FOUND && (u64)pslot >= P.log_base) {  // pending created in this pass
        s.hz |= HZ_SELFDEP;
        return R_OK;
    }
    if (pslot == TB_NOT_FOUND) return CT_PENDING_TRANSFER_NOT_FOUND;
    const Transfer p = T.xlog[pslot];
    if (!(p.flags & TF_PENDING)) return CT_PENDING_TRANSFER_NOT_PENDING;

    const u32 drs = tb_account_find(T, tb_lo(p.debit_account_id), tb_hi(p.debit_account_id));
    const u32 crs = tb_account_find(T, tb_lo(p.credit_account_id), tb_hi(p.credit_account_id));
    if (drs == TB_NOT_FOUND || crs == TB_NOT_FOUND) return TB_CODE_PANIC;  // `.?` at :929-930

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

    if (claim == CLAIM_EXISTS) return tb_post_void_exists(t, T.xlog[es], p);

    const u8 posted = T.xposted[pslot];
    if (posted == POSTED_POSTED) return CT_PENDING_TRANSFER_ALREADY_POSTED;
    if (posted == POSTED_VOIDED) return CT_PENDING_TRANSFER_ALREADY_VOIDED;

    if (!(p.timestamp < ts)) return TB_CODE_PANIC;
    if (p.timeout > 0) {
        const u64 timeout_ns = (u64)p.timeout * 1000000000ULL;
        const u64 expiry = p.timestamp + timeout_ns;
        if (expiry < p.timestamp) return TB_CODE_PANIC;  // checked `+` at :968
        if (ts >= expiry) return CT_PENDING_TRANSFER_EXPIRED;
    }

    s.dr = drs;
    s.cr = crs;
    s.ps = pslot;
    s.hz |= HZ_ACCTS;
    if ((T.acct_hot[drs].flags | T.acct_hot[crs].flags) & AF_LIMITS) s.hz |= HZ_LIMIT;
    s.amount = (f & TF_POST) ? amount : 0;
    // A post moves <= p.amount from pending to posted: dp + dpost never grows, so no S term.

    // Speculative record (composed as at :971-985); kernel 2 withdraws it if the event fails.
    if ((s.hz & HZ_SPEC) && !P.inplace) T.xlog[P.log_base + pe] = tb_compose_post_void(t, p, ts);  // in place: tb_resolve
    return R_OK;
}

__device__ static inline u32 tb_validate_transfer(const PassArgs& P, const Transfer& t, u64 ts, u32 pe,
                                                  TransferScratch& s) {
    const Tables& T = P.T;
    const u16 f = t.flags;
    if (f & TF_PADDING) return CT_RESERVED_FLAG;
    if (t.id == 0) return CT_ID_MUST_NOT_BE_ZERO;
    if (t.id == TB_U128_MAX) return CT_ID_MUST_NOT_BE_INT_MAX;

    if (f & (TF_POST | TF_VOID)) return tb_validate_post_void(P, t, ts, pe, s);

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

    // The first probe of both accounts and the claim of the id's home index entry are independent:
    // issue them together, before any result is consumed.  The claim is speculative (the id check
    // comes after the account checks, :813-824); if the event fails first, kernel 2 withdraws it.
    const u64 dlo = tb_lo(t.debit_account_id), dhi = tb_hi(t.debit_account_id);
    const u64 clo = tb_lo(t.credit_account_id), chi = tb_hi(t.credit_account_id);
    const u64 dpos = tb_hash_id(dlo, dhi) & T.account_mask;
    const u64 cpos = tb_hash_id(clo, chi) & T.account_mask;
    const u64 xpos = tb_hash_id(tb_lo(t.id), tb_hi(t.id)) & T.xidx_mask;
    const bool fake = TB_ABL(P, ABL_ACCTS);
    AccountHot d0 = {}, c0 = {};
    if (!fake) {
        d0 = T.acct_hot[dpos];
        c0 = T.acct_hot[cpos];
    }
    u64 x0 = ~0ULL;
    if (!TB_ABL(P, ABL_SPEC | ABL_CAS)) {
        x0 = tb_transfer_cas_home(T, tb_lo(t.id), tb_hi(t.id), (u32)(P.log_base + pe), xpos);
        if (x0 == 0) {
            s.rs = (u32)xpos;
            s.hz |= HZ_SPEC;
        }
    }
    AccountHot dr = {}, cr = {};
    u32 drs, crs;
    if (fake) {
        drs = (u32)(dlo & 1023);
        crs = (u32)(clo & 1023);
    } else {
        tb_account_find2(T, dlo, dhi, dpos, d0, clo, chi, cpos, c0, &drs, &crs, &dr, &cr);
    }
    u32 early = R_OK;
    if (drs == TB_NOT_FOUND) early = CT_DEBIT_ACCOUNT_NOT_FOUND;
    else if (crs == TB_NOT_FOUND) early = CT_CREDIT_ACCOUNT_NOT_FOUND;
    else if (!(ts > dr.timestamp) || !(ts > cr.timestamp)) early = TB_CODE_PANIC;  // :817-818
    else if (dr.ledger != cr.ledger) early = CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    else if (t.ledger != dr.ledger) early = CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
    const bool balancing = (f & (TF_BAL_DEBIT | TF_BAL_CREDIT)) != 0;
    if (early == R_OK) {
        // From here the event may end up ok: account for it in S and mark balancing accounts before
        // the id check, so that a dependent (colliding) event is covered too.
        s.contrib = balancing && t.amount == 0 ? (u128)UINT64_MAX : t.amount;
        s.dr = drs;
        s.cr = crs;
        s.hz |= HZ_ACCTS;
        if ((dr.flags | cr.flags) & AF_LIMITS) s.hz |= HZ_LIMIT;
        if (balancing) {
            // The amount depends on the running balance (:826-846): dependent, and so is every event
            // touching the balanced account in this pass.
            s.hz |= HZ_BAL;
            if (f & TF_BAL_DEBIT) P.T.account_mark[drs] = P.epoch;
            if (f & TF_BAL_CREDIT) P.T.account_mark[crs] = P.epoch;
            P.pass_words[PW_BAL] = 1;
        }
    }
    // The existence check of `id` (:824) fused with the speculative claim of its index entry.  An
    // event that failed the account checks claims too (its home entry was claimed with the probes
    // anyway): which same-pass events collide, and so which are dependent, is then a function of the
    // input, not of the order the claims landed in (tests/harness/dependence.py).
    u32 es = TB_NOT_FOUND;
    const u32 claim = tb_claim_id(P, t, pe, s, &es, x0);
    if (early != R_OK) return early;
    if (claim == CLAIM_EXISTS) return tb_transfer_exists(t, T.xlog[es]);
    if (claim == CLAIM_COLLIDED || balancing) return R_OK;  // dependent: the replay decides

    s.amount = t.amount;
    // Overflow checks (:848-861) are certified impossible or the event is dependent (resolve);
    // then the timeout check (:862) is the next possible failure.
    const u64 timeout_ns = (u64)t.timeout * 1000000000ULL;
    if (ts + timeout_ns < ts) return CT_OVERFLOWS_TIMEOUT;  // entry withdrawn by kernel 2
    if ((s.hz & HZ_SPEC) && P.inplace) {
        // The record is the event in place: 8 bytes of it written here (its line was just read).  The
        // ordered path reads an HZ_INPLACE event's timestamp field as the 0 it was checked to be.
        s.hz |= HZ_INPLACE;
        P.T.xlog[P.log_base + pe].timestamp = ts;
    } else if ((s.hz & HZ_SPEC) && !TB_ABL(P, ABL_RECORD)) {
        s.rec_ts = ts;
        s.hz |= HZ_REC;
    }
    return R_OK;
}

// Kernel 1 (create_transfers).
// LDS is the 32 KB stage only (five workgroups per CU): the batch search runs on the scalar unit,
// each wave stores its own records, and the block's S partials go through the stage rows their
// waves have finished with.
template <bool SRC>
__global__ __launch_bounds__(VALIDATE_THREADS) void tb_transfers_validate(PassArgs P) {
    __shared__ __attribute__((aligned(16))) u8 stage[VALIDATE_THREADS * STAGE_STRIDE];

    const u32 tile0 = blockIdx.x * VALIDATE_THREADS;
    const u32 count = min((u32)VALIDATE_THREADS, P.n - tile0);
    tb_stage_tile<SRC>(P, tile0, count, stage, TB_ABL(P, EXP_NT));

    const u32 pe = tile0 + threadIdx.x;  // pass-relative event
    const u64 e = P.e0 + pe;
    const u32 b = tb_wave_batch(P.batch_off, P.b0, P.b1, P.e0 + tile0, count, e);
    TransferScratch s;
    if (threadIdx.x < count) {
        Transfer t = tb_read_staged<Transfer>(stage);
        const u32 L = (u32)(P.batch_off[b + 1] - P.batch_off[b]);
        const u32 j = (u32)(e - P.batch_off[b]);
        u32 code;
        u64 routed_ts = 0;
        if (P.routed) {
            if (t.flags & (TF_LINKED | TF_POST | TF_VOID | TF_BAL_DEBIT | TF_BAL_CREDIT)) {
                tb_panic(P.T.g, PANIC_ASSERT);  // routed shards never receive these (router bug)
            }
            routed_ts = t.timestamp;
            t.timestamp = 0;
        }
        if ((t.flags & TF_LINKED) && j == L - 1) {
            code = R_LINKED_EVENT_CHAIN_OPEN;  // execute :632-640
        } else if (t.timestamp != 0) {
            code = R_TIMESTAMP_MUST_BE_ZERO;  // :643
        } else {
            const u64 ts = P.routed ? routed_ts : P.ev_ts ? P.ev_ts[e] : P.batch_ts[b] - L + j + 1;  // :645
            code = tb_validate_transfer(P, t, ts, pe, s);
        }
        if (tb_hi(s.amount)) s.hz |= HZ_AMT_HI;
        P.info[pe] = code | s.hz;
        P.eflags[pe] = t.flags;
        P.dr[pe] = s.dr;
        P.cr[pe] = s.cr;
        // ps and kpid are read only for post/void events (HZ_POSTVOID / HZ_PV_KEY): 12 B per event
        // of scratch writes skipped for the others.
        if (s.hz & (HZ_POSTVOID | HZ_PV_KEY)) {
            P.ps[pe] = s.ps;
            P.kpid[pe] = s.kpid;
        }
        P.rs[pe] = s.rs;
        // 26 B of scratch per event in the common case: the amount's high word only when it is
        // non-zero, and no id key (tb_resolve recomputes it from the event when a post/void of
        // the pass makes it matter).
        P.amt[pe] = tb_lo(s.amount);
        if (s.hz & HZ_AMT_HI) P.amt_hi[pe] = tb_hi(s.amount);
        if (code != R_OK) s.contrib = 0;
        // The record (create_transfer :870) is the event as staged, with its timestamp.
        if (s.rec_ts) *(u64*)(stage + tb_stage_off(threadIdx.x, 7) + 8) = s.rec_ts;  // timestamp @120
    }
    const u128 w = tb_wave_sum_u128(s.contrib);
    const u64 rec = __ballot(s.rec_ts != 0);
    const u32 lane = threadIdx.x & 63, w0 = threadIdx.x & ~63u;
    // The wave's records (its own 64 stage rows): consecutive lanes store consecutive 16-B chunks
    // of consecutive records.  LDS operations of one wave complete in order, so the timestamps
    // written above are visible here without a workgroup barrier.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (u32 r = 0; r < 8; r++) {
        const u32 c = lane + r * 64;
        const u32 row = c >> 3, part = c & 7;
        if ((rec >> row) & 1) {
            const u32x4 v = *(const u32x4*)(stage + tb_stage_off(w0 + row, part));
            u32x4* dst = (u32x4*)&P.T.xlog[P.log_base + tile0 + w0 + row] + part;
            if (TB_ABL(P, EXP_NT)) __builtin_nontemporal_store(v, dst);
            else *dst = v;
        }
    }
    // Block partial of S (saturating), then one sharded atomic per block.  Each wave parks its
    // partial in the first row of its own stage rows, which it has finished reading.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        *(u64*)(stage + w0 * STAGE_STRIDE) = tb_lo(w);
        *(u64*)(stage + w0 * STAGE_STRIDE + 8) = tb_hi(w);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        u128 total = 0;
        for (u32 k = 0; k < VALIDATE_THREADS / 64; k++) {
            const u8* q = stage + k * 64 * STAGE_STRIDE;
            total = tb_sat_add(total, tb_u128(*(const u64*)q, *(const u64*)(q + 8)));
        }
        tb_sum_publish(P, total);
    }
}

// create_account_exists (state_machine.zig:767-777).
__device__ static inline u32 tb_account_exists(const Account& a, const Account& e) {
    if (a.flags != e.flags) return CA_EXISTS_WITH_DIFFERENT_FLAGS;
    if (a.user_data_128 != e.user_data_128) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a.user_data_64 != e.user_data_64) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a.user_data_32 != e.user_data_32) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a.ledger != e.ledger) return CA_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a.code != e.code) return CA_EXISTS_WITH_DIFFERENT_CODE;
    return CA_EXISTS;
}

// Stateless prefix of create_account (state_machine.zig:741-756).
__device__ static inline u32 tb_account_stateless(const Account& a) {
    if (a.reserved != 0) return CA_RESERVED_FIELD;
    if (a.flags & AF_PADDING) return CA_RESERVED_FLAG;
    if (a.id == 0) return CA_ID_MUST_NOT_BE_ZERO;
    if (a.id == TB_U128_MAX) return CA_ID_MUST_NOT_BE_INT_MAX;
    if ((a.flags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS) && (a.flags & AF_CREDITS_MUST_NOT_EXCEED_DEBITS)) {
        return CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    }
    if (a.debits_pending != 0) return CA_DEBITS_PENDING_MUST_BE_ZERO;
    if (a.debits_posted != 0) return CA_DEBITS_POSTED_MUST_BE_ZERO;
    if (a.credits_pending != 0) return CA_CREDITS_PENDING_MUST_BE_ZERO;
    if (a.credits_posted != 0) return CA_CREDITS_POSTED_MUST_BE_ZERO;
    if (a.ledger == 0) return CA_LEDGER_MUST_NOT_BE_ZERO;
    if (a.code == 0) return CA_CODE_MUST_NOT_BE_ZERO;
    return R_OK;
}

// Kernel 1 (create_accounts).
template <bool SRC>
__global__ __launch_bounds__(VALIDATE_THREADS) void tb_accounts_validate(PassArgs P) {
    __shared__ __attribute__((aligned(16))) u8 stage[VALIDATE_THREADS * STAGE_STRIDE];
    const u32 tile0 = blockIdx.x * VALIDATE_THREADS;
    const u32 count = min((u32)VALIDATE_THREADS, P.n - tile0);
    tb_stage_tile<SRC>(P, tile0, count, stage);
    const u32 pe = tile0 + threadIdx.x;
    const u64 e = P.e0 + pe;
    const u32 b = tb_wave_batch(P.batch_off, P.b0, P.b1, P.e0 + tile0, count, e);
    if (threadIdx.x >= count) return;

    const Account a = tb_read_staged<Account>(stage);
    const u32 L = (u32)(P.batch_off[b + 1] - P.batch_off[b]);
    const u32 j = (u32)(e - P.batch_off[b]);
    u32 code, hz = 0;
    u64 kid = 0;
    if ((a.flags & AF_LINKED) && j == L - 1) {
        code = R_LINKED_EVENT_CHAIN_OPEN;
    } else if (a.timestamp != 0) {
        code = R_TIMESTAMP_MUST_BE_ZERO;
    } else {
        code = tb_account_stateless(a);
        if (code == R_OK) {
            hz |= HZ_KEYS;
            kid = tb_dedup_key(tb_lo(a.id), tb_hi(a.id));
            tb_dedup_mark(P);
            if (tb_dedup_insert(P.dedup, P.dedup_mask, kid)) P.pass_words[PW_DUP] = 1;
            const u32 slot = tb_account_find(P.T, tb_lo(a.id), tb_hi(a.id));
            if (slot != TB_NOT_FOUND) code = tb_account_exists(a, tb_account_load(P.T, slot));
        }
    }
    P.info[pe] = code | hz;
    P.eflags[pe] = a.flags;
    P.kid[pe] = kid;
    P.kpid[pe] = 0;
}
