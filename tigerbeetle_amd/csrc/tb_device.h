// tb_device.h — records, result codes and HBM tables of the MI355X commit engine.
//
// Layouts follow src/tigerbeetle.zig:7-104 (Account / Transfer extern structs, 128 B, align 16);
// result codes follow src/tigerbeetle.zig:109-229 (values == declaration index).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define TB_U128_MAX (~(u128)0)

struct alignas(16) Account {
    u128 id;
    u128 debits_pending;
    u128 debits_posted;
    u128 credits_pending;
    u128 credits_posted;
    u128 user_data_128;
    u64 user_data_64;
    u32 user_data_32;
    u32 reserved;
    u32 ledger;
    u16 code;
    u16 flags;
    u64 timestamp;
};

struct alignas(16) Transfer {
    u128 id;
    u128 debit_account_id;
    u128 credit_account_id;
    u128 amount;
    u128 pending_id;
    u128 user_data_128;
    u64 user_data_64;
    u32 user_data_32;
    u32 timeout;
    u32 ledger;
    u16 code;
    u16 flags;
    u64 timestamp;
};

static_assert(sizeof(Account) == 128, "Account is 128 bytes");
static_assert(sizeof(Transfer) == 128, "Transfer is 128 bytes");


// AccountFlags (tigerbeetle.zig:42-62), TransferFlags (:91-104).
enum : u16 {
    AF_LINKED = 1, AF_DEBITS_MUST_NOT_EXCEED_CREDITS = 2, AF_CREDITS_MUST_NOT_EXCEED_DEBITS = 4,
    AF_LIMITS = 6, AF_PADDING = 0xFFF8,
};
enum : u16 {
    TF_LINKED = 1, TF_PENDING = 2, TF_POST = 4, TF_VOID = 8, TF_BAL_DEBIT = 16, TF_BAL_CREDIT = 32,
    TF_PADDING = 0xFFC0,
};

enum : u8 {
    OP_CREATE_ACCOUNTS = 128, OP_CREATE_TRANSFERS = 129, OP_LOOKUP_ACCOUNTS = 130,
    OP_LOOKUP_TRANSFERS = 131,
};

// Shared by both result enums.
enum : u32 { R_OK = 0, R_LINKED_EVENT_FAILED = 1, R_LINKED_EVENT_CHAIN_OPEN = 2, R_TIMESTAMP_MUST_BE_ZERO = 3 };

// CreateAccountResult (tigerbeetle.zig:109-143).
enum : u32 {
    CA_RESERVED_FIELD = 4, CA_RESERVED_FLAG = 5, CA_ID_MUST_NOT_BE_ZERO = 6,
    CA_ID_MUST_NOT_BE_INT_MAX = 7, CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 8,
    CA_DEBITS_PENDING_MUST_BE_ZERO = 9, CA_DEBITS_POSTED_MUST_BE_ZERO = 10,
    CA_CREDITS_PENDING_MUST_BE_ZERO = 11, CA_CREDITS_POSTED_MUST_BE_ZERO = 12,
    CA_LEDGER_MUST_NOT_BE_ZERO = 13, CA_CODE_MUST_NOT_BE_ZERO = 14,
    CA_EXISTS_WITH_DIFFERENT_FLAGS = 15, CA_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 16,
    CA_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 17, CA_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 18,
    CA_EXISTS_WITH_DIFFERENT_LEDGER = 19, CA_EXISTS_WITH_DIFFERENT_CODE = 20, CA_EXISTS = 21,
};

// CreateTransferResult (tigerbeetle.zig:145-229).
enum : u32 {
    CT_RESERVED_FLAG = 4, CT_ID_MUST_NOT_BE_ZERO = 5, CT_ID_MUST_NOT_BE_INT_MAX = 6,
    CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 7, CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 8,
    CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 9, CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 10,
    CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 11, CT_ACCOUNTS_MUST_BE_DIFFERENT = 12,
    CT_PENDING_ID_MUST_BE_ZERO = 13, CT_PENDING_ID_MUST_NOT_BE_ZERO = 14,
    CT_PENDING_ID_MUST_NOT_BE_INT_MAX = 15, CT_PENDING_ID_MUST_BE_DIFFERENT = 16,
    CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17, CT_AMOUNT_MUST_NOT_BE_ZERO = 18,
    CT_LEDGER_MUST_NOT_BE_ZERO = 19, CT_CODE_MUST_NOT_BE_ZERO = 20,
    CT_DEBIT_ACCOUNT_NOT_FOUND = 21, CT_CREDIT_ACCOUNT_NOT_FOUND = 22,
    CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER = 23, CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS = 24,
    CT_PENDING_TRANSFER_NOT_FOUND = 25, CT_PENDING_TRANSFER_NOT_PENDING = 26,
    CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID = 27,
    CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID = 28,
    CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER = 29, CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE = 30,
    CT_EXCEEDS_PENDING_TRANSFER_AMOUNT = 31, CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT = 32,
    CT_PENDING_TRANSFER_ALREADY_POSTED = 33, CT_PENDING_TRANSFER_ALREADY_VOIDED = 34,
    CT_PENDING_TRANSFER_EXPIRED = 35, CT_EXISTS_WITH_DIFFERENT_FLAGS = 36,
    CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID = 37, CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID = 38,
    CT_EXISTS_WITH_DIFFERENT_AMOUNT = 39, CT_EXISTS_WITH_DIFFERENT_PENDING_ID = 40,
    CT_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 41, CT_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 42,
    CT_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 43, CT_EXISTS_WITH_DIFFERENT_TIMEOUT = 44,
    CT_EXISTS_WITH_DIFFERENT_CODE = 45, CT_EXISTS = 46, CT_OVERFLOWS_DEBITS_PENDING = 47,
    CT_OVERFLOWS_CREDITS_PENDING = 48, CT_OVERFLOWS_DEBITS_POSTED = 49,
    CT_OVERFLOWS_CREDITS_POSTED = 50, CT_OVERFLOWS_DEBITS = 51, CT_OVERFLOWS_CREDITS = 52,
    CT_OVERFLOWS_TIMEOUT = 53, CT_EXCEEDS_CREDITS = 54, CT_EXCEEDS_DEBITS = 55,
};

// Posted groove value (state_machine.zig:185-198), kept per transfer-table slot of the PENDING
// transfer (the pending timestamp uniquely names that slot).
enum : u8 { POSTED_NONE = 0, POSTED_POSTED = 1, POSTED_VOIDED = 2 };

// Device panic codes (the reference would trap).
enum : u32 {
    PANIC_NONE = 0, PANIC_OVERFLOW = 1, PANIC_ASSERT = 2, PANIC_TABLE_FULL = 4, PANIC_UNDO_FULL = 8,
    PANIC_FLOW_STALL = 16,  // engine bug guard: a flow-path wait exceeded its bound
};

#define TB_NOT_FOUND 0xFFFFFFFFu

// ------------------------------------------------------------------------------------------------
// Hashing.  Ids from IdPermutation.inversion (testing/id.zig:31) differ only in their low bits, so
// both halves go through a full avalanche mixer.
// ------------------------------------------------------------------------------------------------
__host__ __device__ static inline u64 tb_mix64(u64 x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

__host__ __device__ static inline u64 tb_hash_id(u64 lo, u64 hi) {
    return tb_mix64(lo ^ tb_mix64(hi ^ 0x243f6a8885a308d3ULL));
}

// home(id) of a transfer / owner(id) of an account among `world` shards: the top 32 bits of the id
// hash scaled to [0, world) — independent of the low hash bits that pick the table position, so
// each shard's tables stay uniformly loaded.
__host__ __device__ static inline u32 tb_home(u64 lo, u64 hi, u32 world) {
    return (u32)(((tb_hash_id(lo, hi) >> 32) * (u64)world) >> 32);
}

__host__ __device__ static inline u128 tb_u128(u64 lo, u64 hi) { return ((u128)hi << 64) | lo; }
__host__ __device__ static inline u64 tb_lo(u128 v) { return (u64)v; }
__host__ __device__ static inline u64 tb_hi(u128 v) { return (u64)(v >> 64); }

// Checked u128 add: returns true on overflow (sum_overflows, state_machine.zig:1152-1157).
__device__ static inline bool tb_add_overflows(u128 a, u128 b, u128* r) {
    *r = a + b;
    return *r < a;
}

__device__ static inline u128 tb_sat_add(u128 a, u128 b) {
    u128 r = a + b;
    return r < a ? TB_U128_MAX : r;
}

// ------------------------------------------------------------------------------------------------
// Engine state in HBM.
//
// Accounts: open-addressing hash table of 32-byte HOT entries {id, ledger, code, flags, timestamp}
// (one 64-byte sector holds two entries, so a probe step costs one sector), with the balances
// (64 B) and the cold fields (user_data_*, reserved; 32 B) in parallel arrays at the same slot.
//   * empty:     id == 0 (never a live id: id_must_not_be_zero)
//   * tombstone: id == maxInt(u128) (never a live id: id_must_not_be_int_max) — a rolled-back
//                insert; probes continue past it and it is never reclaimed
//   Inserts claim an empty entry with a 64-bit CAS of its timestamp word (0 -> ts; timestamps are
//   always >= 1), then write the id.
//
// Transfers: an append LOG of 128-byte records — event e of a pass is written at log position
// pass_base + e, so kernel 1 stores records fully coalesced — plus an 8-byte INDEX entry per
// record: {fingerprint32 (never 0) << 32 | (log position + 1)}, 0 = empty, bit 31 of the low word
// = TOMB (withdrawn).  One 64-bit CAS publishes a whole entry.  A probe compares fingerprints and
// confirms a match against the log record's id.  A second event of the same pass with the same id
// meets the claimed fingerprint on its probe path (or loses the CAS to it) — that is how same-pass
// duplicate ids are detected, with no separate dedup set.
// ------------------------------------------------------------------------------------------------
#ifndef FL_BAR_GROUPS
#define FL_BAR_GROUPS 8
#endif
#define FL_BAR_STRIDE 32  // u32 words: one 128-B line per counter
#define FL_BAR_WORDS (FL_BAR_GROUPS + 4)
struct Globals {
    u64 commit_timestamp;     // max timestamp of an event that returned ok when evaluated
    u64 panic;                // PANIC_* bits
    u64 log_next;             // next free transfer-log position
    u64 dedup_dirty;          // (pass epoch << 8) | log2(entries) of the last pass that inserted into the dedup set
    u64 bound_lo, bound_hi;   // upper bound of dp+dpost and cp+cpost over every account
    u64 dependent_total;      // dependent events of this pass
    u64 dependent_all;        // cumulative
    u64 account_count;
    u64 transfer_count;
    u64 export_count;
    u32 flow_barrier;         // (unused since the two-level barrier; kept for the layout)
    u32 flow_passes;          // passes whose dependent events ran on the parallel flow path
    u64 flow_units;           // cumulative units (chains / single events) the flow path executed
    u64 flow_runs;            // runs (k_flow.h) and the units they covered
    u64 flow_run_units;
    u64 limit_accounts;       // accounts ever created with a limit flag (never decremented: an upper bound)
    u64 flow_plan_ticks;      // tb_flow wall-clock ticks (workgroup 0): planning, then the ordered run
    u64 flow_run_ticks;
    u64 bounds_passes;        // passes whose dependent events were all decided by bounds (k_flow.h fl_bounds)
    u64 bounds_units;         // units they decided
    u64 bounds_rounds;        // scan rounds they took (and the rounds of abandoned attempts)
    u64 bounds_skipped;       // dependent passes with an event the bounds do not cover (ordered run)
    u64 bounds_swept;         // units the in-order sweep decided (fl_sweep)
    u64 sweep_ticks[3];       // fl_sweep wall-clock ticks: the whole walk, its in-window loops, its memory waits
    u64 flow_phase_ticks[8];  // tb_flow wall-clock ticks per phase (k_flow.h FP_*)
    u64 flow_exec_ticks;      // tb_flow run: lanes' time executing units, summed over lanes
    u64 walk[12];             // fl_walk: segments, heavy segments; over the heavy walkers: positions,
                              // windows, partner stops, blocked returns, blocked ticks; the longest segment;
                              // the critical (longest-segment) walker's windows, waits, wait and total ticks
    u64 walk_dbg[4];          // fl_walk: what a walker that stalled was waiting on (diagnostics)
    u64 sweep_u64_passes;     // sweeps that ran in the u64 X/Y form (bound + S >= 2^63)
    u64 bounds_abandoned;     // passes whose bounds did not converge in FLOW_BOUNDS_ROUNDS_MAX rounds
    // tb_flow's two-level grid barrier (k_flow.h fl_grid_sync): FL_BAR_GROUPS group counters, the
    // root counter, the published generation; then its admission (fl_admit): the entry counter and
    // the admitted grid.  One 128-B line each.  Zeroed by tb_resolve every pass.
    u32 flow_bar[FL_BAR_STRIDE * FL_BAR_WORDS];
};

struct AccountHot {
    u64 id_lo, id_hi;
    u32 ledger;
    u16 code;
    u16 flags;
    u64 timestamp;
};
struct AccountBal {
    u128 debits_pending, debits_posted, credits_pending, credits_posted;
};
struct AccountCold {
    u128 user_data_128;
    u64 user_data_64;
    u32 user_data_32;
    u32 reserved;
};
static_assert(sizeof(AccountHot) == 32 && sizeof(AccountBal) == 64 && sizeof(AccountCold) == 32, "account split");

// Balances in two planes (round 5): the low words of an account's four balances side by side, 32 B
// per slot at lo[4 * slot + f], and their high words the same way in `hi`.  Every balance the engine
// holds stays below 2^64 unless an event makes it larger, and the balance-leg write-back
// (k_apply.h tb_apply_legs) adds low words only under the 64-bit certificate: it reads and writes the
// low plane alone, four accounts to a 128-B line, and never touches a high word.  The two planes are
// one allocation (hi = lo + 4 * account_cap), so a snapshot is one copy of it.
#define BAL_DP 0     // debits_pending
#define BAL_DPOST 1  // debits_posted
#define BAL_CP 2     // credits_pending
#define BAL_CPOST 3  // credits_posted
struct BalView {
    u64* lo;  // [4 * account_cap]
    u64* hi;  // [4 * account_cap]
};

#define XI_TOMB (1ULL << 31)  // withdrawn (failed / dependent / rolled back)
#define XI_POS_MASK 0x7FFFFFFFULL

struct Tables {
    AccountHot* acct_hot;     // [account_cap]
    BalView bal;              // balances, by plane (above)
    AccountCold* acct_cold;   // [account_cap]
    u32* account_mark;        // [account_cap] pass epoch of the last balancing mark
    u64 account_mask;         // account_cap - 1
    u64* xidx;                // [xidx_cap] index entries
    u8* xdup;                 // [xidx_cap] 1: another event of the claiming pass met this entry
    u64 xidx_mask;
    Transfer* xlog;           // [xlog_cap]
    u8* xposted;              // [xlog_cap] POSTED_* of the pending transfer at that log position
    u64 xlog_cap;
    Globals* g;
};

__device__ static inline void tb_panic(Globals* g, u32 code) {
    atomicOr((unsigned long long*)&g->panic, (unsigned long long)code);
}

__host__ __device__ static inline bool tb_id_reserved(u64 lo, u64 hi) {
    return (lo | hi) == 0 || (lo & hi) == ~0ULL;  // 0 or maxInt: never a live id
}

// ---- accounts -----------------------------------------------------------------------------------
__device__ static inline u32 tb_account_find(const Tables& T, u64 lo, u64 hi) {
    if (tb_id_reserved(lo, hi)) return TB_NOT_FOUND;
    u64 pos = tb_hash_id(lo, hi) & T.account_mask;
    for (u64 n = 0; n <= T.account_mask; n++) {
        const AccountHot* h = &T.acct_hot[pos];
        const u64 a = h->id_lo, b = h->id_hi;
        if (a == lo && b == hi) return (u32)pos;
        if ((a | b) == 0) return TB_NOT_FOUND;
        pos = (pos + 1) & T.account_mask;
    }
    return TB_NOT_FOUND;
}

// Continue an account probe whose first entry (at `pos`) was already loaded; *hit = the matching
// entry (no second load of it).
__device__ static inline u32 tb_account_find_from(const Tables& T, u64 lo, u64 hi, u64 pos, const AccountHot& first,
                                                  AccountHot* hit) {
    if (first.id_lo == lo && first.id_hi == hi) {
        *hit = first;
        return (u32)pos;
    }
    if ((first.id_lo | first.id_hi) == 0 || tb_id_reserved(lo, hi)) return TB_NOT_FOUND;
    pos = (pos + 1) & T.account_mask;
    for (u64 n = 1; n <= T.account_mask; n++) {
        const AccountHot h = T.acct_hot[pos];
        if (h.id_lo == lo && h.id_hi == hi) {
            *hit = h;
            return (u32)pos;
        }
        if ((h.id_lo | h.id_hi) == 0) return TB_NOT_FOUND;
        pos = (pos + 1) & T.account_mask;
    }
    return TB_NOT_FOUND;
}

// Both accounts of a transfer at once (kernel 1).  Their first entries were loaded together; the
// two chains then advance together — a wave waits for the longer chain, not for the sum of both —
// two entries per account per round, reading only the 16-B ids (one 32-B span); a hit found in the
// chain has its full entry read once at the end (its line was just fetched).  At load 1/2 the
// longest of 128 chains in a wave is ~8 entries: ~4 rounds instead of ~2 x 8.
__device__ static inline void tb_account_find2(const Tables& T, u64 dlo, u64 dhi, u64 dpos, const AccountHot& d0,
                                               u64 clo, u64 chi, u64 cpos, const AccountHot& c0, u32* drs, u32* crs,
                                               AccountHot* dh, AccountHot* ch) {
    const u64 mask = T.account_mask;
    u32 ds = TB_NOT_FOUND, cs = TB_NOT_FOUND;
    bool dgo = false, cgo = false, dlate = false, clate = false;
    if (d0.id_lo == dlo && d0.id_hi == dhi) {
        ds = (u32)dpos;
        *dh = d0;
    } else {
        dgo = (d0.id_lo | d0.id_hi) != 0;
    }
    if (c0.id_lo == clo && c0.id_hi == chi) {
        cs = (u32)cpos;
        *ch = c0;
    } else {
        cgo = (c0.id_lo | c0.id_hi) != 0;
    }
    u64 dp = (dpos + 1) & mask, cp = (cpos + 1) & mask;
    for (u64 n = 0; (dgo || cgo) && n <= mask; n += 2) {
        ulonglong2 da = {0, 0}, db = {0, 0}, ca = {0, 0}, cb = {0, 0};
        const u64 dq = (dp + 1) & mask, cq = (cp + 1) & mask;
        if (dgo) {
            da = *(const ulonglong2*)&T.acct_hot[dp];
            db = *(const ulonglong2*)&T.acct_hot[dq];
        }
        if (cgo) {
            ca = *(const ulonglong2*)&T.acct_hot[cp];
            cb = *(const ulonglong2*)&T.acct_hot[cq];
        }
        if (dgo) {
            if (da.x == dlo && da.y == dhi) {
                ds = (u32)dp;
                dgo = false;
                dlate = true;
            } else if ((da.x | da.y) == 0) {
                dgo = false;
            } else if (db.x == dlo && db.y == dhi) {
                ds = (u32)dq;
                dgo = false;
                dlate = true;
            } else if ((db.x | db.y) == 0) {
                dgo = false;
            }
            dp = (dp + 2) & mask;
        }
        if (cgo) {
            if (ca.x == clo && ca.y == chi) {
                cs = (u32)cp;
                cgo = false;
                clate = true;
            } else if ((ca.x | ca.y) == 0) {
                cgo = false;
            } else if (cb.x == clo && cb.y == chi) {
                cs = (u32)cq;
                cgo = false;
                clate = true;
            } else if ((cb.x | cb.y) == 0) {
                cgo = false;
            }
            cp = (cp + 2) & mask;
        }
    }
    if (dlate) *dh = T.acct_hot[ds];
    if (clate) *ch = T.acct_hot[cs];
    *drs = ds;
    *crs = cs;
}

__device__ static inline u32 tb_account_claim(const Tables& T, u64 lo, u64 hi, u64 ts) {
    u64 pos = tb_hash_id(lo, hi) & T.account_mask;
    for (u64 n = 0; n <= T.account_mask; n++) {
        u64* w = &T.acct_hot[pos].timestamp;
        if (*(volatile u64*)w == 0 &&
            atomicCAS((unsigned long long*)w, 0ULL, (unsigned long long)ts) == 0ULL) {
            return (u32)pos;
        }
        pos = (pos + 1) & T.account_mask;
    }
    tb_panic(T.g, PANIC_TABLE_FULL);
    return TB_NOT_FOUND;
}

__device__ static inline void tb_account_tombstone(const Tables& T, u32 slot) {
    T.acct_hot[slot].id_lo = ~0ULL;
    T.acct_hot[slot].id_hi = ~0ULL;
}

__device__ static inline AccountBal tb_bal_load(const BalView& V, u64 slot) {
    const u64* l = V.lo + 4 * slot;
    const u64* h = V.hi + 4 * slot;
    AccountBal b;
    b.debits_pending = tb_u128(l[0], h[0]);
    b.debits_posted = tb_u128(l[1], h[1]);
    b.credits_pending = tb_u128(l[2], h[2]);
    b.credits_posted = tb_u128(l[3], h[3]);
    return b;
}

__device__ static inline void tb_bal_store(const BalView& V, u64 slot, const AccountBal& b) {
    u64* l = V.lo + 4 * slot;
    u64* h = V.hi + 4 * slot;
    l[0] = tb_lo(b.debits_pending);
    l[1] = tb_lo(b.debits_posted);
    l[2] = tb_lo(b.credits_pending);
    l[3] = tb_lo(b.credits_posted);
    h[0] = tb_hi(b.debits_pending);
    h[1] = tb_hi(b.debits_posted);
    h[2] = tb_hi(b.credits_pending);
    h[3] = tb_hi(b.credits_posted);
}

// Balance f (BAL_*) of a slot as one u128.
__device__ static inline u128 tb_bal_get(const BalView& V, u64 slot, u32 f) {
    return tb_u128(V.lo[4 * slot + f], V.hi[4 * slot + f]);
}

__device__ static inline Account tb_account_load(const Tables& T, u32 slot) {
    const AccountHot h = T.acct_hot[slot];
    const AccountBal b = tb_bal_load(T.bal, slot);
    const AccountCold c = T.acct_cold[slot];
    Account a;
    a.id = tb_u128(h.id_lo, h.id_hi);
    a.debits_pending = b.debits_pending;
    a.debits_posted = b.debits_posted;
    a.credits_pending = b.credits_pending;
    a.credits_posted = b.credits_posted;
    a.user_data_128 = c.user_data_128;
    a.user_data_64 = c.user_data_64;
    a.user_data_32 = c.user_data_32;
    a.reserved = c.reserved;
    a.ledger = h.ledger;
    a.code = h.code;
    a.flags = h.flags;
    a.timestamp = h.timestamp;
    return a;
}

// Write every field of a claimed slot (the timestamp word was set by the claim).
__device__ static inline void tb_account_store_new(const Tables& T, u32 slot, const Account& a) {
    AccountCold c;
    c.user_data_128 = a.user_data_128;
    c.user_data_64 = a.user_data_64;
    c.user_data_32 = a.user_data_32;
    c.reserved = a.reserved;
    T.acct_cold[slot] = c;
    AccountBal b;
    b.debits_pending = a.debits_pending;
    b.debits_posted = a.debits_posted;
    b.credits_pending = a.credits_pending;
    b.credits_posted = a.credits_posted;
    tb_bal_store(T.bal, slot, b);
    if (a.flags & AF_LIMITS) atomicAdd((unsigned long long*)&T.g->limit_accounts, 1ULL);
    AccountHot* h = &T.acct_hot[slot];
    h->ledger = a.ledger;
    h->code = a.code;
    h->flags = a.flags;
    h->id_lo = tb_lo(a.id);
    h->id_hi = tb_hi(a.id);
}

// ---- transfers ----------------------------------------------------------------------------------
__host__ __device__ static inline u64 tb_fingerprint(u64 lo, u64 hi) {
    const u64 f = tb_mix64(hi ^ tb_mix64(lo ^ 0x6a09e667f3bcc909ULL));
    return f ? f : 1;
}

__host__ __device__ static inline u64 tb_fp32(u64 lo, u64 hi) { return (tb_fingerprint(lo, hi) >> 32) | 1; }
__device__ static inline u32 tb_xi_pos(u64 e) { return (u32)((e & XI_POS_MASK) - 1); }

// Find a live transfer; returns its log position or TB_NOT_FOUND.
__device__ static inline u32 tb_transfer_find(const Tables& T, u64 lo, u64 hi) {
    if (tb_id_reserved(lo, hi)) return TB_NOT_FOUND;
    const u64 fp = tb_fp32(lo, hi);
    u64 pos = tb_hash_id(lo, hi) & T.xidx_mask;
    for (u64 n = 0; n <= T.xidx_mask; n++) {
        const u64 e = T.xidx[pos];
        if (e == 0) return TB_NOT_FOUND;
        if ((e >> 32) == fp && !(e & XI_TOMB)) {
            const u32 lp = tb_xi_pos(e);
            const u64* idw = (const u64*)&T.xlog[lp];
            if (idw[0] == lo && idw[1] == hi) return lp;
        }
        pos = (pos + 1) & T.xidx_mask;
    }
    return TB_NOT_FOUND;
}

enum : u32 { CLAIM_NEW = 0, CLAIM_EXISTS = 1, CLAIM_COLLIDED = 2, CLAIM_FULL = 3 };

// Find-or-claim for `id` at log position `log_pos`.
//  CLAIM_EXISTS:   a live record from an earlier pass has this id (*found = its log position)
//  CLAIM_COLLIDED: another event of this pass (log position >= pass_base) holds the same
//                  fingerprint — both events become dependent (xdup[] marks the holder's entry;
//                  kernel 2 reads it)
//  CLAIM_NEW:      entry claimed (*entry = index position); the caller writes the record
// `first` is the value the caller's home-entry CAS (tb_transfer_cas_home) returned, else ~0.
__device__ static inline u32 tb_transfer_claim(const Tables& T, u64 lo, u64 hi, u32 log_pos, u64 pass_base,
                                               u32* found, u32* entry, u64 first = ~0ULL) {
    const u64 fp = tb_fp32(lo, hi);
    const u64 mine = (fp << 32) | ((u64)log_pos + 1);
    const u64 mask = T.xidx_mask;
    u64 pos = tb_hash_id(lo, hi) & mask;
    // One entry: claim it if empty, else decide on its fingerprint.  Returns CLAIM_FULL to go on.
    auto step = [&](u64 p, u64 cur) -> u32 {
        if (cur == 0) {
            cur = atomicCAS((unsigned long long*)&T.xidx[p], 0ULL, (unsigned long long)mine);
            if (cur == 0) {
                *entry = (u32)p;
                return CLAIM_NEW;
            }
        }
        if ((cur >> 32) == fp && !(cur & XI_TOMB)) {
            const u32 lp = tb_xi_pos(cur);
            if ((u64)lp >= pass_base) {
                T.xdup[p] = 1;
                return CLAIM_COLLIDED;
            }
            const u64* idw = (const u64*)&T.xlog[lp];
            if (idw[0] == lo && idw[1] == hi) {
                *found = lp;
                return CLAIM_EXISTS;
            }
        }
        return CLAIM_FULL;
    };
    u64 n = 0;
    if (first != ~0ULL) {  // the caller's home CAS returned `first`
        if (first == 0) {
            *entry = (u32)pos;
            return CLAIM_NEW;
        }
        const u32 r = step(pos, first);
        if (r != CLAIM_FULL) return r;
        pos = (pos + 1) & mask;
        n = 1;
    }
    // The chain, two entries per read round (entries never return to empty, so a value read before
    // the first one's CAS is still a valid lower bound for the second).
    for (; n <= mask; n += 2) {
        const u64 q = (pos + 1) & mask;
        const u64 e0 = *(volatile u64*)&T.xidx[pos];
        const u64 e1 = *(volatile u64*)&T.xidx[q];
        u32 r = step(pos, e0);
        if (r != CLAIM_FULL) return r;
        r = step(q, e1);
        if (r != CLAIM_FULL) return r;
        pos = (q + 1) & mask;
    }
    tb_panic(T.g, PANIC_TABLE_FULL);
    return CLAIM_FULL;
}

// Speculative claim of the home entry, issued before the event's account checks: for a new id
// (the common case) the whole claim is one memory-side atomic, with no probe read in front of it.
// Returns the entry's previous value (0: claimed).  A claim whose event then fails is withdrawn by
// the resolve kernel like any other failed speculative insert.
__device__ static inline u64 tb_transfer_cas_home(const Tables& T, u64 lo, u64 hi, u32 log_pos, u64 xpos) {
    const u64 mine = (tb_fp32(lo, hi) << 32) | ((u64)log_pos + 1);
    return atomicCAS((unsigned long long*)&T.xidx[xpos], 0ULL, (unsigned long long)mine);
}

// Claim the first empty entry for an id known to be absent (the ordered replay).
__device__ static inline u32 tb_transfer_claim_new(const Tables& T, u64 lo, u64 hi, u32 log_pos) {
    const u64 mine = (tb_fp32(lo, hi) << 32) | ((u64)log_pos + 1);
    u64 pos = tb_hash_id(lo, hi) & T.xidx_mask;
    for (u64 n = 0; n <= T.xidx_mask; n++) {
        u64* e = &T.xidx[pos];
        if (*e == 0 && atomicCAS((unsigned long long*)e, 0ULL, (unsigned long long)mine) == 0ULL) return (u32)pos;
        pos = (pos + 1) & T.xidx_mask;
    }
    tb_panic(T.g, PANIC_TABLE_FULL);
    return TB_NOT_FOUND;
}

// Did any event of the current pass (log positions >= pass_base) claim this id — whether its
// entry is live or withdrawn (tombstoned)?  Fingerprint-level, so conservative.
__device__ static inline bool tb_transfer_claimed_in_pass(const Tables& T, u64 lo, u64 hi, u64 pass_base) {
    if (tb_id_reserved(lo, hi)) return false;
    const u64 fp = tb_fp32(lo, hi);
    u64 pos = tb_hash_id(lo, hi) & T.xidx_mask;
    for (u64 n = 0; n <= T.xidx_mask; n++) {
        const u64 e = T.xidx[pos];
        if (e == 0) return false;
        if ((e >> 32) == fp && (u64)tb_xi_pos(e) >= pass_base) return true;
        pos = (pos + 1) & T.xidx_mask;
    }
    return true;
}

__device__ static inline void tb_xindex_tombstone(const Tables& T, u32 entry) {
    atomicOr((unsigned long long*)&T.xidx[entry], (unsigned long long)XI_TOMB);
}

// In-place u128 atomic add (mod 2^128) on a balance field: exact for any interleaving because
// every adder carries its own low-word carry into the high word.
__device__ static inline void tb_atomic_add_u128(void* field, u128 v) {
    unsigned long long* w = (unsigned long long*)field;
    const u64 lo = tb_lo(v), hi = tb_hi(v);
    u64 carry = 0;
    if (lo != 0) {
        const u64 old = atomicAdd(&w[0], (unsigned long long)lo);
        carry = (old + lo) < old ? 1 : 0;
    }
    if (hi + carry != 0) atomicAdd(&w[1], (unsigned long long)(hi + carry));
}

// Fire-and-forget add to the low word only: valid when no low word can carry this pass (the
// 64-bit certificate: bound + S < 2^64, so every balance stays below 2^64).
__device__ static inline void tb_atomic_add_lo_noret(void* field, u64 v) {
    __hip_atomic_fetch_add((unsigned long long*)field, (unsigned long long)v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Exact u128 add to balance f of a slot (mod 2^128): the low word, then the carry into the high.
__device__ static inline void tb_bal_add(const BalView& V, u64 slot, u32 f, u128 v) {
    const u64 lo = tb_lo(v), hi = tb_hi(v);
    u64 carry = 0;
    if (lo != 0) {
        const u64 old = atomicAdd((unsigned long long*)&V.lo[4 * slot + f], (unsigned long long)lo);
        carry = (old + lo) < old ? 1 : 0;
    }
    if (hi + carry != 0) atomicAdd((unsigned long long*)&V.hi[4 * slot + f], (unsigned long long)(hi + carry));
}

// Low-word add to balance f of a slot (the certificate's no-carry case).
__device__ static inline void tb_bal_add_lo(const BalView& V, u64 slot, u32 f, u64 v) {
    tb_atomic_add_lo_noret(&V.lo[4 * slot + f], v);
}

// ------------------------------------------------------------------------------------------------
// Per-pass dedup set of 63-bit id fingerprints: collisions between the ids / pending ids of two
// events of one pass mark both events dependent (ordered fallback).  0 = empty, bit 63 = DUP.
// A fingerprint collision of two different ids only costs a spurious fallback, never a wrong
// result.
// ------------------------------------------------------------------------------------------------
#define DEDUP_DUP (1ULL << 63)

__device__ static inline u64 tb_dedup_key(u64 lo, u64 hi) {
    const u64 h = tb_hash_id(lo ^ 0x5bd1e9955bd1e995ULL, hi);
    return (h >> 1) | 1;  // nonzero, bit 63 clear
}

// Returns true when the key was already present (a collision: both events become dependent).
__device__ static inline bool tb_dedup_insert(u64* table, u64 mask, u64 key) {
    u64 pos = tb_mix64(key) & mask;
    for (u64 n = 0; n <= mask; n++) {
        u64 cur = *(volatile u64*)&table[pos];
        if (cur == 0) {
            cur = atomicCAS((unsigned long long*)&table[pos], 0ULL, (unsigned long long)key);
            if (cur == 0) return false;
        }
        if ((cur & ~DEDUP_DUP) == key) {
            if (!(cur & DEDUP_DUP)) atomicOr((unsigned long long*)&table[pos], (unsigned long long)DEDUP_DUP);
            return true;
        }
        pos = (pos + 1) & mask;
    }
    return true;
}

// True when `key` is in the set (inserted by anyone).
__device__ static inline bool tb_dedup_is_dup_or_present(const u64* table, u64 mask, u64 key) {
    u64 pos = tb_mix64(key) & mask;
    for (u64 n = 0; n <= mask; n++) {
        const u64 cur = table[pos];
        if (cur == 0) return false;
        if ((cur & ~DEDUP_DUP) == key) return true;
        pos = (pos + 1) & mask;
    }
    return true;
}

__device__ static inline bool tb_dedup_is_dup(const u64* table, u64 mask, u64 key) {
    u64 pos = tb_mix64(key) & mask;
    for (u64 n = 0; n <= mask; n++) {
        const u64 cur = table[pos];
        if (cur == 0) return false;  // (unreachable for an inserted key)
        if ((cur & ~DEDUP_DUP) == key) return (cur & DEDUP_DUP) != 0;
        pos = (pos + 1) & mask;
    }
    return true;
}
