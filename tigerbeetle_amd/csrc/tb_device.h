// tb_device.h — records, result codes and HBM tables of the MI355X commit engine.
//
// Layouts follow src/tigerbeetle.zig:7-104 (Account / Transfer extern structs, 128 B, align 16);
// result codes follow src/tigerbeetle.zig:109-229 (values == declaration index).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
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

// Byte offsets used by the in-place balance atomics.
#define ACCOUNT_OFF_DEBITS_PENDING 16
#define ACCOUNT_OFF_DEBITS_POSTED 32
#define ACCOUNT_OFF_CREDITS_PENDING 48
#define ACCOUNT_OFF_CREDITS_POSTED 64

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
// Both object tables are open-addressing hash tables whose slots ARE the 128-byte records
// (record-in-table): a hit costs one HBM line, and a transfer probe reads only the first 64-byte
// sector (the id).
//   * empty slot:  id == 0 (ids are never 0 for live objects: id_must_not_be_zero)
//   * live slot:   id != 0, id != maxInt; timestamp != 0
//   * tombstone:   id == maxInt(u128) (never a live id: id_must_not_be_int_max) — a rolled-back or
//                  withdrawn insert; probes continue past it, it is never reclaimed
// Inserts claim an empty slot with a 64-bit CAS of the timestamp word (0 -> ts) and then write the
// record; a slot claimed in the current kernel may still read id == 0 to a concurrent prober, which
// can only be a prober of an id that is absent from the pre-kernel table (a claimed slot was empty,
// so it never lies on the probe path of an older key) — every such pair of events collides in the
// pass dedup set and is resolved by the ordered replay.
// ------------------------------------------------------------------------------------------------
struct Globals {
    u64 commit_timestamp;     // max timestamp of an event that returned ok when evaluated
    u64 panic;                // PANIC_* bits
    u64 sum_lo, sum_hi;       // (unused)
    u64 bound_lo, bound_hi;   // upper bound of dp+dpost and cp+cpost over every account
    u64 dependent_total;      // dependent events of this pass
    u64 dependent_all;        // cumulative
    u64 account_count;
    u64 transfer_count;
    u64 export_count;
    u64 pad[5];
};

struct Tables {
    Account* accounts;        // [account_cap]
    u32* account_mark;        // [account_cap] pass epoch of the last balancing mark
    u64 account_mask;         // account_cap - 1
    Transfer* transfers;      // [transfer_cap]
    u8* posted;               // [transfer_cap] POSTED_* of the pending transfer in that slot
    u64 transfer_mask;
    Globals* g;
};

__device__ static inline void tb_panic(Globals* g, u32 code) {
    atomicOr((unsigned long long*)&g->panic, (unsigned long long)code);
}

// Probe a record-in-table for a live id.  Returns the slot or TB_NOT_FOUND.
template <typename R>
__device__ static inline u32 tb_find(const R* table, u64 mask, u64 lo, u64 hi) {
    // 0 marks an empty slot and maxInt a tombstone: neither is ever a live id.
    if ((lo | hi) == 0 || (lo & hi) == ~0ULL) return TB_NOT_FOUND;
    u64 pos = tb_hash_id(lo, hi) & mask;
    for (u64 n = 0; n <= mask; n++) {
        const u64* idw = (const u64*)&table[pos];
        const u64 a = idw[0], b = idw[1];
        if (a == lo && b == hi) return (u32)pos;
        if ((a | b) == 0) return TB_NOT_FOUND;
        pos = (pos + 1) & mask;
    }
    return TB_NOT_FOUND;
}

__device__ static inline u32 tb_account_find(const Tables& T, u64 lo, u64 hi) {
    return tb_find(T.accounts, T.account_mask, lo, hi);
}

__device__ static inline u32 tb_transfer_find(const Tables& T, u64 lo, u64 hi) {
    return tb_find(T.transfers, T.transfer_mask, lo, hi);
}

// Tombstone a slot (id = maxInt), keeping its timestamp so it is never reclaimed.
template <typename R>
__device__ static inline void tb_tombstone(R* rec) {
    u64* w = (u64*)rec;
    w[0] = ~0ULL;
    w[1] = ~0ULL;
}

// Claim an empty slot for a key that is known to be absent; CAS the timestamp word 0 -> ts.
__device__ static inline u32 tb_claim_slot(u64* ts_word0, size_t stride_words, u64 mask, u64 hash, u64 ts,
                                           Globals* g) {
    u64 pos = hash & mask;
    for (u64 n = 0; n <= mask; n++) {
        u64* w = ts_word0 + pos * stride_words;
        if (*(volatile u64*)w == 0) {
            if (atomicCAS((unsigned long long*)w, 0ULL, (unsigned long long)ts) == 0ULL) return (u32)pos;
        }
        pos = (pos + 1) & mask;
    }
    tb_panic(g, PANIC_TABLE_FULL);
    return TB_NOT_FOUND;
}

__device__ static inline u32 tb_account_claim(const Tables& T, u64 lo, u64 hi, u64 ts) {
    return tb_claim_slot((u64*)&T.accounts[0].timestamp, sizeof(Account) / 8, T.account_mask,
                         tb_hash_id(lo, hi), ts, T.g);
}

__device__ static inline u32 tb_transfer_claim(const Tables& T, u64 lo, u64 hi, u64 ts) {
    return tb_claim_slot((u64*)&T.transfers[0].timestamp, sizeof(Transfer) / 8, T.transfer_mask,
                         tb_hash_id(lo, hi), ts, T.g);
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
