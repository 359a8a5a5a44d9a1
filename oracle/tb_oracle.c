/*
 * tb_oracle.c — TEST INFRASTRUCTURE ONLY (see tb_oracle.h).
 *
 * A single-threaded, in-memory restatement of the reference StateMachine commit path.
 * "Grooves" are open-addressing hash maps with an undo log for linked-chain scopes.
 * Every function cites the reference lines it restates.
 */
#include "tb_oracle.h"

#include <setjmp.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define U128_MAX (~(u128)0)

/* src/tigerbeetle.zig:7-29 */
typedef struct {
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
} account_t;

/* src/tigerbeetle.zig:64-89 */
typedef struct {
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
} transfer_t;

_Static_assert(sizeof(account_t) == 128, "Account is 128 bytes");
_Static_assert(sizeof(transfer_t) == 128, "Transfer is 128 bytes");

/* AccountFlags (tigerbeetle.zig:42-62). */
enum { AF_LINKED = 1, AF_DEBITS_MUST_NOT_EXCEED_CREDITS = 2, AF_CREDITS_MUST_NOT_EXCEED_DEBITS = 4,
       AF_PADDING = 0xFFF8 };
/* TransferFlags (tigerbeetle.zig:91-104). */
enum { TF_LINKED = 1, TF_PENDING = 2, TF_POST = 4, TF_VOID = 8, TF_BAL_DEBIT = 16,
       TF_BAL_CREDIT = 32, TF_PADDING = 0xFFC0 };

/* Operation (state_machine.zig:208-214, vsr_operations_reserved = 128). */
enum { OP_CREATE_ACCOUNTS = 128, OP_CREATE_TRANSFERS = 129, OP_LOOKUP_ACCOUNTS = 130,
       OP_LOOKUP_TRANSFERS = 131 };

/* CreateAccountResult (tigerbeetle.zig:109-143). */
enum {
    CA_OK = 0, CA_LINKED_EVENT_FAILED = 1, CA_LINKED_EVENT_CHAIN_OPEN = 2,
    CA_TIMESTAMP_MUST_BE_ZERO = 3, CA_RESERVED_FIELD = 4, CA_RESERVED_FLAG = 5,
    CA_ID_MUST_NOT_BE_ZERO = 6, CA_ID_MUST_NOT_BE_INT_MAX = 7, CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 8,
    CA_DEBITS_PENDING_MUST_BE_ZERO = 9, CA_DEBITS_POSTED_MUST_BE_ZERO = 10,
    CA_CREDITS_PENDING_MUST_BE_ZERO = 11, CA_CREDITS_POSTED_MUST_BE_ZERO = 12,
    CA_LEDGER_MUST_NOT_BE_ZERO = 13, CA_CODE_MUST_NOT_BE_ZERO = 14,
    CA_EXISTS_WITH_DIFFERENT_FLAGS = 15, CA_EXISTS_WITH_DIFFERENT_USER_DATA_128 = 16,
    CA_EXISTS_WITH_DIFFERENT_USER_DATA_64 = 17, CA_EXISTS_WITH_DIFFERENT_USER_DATA_32 = 18,
    CA_EXISTS_WITH_DIFFERENT_LEDGER = 19, CA_EXISTS_WITH_DIFFERENT_CODE = 20, CA_EXISTS = 21,
};

/* CreateTransferResult (tigerbeetle.zig:145-229). */
enum {
    CT_OK = 0, CT_LINKED_EVENT_FAILED = 1, CT_LINKED_EVENT_CHAIN_OPEN = 2,
    CT_TIMESTAMP_MUST_BE_ZERO = 3, CT_RESERVED_FLAG = 4, CT_ID_MUST_NOT_BE_ZERO = 5,
    CT_ID_MUST_NOT_BE_INT_MAX = 6, CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE = 7,
    CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 8, CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 9,
    CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO = 10, CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX = 11,
    CT_ACCOUNTS_MUST_BE_DIFFERENT = 12, CT_PENDING_ID_MUST_BE_ZERO = 13,
    CT_PENDING_ID_MUST_NOT_BE_ZERO = 14, CT_PENDING_ID_MUST_NOT_BE_INT_MAX = 15,
    CT_PENDING_ID_MUST_BE_DIFFERENT = 16, CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17,
    CT_AMOUNT_MUST_NOT_BE_ZERO = 18, CT_LEDGER_MUST_NOT_BE_ZERO = 19, CT_CODE_MUST_NOT_BE_ZERO = 20,
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

/* ------------------------------------------------------------------------------------------ */
/* Open-addressing maps with tombstones.                                                      */
/* ------------------------------------------------------------------------------------------ */

enum { SLOT_EMPTY = 0, SLOT_FULL = 1, SLOT_TOMB = 2 };

typedef struct {
    u128 key;
    u64 value;
    u8 state;
} map_slot;

typedef struct {
    map_slot* slots;
    u64 cap;   /* power of two */
    u64 used;  /* FULL + TOMB */
    u64 count; /* FULL */
} map_t;

static u64 mix64(u64 x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

static u64 hash128(u128 k) { return mix64((u64)k ^ mix64((u64)(k >> 64) + 0x9e3779b97f4a7c15ULL)); }

static void map_init(map_t* m, u64 cap) {
    u64 c = 64;
    while (c < cap) c <<= 1;
    m->slots = (map_slot*)calloc(c, sizeof(map_slot));
    m->cap = c;
    m->used = 0;
    m->count = 0;
}

static void map_free(map_t* m) {
    free(m->slots);
    memset(m, 0, sizeof(*m));
}

static void map_put(map_t* m, u128 key, u64 value);

static void map_grow(map_t* m) {
    map_t n;
    map_init(&n, m->count * 4 > m->cap ? m->cap * 2 : m->cap);
    for (u64 i = 0; i < m->cap; i++) {
        if (m->slots[i].state == SLOT_FULL) map_put(&n, m->slots[i].key, m->slots[i].value);
    }
    free(m->slots);
    *m = n;
}

/* Returns the FULL slot holding key, or NULL. */
static map_slot* map_find(const map_t* m, u128 key) {
    u64 mask = m->cap - 1;
    for (u64 i = hash128(key) & mask;; i = (i + 1) & mask) {
        map_slot* s = &m->slots[i];
        if (s->state == SLOT_EMPTY) return NULL;
        if (s->state == SLOT_FULL && s->key == key) return s;
    }
}

static void map_put(map_t* m, u128 key, u64 value) {
    map_slot* found = map_find(m, key);
    if (found) {
        found->value = value;
        return;
    }
    if ((m->used + 1) * 2 > m->cap) {
        map_grow(m);
    }
    u64 mask = m->cap - 1;
    for (u64 i = hash128(key) & mask;; i = (i + 1) & mask) {
        map_slot* s = &m->slots[i];
        if (s->state != SLOT_FULL) {
            if (s->state == SLOT_EMPTY) m->used++;
            s->key = key;
            s->value = value;
            s->state = SLOT_FULL;
            m->count++;
            return;
        }
    }
}

static void map_remove(map_t* m, u128 key) {
    map_slot* s = map_find(m, key);
    if (s) {
        s->state = SLOT_TOMB;
        m->count--;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* State: three "grooves" (state_machine.zig:103-206) and the scope undo log.                 */
/* ------------------------------------------------------------------------------------------ */

typedef enum { UNDO_ACCOUNT_INSERT, UNDO_ACCOUNT_UPDATE, UNDO_TRANSFER_INSERT, UNDO_POSTED_INSERT } undo_kind;

typedef struct {
    undo_kind kind;
    u64 index;        /* record index, or posted key */
    account_t before; /* UNDO_ACCOUNT_UPDATE */
} undo_entry;

struct tbo_state {
    u64 prepare_timestamp_unused;
    u64 commit_timestamp;

    account_t* accounts;
    u64 accounts_len, accounts_cap;
    map_t account_ids; /* id -> index into accounts */

    transfer_t* transfers;
    u64 transfers_len, transfers_cap;
    map_t transfer_ids; /* id -> index into transfers */

    map_t posted; /* pending timestamp -> fulfillment (0 posted, 1 voided) (state_machine.zig:185-198) */

    int scope_open;
    undo_entry* undo;
    u64 undo_len, undo_cap;

    jmp_buf panic_jmp;
};

static void panic(tbo_state* s) { longjmp(s->panic_jmp, 1); }

/* Zig checked `+` (ReleaseSafe traps on overflow). */
static u128 add_checked(tbo_state* s, u128 a, u128 b) {
    u128 r;
    if (__builtin_add_overflow(a, b, &r)) panic(s);
    return r;
}

static u128 sub_checked(tbo_state* s, u128 a, u128 b) {
    if (b > a) panic(s);
    return a - b;
}

/* sum_overflows (state_machine.zig:1152-1157). */
static int sum_overflows_u128(u128 a, u128 b) {
    u128 r;
    return __builtin_add_overflow(a, b, &r);
}

static int sum_overflows_u64(u64 a, u64 b) {
    u64 r;
    return __builtin_add_overflow(a, b, &r);
}

static void undo_push(tbo_state* s, undo_entry e) {
    if (!s->scope_open) return;
    if (s->undo_len == s->undo_cap) {
        s->undo_cap = s->undo_cap ? s->undo_cap * 2 : 64;
        s->undo = (undo_entry*)realloc(s->undo, s->undo_cap * sizeof(undo_entry));
    }
    s->undo[s->undo_len++] = e;
}

static const account_t* accounts_get(const tbo_state* s, u128 id) {
    map_slot* m = map_find(&s->account_ids, id);
    return m ? &s->accounts[m->value] : NULL;
}

/* groove.insert (lsm/groove.zig:902-921): asserts absence. */
static void accounts_insert(tbo_state* s, const account_t* a) {
    if (map_find(&s->account_ids, a->id)) panic(s);
    if (s->accounts_len == s->accounts_cap) {
        s->accounts_cap = s->accounts_cap ? s->accounts_cap * 2 : 1024;
        s->accounts = (account_t*)realloc(s->accounts, s->accounts_cap * sizeof(account_t));
    }
    s->accounts[s->accounts_len] = *a;
    map_put(&s->account_ids, a->id, s->accounts_len);
    undo_entry e = {UNDO_ACCOUNT_INSERT, s->accounts_len, {0}};
    undo_push(s, e);
    s->accounts_len++;
}

/* groove.upsert (lsm/groove.zig:925-963) for an existing object. */
static void accounts_upsert(tbo_state* s, const account_t* a) {
    map_slot* m = map_find(&s->account_ids, a->id);
    if (!m) panic(s);
    account_t* cur = &s->accounts[m->value];
    if (cur->timestamp != a->timestamp) panic(s); /* groove.zig:932 */
    undo_entry e = {UNDO_ACCOUNT_UPDATE, m->value, *cur};
    undo_push(s, e);
    *cur = *a;
}

static const transfer_t* transfers_get(const tbo_state* s, u128 id) {
    map_slot* m = map_find(&s->transfer_ids, id);
    return m ? &s->transfers[m->value] : NULL;
}

static void transfers_insert(tbo_state* s, const transfer_t* t) {
    if (map_find(&s->transfer_ids, t->id)) panic(s);
    if (s->transfers_len == s->transfers_cap) {
        s->transfers_cap = s->transfers_cap ? s->transfers_cap * 2 : 1024;
        s->transfers = (transfer_t*)realloc(s->transfers, s->transfers_cap * sizeof(transfer_t));
    }
    s->transfers[s->transfers_len] = *t;
    map_put(&s->transfer_ids, t->id, s->transfers_len);
    undo_entry e = {UNDO_TRANSFER_INSERT, s->transfers_len, {0}};
    undo_push(s, e);
    s->transfers_len++;
}

/* get_posted (state_machine.zig:1084-1089): returns 0 if absent, 1 posted, 2 voided. */
static int posted_get(const tbo_state* s, u64 pending_timestamp) {
    map_slot* m = map_find(&s->posted, pending_timestamp);
    return m ? (int)m->value + 1 : 0;
}

static void posted_insert(tbo_state* s, u64 pending_timestamp, u64 fulfillment) {
    if (map_find(&s->posted, pending_timestamp)) panic(s);
    map_put(&s->posted, pending_timestamp, fulfillment);
    undo_entry e = {UNDO_POSTED_INSERT, pending_timestamp, {0}};
    undo_push(s, e);
}

/* scope_open / scope_close (state_machine.zig:584-610, cache_map.zig:266-309). */
static void scope_open(tbo_state* s) {
    if (s->scope_open) panic(s);
    s->scope_open = 1;
    s->undo_len = 0;
}

static void scope_close(tbo_state* s, int persist) {
    if (!s->scope_open) panic(s);
    if (!persist) {
        /* Replay the undo log LIFO to restore exactly the pre-scope state. */
        while (s->undo_len > 0) {
            undo_entry* e = &s->undo[--s->undo_len];
            switch (e->kind) {
            case UNDO_ACCOUNT_INSERT:
                map_remove(&s->account_ids, s->accounts[e->index].id);
                s->accounts_len--; /* LIFO: the inserted record is the last one */
                break;
            case UNDO_ACCOUNT_UPDATE:
                s->accounts[e->index] = e->before;
                break;
            case UNDO_TRANSFER_INSERT:
                map_remove(&s->transfer_ids, s->transfers[e->index].id);
                s->transfers_len--;
                break;
            case UNDO_POSTED_INSERT:
                map_remove(&s->posted, (u128)e->index);
                break;
            }
        }
    }
    s->undo_len = 0;
    s->scope_open = 0;
}

/* ------------------------------------------------------------------------------------------ */
/* create_account (state_machine.zig:738-777)                                                  */
/* ------------------------------------------------------------------------------------------ */

static u32 create_account_exists(const account_t* a, const account_t* e) {
    if (a->flags != e->flags) return CA_EXISTS_WITH_DIFFERENT_FLAGS;
    if (a->user_data_128 != e->user_data_128) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a->user_data_64 != e->user_data_64) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a->user_data_32 != e->user_data_32) return CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a->ledger != e->ledger) return CA_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a->code != e->code) return CA_EXISTS_WITH_DIFFERENT_CODE;
    return CA_EXISTS;
}

static u32 create_account(tbo_state* s, const account_t* a) {
    if (!(a->timestamp > s->commit_timestamp)) panic(s);

    if (a->reserved != 0) return CA_RESERVED_FIELD;
    if (a->flags & AF_PADDING) return CA_RESERVED_FLAG;

    if (a->id == 0) return CA_ID_MUST_NOT_BE_ZERO;
    if (a->id == U128_MAX) return CA_ID_MUST_NOT_BE_INT_MAX;

    if ((a->flags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS) && (a->flags & AF_CREDITS_MUST_NOT_EXCEED_DEBITS)) {
        return CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    }

    if (a->debits_pending != 0) return CA_DEBITS_PENDING_MUST_BE_ZERO;
    if (a->debits_posted != 0) return CA_DEBITS_POSTED_MUST_BE_ZERO;
    if (a->credits_pending != 0) return CA_CREDITS_PENDING_MUST_BE_ZERO;
    if (a->credits_posted != 0) return CA_CREDITS_POSTED_MUST_BE_ZERO;
    if (a->ledger == 0) return CA_LEDGER_MUST_NOT_BE_ZERO;
    if (a->code == 0) return CA_CODE_MUST_NOT_BE_ZERO;

    const account_t* e = accounts_get(s, a->id);
    if (e) return create_account_exists(a, e);

    accounts_insert(s, a);
    s->commit_timestamp = a->timestamp;
    return CA_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* create_transfer (state_machine.zig:779-905)                                                 */
/* ------------------------------------------------------------------------------------------ */

static u32 create_transfer_exists(const transfer_t* t, const transfer_t* e) {
    if (t->flags != e->flags) return CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t->debit_account_id != e->debit_account_id) return CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (t->credit_account_id != e->credit_account_id) return CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t->amount != e->amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    if (t->user_data_128 != e->user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t->user_data_64 != e->user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t->user_data_32 != e->user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t->timeout != e->timeout) return CT_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t->code != e->code) return CT_EXISTS_WITH_DIFFERENT_CODE;
    return CT_EXISTS;
}

/* Account.debits_exceed_credits / credits_exceed_debits (tigerbeetle.zig:31-39). */
static int debits_exceed_credits(tbo_state* s, const account_t* a, u128 amount) {
    if (!(a->flags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS)) return 0;
    return add_checked(s, add_checked(s, a->debits_pending, a->debits_posted), amount) > a->credits_posted;
}

static int credits_exceed_debits(tbo_state* s, const account_t* a, u128 amount) {
    if (!(a->flags & AF_CREDITS_MUST_NOT_EXCEED_DEBITS)) return 0;
    return add_checked(s, add_checked(s, a->credits_pending, a->credits_posted), amount) > a->debits_posted;
}

static u32 post_or_void_pending_transfer_exists(const transfer_t* t, const transfer_t* e, const transfer_t* p) {
    /* state_machine.zig:1016-1077 */
    if (t->flags != e->flags) return CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (t->amount == 0) {
        if (e->amount != p->amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else {
        if (t->amount != e->amount) return CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (t->pending_id != e->pending_id) return CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (t->user_data_128 == 0) {
        if (e->user_data_128 != p->user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else {
        if (t->user_data_128 != e->user_data_128) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t->user_data_64 == 0) {
        if (e->user_data_64 != p->user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else {
        if (t->user_data_64 != e->user_data_64) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t->user_data_32 == 0) {
        if (e->user_data_32 != p->user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else {
        if (t->user_data_32 != e->user_data_32) return CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    return CT_EXISTS;
}

static u32 post_or_void_pending_transfer(tbo_state* s, const transfer_t* t) {
    /* state_machine.zig:907-1014 */
    const u16 f = t->flags;
    if ((f & TF_POST) && (f & TF_VOID)) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_PENDING) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_DEBIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & TF_BAL_CREDIT) return CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;

    if (t->pending_id == 0) return CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (t->pending_id == U128_MAX) return CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (t->pending_id == t->id) return CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t->timeout != 0) return CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    const transfer_t* p = transfers_get(s, t->pending_id);
    if (!p) return CT_PENDING_TRANSFER_NOT_FOUND;
    if (!(p->flags & TF_PENDING)) return CT_PENDING_TRANSFER_NOT_PENDING;

    const account_t* dr = accounts_get(s, p->debit_account_id);
    const account_t* cr = accounts_get(s, p->credit_account_id);
    if (!dr || !cr) panic(s); /* `.?` at :929-930 */

    if (t->debit_account_id > 0 && t->debit_account_id != p->debit_account_id) {
        return CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    }
    if (t->credit_account_id > 0 && t->credit_account_id != p->credit_account_id) {
        return CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    }
    if (t->ledger > 0 && t->ledger != p->ledger) return CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t->code > 0 && t->code != p->code) return CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;

    const u128 amount = t->amount > 0 ? t->amount : p->amount;
    if (amount > p->amount) return CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if ((f & TF_VOID) && amount < p->amount) return CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    const transfer_t* e = transfers_get(s, t->id);
    if (e) return post_or_void_pending_transfer_exists(t, e, p);

    switch (posted_get(s, p->timestamp)) {
    case 1: return CT_PENDING_TRANSFER_ALREADY_POSTED;
    case 2: return CT_PENDING_TRANSFER_ALREADY_VOIDED;
    default: break;
    }

    if (!(p->timestamp < t->timestamp)) panic(s);
    if (p->timeout > 0) {
        const u64 timeout_ns = (u64)p->timeout * 1000000000ULL;
        u64 expiry;
        if (__builtin_add_overflow(p->timestamp, timeout_ns, &expiry)) panic(s);
        if (t->timestamp >= expiry) return CT_PENDING_TRANSFER_EXPIRED;
    }

    /* Copy p before inserting: the insert may reallocate the transfer array. */
    const transfer_t pc = *p;
    const account_t dr0 = *dr;
    const account_t cr0 = *cr;

    transfer_t t2;
    memset(&t2, 0, sizeof(t2));
    t2.id = t->id;
    t2.debit_account_id = pc.debit_account_id;
    t2.credit_account_id = pc.credit_account_id;
    t2.user_data_128 = t->user_data_128 > 0 ? t->user_data_128 : pc.user_data_128;
    t2.user_data_64 = t->user_data_64 > 0 ? t->user_data_64 : pc.user_data_64;
    t2.user_data_32 = t->user_data_32 > 0 ? t->user_data_32 : pc.user_data_32;
    t2.ledger = pc.ledger;
    t2.code = pc.code;
    t2.pending_id = t->pending_id;
    t2.timeout = 0;
    t2.timestamp = t->timestamp;
    t2.flags = t->flags;
    t2.amount = amount;
    transfers_insert(s, &t2);

    posted_insert(s, pc.timestamp, (f & TF_POST) ? 0 : 1);

    account_t dr_new = dr0;
    account_t cr_new = cr0;
    dr_new.debits_pending = sub_checked(s, dr_new.debits_pending, pc.amount);
    cr_new.credits_pending = sub_checked(s, cr_new.credits_pending, pc.amount);
    if (f & TF_POST) {
        dr_new.debits_posted = add_checked(s, dr_new.debits_posted, amount);
        cr_new.credits_posted = add_checked(s, cr_new.credits_posted, amount);
    }
    accounts_upsert(s, &dr_new);
    accounts_upsert(s, &cr_new);

    s->commit_timestamp = t->timestamp;
    return CT_OK;
}

static u32 create_transfer(tbo_state* s, const transfer_t* t) {
    if (!(t->timestamp > s->commit_timestamp)) panic(s);

    if (t->flags & TF_PADDING) return CT_RESERVED_FLAG;

    if (t->id == 0) return CT_ID_MUST_NOT_BE_ZERO;
    if (t->id == U128_MAX) return CT_ID_MUST_NOT_BE_INT_MAX;

    if (t->flags & (TF_POST | TF_VOID)) return post_or_void_pending_transfer(s, t);

    if (t->debit_account_id == 0) return CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t->debit_account_id == U128_MAX) return CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t->credit_account_id == 0) return CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (t->credit_account_id == U128_MAX) return CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (t->credit_account_id == t->debit_account_id) return CT_ACCOUNTS_MUST_BE_DIFFERENT;

    if (t->pending_id != 0) return CT_PENDING_ID_MUST_BE_ZERO;
    if (!(t->flags & TF_PENDING)) {
        if (t->timeout != 0) return CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    }
    if (!(t->flags & (TF_BAL_DEBIT | TF_BAL_CREDIT))) {
        if (t->amount == 0) return CT_AMOUNT_MUST_NOT_BE_ZERO;
    }

    if (t->ledger == 0) return CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t->code == 0) return CT_CODE_MUST_NOT_BE_ZERO;

    const account_t* dr = accounts_get(s, t->debit_account_id);
    if (!dr) return CT_DEBIT_ACCOUNT_NOT_FOUND;
    const account_t* cr = accounts_get(s, t->credit_account_id);
    if (!cr) return CT_CREDIT_ACCOUNT_NOT_FOUND;
    if (!(t->timestamp > dr->timestamp) || !(t->timestamp > cr->timestamp)) panic(s);

    if (dr->ledger != cr->ledger) return CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t->ledger != dr->ledger) return CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    const transfer_t* e = transfers_get(s, t->id);
    if (e) return create_transfer_exists(t, e);

    /* :826-846 balancing amount. */
    u128 amount = t->amount;
    if (t->flags & (TF_BAL_DEBIT | TF_BAL_CREDIT)) {
        if (amount == 0) amount = (u128)UINT64_MAX; /* maxInt(u64), not u128 (:829) */
    }
    if (t->flags & TF_BAL_DEBIT) {
        const u128 dr_balance = add_checked(s, dr->debits_posted, dr->debits_pending);
        const u128 headroom = dr->credits_posted > dr_balance ? dr->credits_posted - dr_balance : 0; /* -| */
        if (headroom < amount) amount = headroom;
        if (amount == 0) return CT_EXCEEDS_CREDITS;
    }
    if (t->flags & TF_BAL_CREDIT) {
        const u128 cr_balance = add_checked(s, cr->credits_posted, cr->credits_pending);
        const u128 headroom = cr->debits_posted > cr_balance ? cr->debits_posted - cr_balance : 0;
        if (headroom < amount) amount = headroom;
        if (amount == 0) return CT_EXCEEDS_DEBITS;
    }

    if (t->flags & TF_PENDING) {
        if (sum_overflows_u128(amount, dr->debits_pending)) return CT_OVERFLOWS_DEBITS_PENDING;
        if (sum_overflows_u128(amount, cr->credits_pending)) return CT_OVERFLOWS_CREDITS_PENDING;
    }
    if (sum_overflows_u128(amount, dr->debits_posted)) return CT_OVERFLOWS_DEBITS_POSTED;
    if (sum_overflows_u128(amount, cr->credits_posted)) return CT_OVERFLOWS_CREDITS_POSTED;
    if (sum_overflows_u128(amount, add_checked(s, dr->debits_pending, dr->debits_posted))) {
        return CT_OVERFLOWS_DEBITS;
    }
    if (sum_overflows_u128(amount, add_checked(s, cr->credits_pending, cr->credits_posted))) {
        return CT_OVERFLOWS_CREDITS;
    }

    if (sum_overflows_u64(t->timestamp, (u64)t->timeout * 1000000000ULL)) return CT_OVERFLOWS_TIMEOUT;
    if (debits_exceed_credits(s, dr, amount)) return CT_EXCEEDS_CREDITS;
    if (credits_exceed_debits(s, cr, amount)) return CT_EXCEEDS_DEBITS;

    const account_t dr0 = *dr;
    const account_t cr0 = *cr;

    transfer_t t2 = *t;
    t2.amount = amount;
    transfers_insert(s, &t2);

    account_t dr_new = dr0;
    account_t cr_new = cr0;
    if (t->flags & TF_PENDING) {
        dr_new.debits_pending = add_checked(s, dr_new.debits_pending, amount);
        cr_new.credits_pending = add_checked(s, cr_new.credits_pending, amount);
    } else {
        dr_new.debits_posted = add_checked(s, dr_new.debits_posted, amount);
        cr_new.credits_posted = add_checked(s, cr_new.credits_posted, amount);
    }
    accounts_upsert(s, &dr_new);
    accounts_upsert(s, &cr_new);

    s->commit_timestamp = t->timestamp;
    return CT_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* execute (state_machine.zig:612-698)                                                         */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    u32 index;
    u32 result;
} result_t;

static u32 execute(tbo_state* s, int operation, u64 timestamp, const void* input, u32 count, result_t* results) {
    u32 n = 0;
    int in_chain = 0;
    u32 chain_start = 0;
    int chain_broken = 0;

    for (u32 index = 0; index < count; index++) {
        /* Events are copied (`var event = event_.*`). */
        account_t a;
        transfer_t t;
        u16 flags;
        u64 event_timestamp;
        if (operation == OP_CREATE_ACCOUNTS) {
            memcpy(&a, (const u8*)input + (u64)index * 128, 128);
            flags = a.flags;
            event_timestamp = a.timestamp;
        } else {
            memcpy(&t, (const u8*)input + (u64)index * 128, 128);
            flags = t.flags;
            event_timestamp = t.timestamp;
        }
        const int linked = (flags & 1) != 0; /* bit 0 is `linked` for both flag types */

        u32 result;
        if (linked && !in_chain) {
            in_chain = 1;
            chain_start = index;
            if (chain_broken) panic(s);
            scope_open(s);
        }
        if (linked && index == count - 1) {
            result = CT_LINKED_EVENT_CHAIN_OPEN; /* == CA_LINKED_EVENT_CHAIN_OPEN == 2 */
        } else if (chain_broken) {
            result = CT_LINKED_EVENT_FAILED;
        } else if (event_timestamp != 0) {
            result = CT_TIMESTAMP_MUST_BE_ZERO;
        } else {
            /* event.timestamp = timestamp - events.len + index + 1 (checked u64). */
            if (timestamp < count) panic(s);
            const u64 ts = timestamp - count + index + 1;
            if (operation == OP_CREATE_ACCOUNTS) {
                a.timestamp = ts;
                result = create_account(s, &a);
            } else {
                t.timestamp = ts;
                result = create_transfer(s, &t);
            }
        }

        if (result != 0) {
            if (in_chain) {
                if (!chain_broken) {
                    chain_broken = 1;
                    scope_close(s, 0);
                    for (u32 ci = chain_start; ci < index; ci++) {
                        results[n].index = ci;
                        results[n].result = CT_LINKED_EVENT_FAILED;
                        n++;
                    }
                } else {
                    if (!(result == CT_LINKED_EVENT_FAILED || result == CT_LINKED_EVENT_CHAIN_OPEN)) panic(s);
                }
            }
            results[n].index = index;
            results[n].result = result;
            n++;
        }
        if (in_chain && (!linked || result == CT_LINKED_EVENT_CHAIN_OPEN)) {
            if (!chain_broken) scope_close(s, 1);
            in_chain = 0;
            chain_broken = 0;
        }
    }
    if (in_chain || chain_broken) panic(s);
    return n;
}

/* ------------------------------------------------------------------------------------------ */
/* Public API                                                                                  */
/* ------------------------------------------------------------------------------------------ */

tbo_state* tbo_init(uint64_t accounts_hint, uint64_t transfers_hint) {
    tbo_state* s = (tbo_state*)calloc(1, sizeof(tbo_state));
    map_init(&s->account_ids, accounts_hint * 2);
    map_init(&s->transfer_ids, transfers_hint * 2);
    map_init(&s->posted, 1024);
    s->accounts_cap = accounts_hint > 0 ? accounts_hint : 1024;
    s->accounts = (account_t*)malloc(s->accounts_cap * sizeof(account_t));
    s->transfers_cap = transfers_hint > 0 ? transfers_hint : 1024;
    s->transfers = (transfer_t*)malloc(s->transfers_cap * sizeof(transfer_t));
    return s;
}

void tbo_deinit(tbo_state* s) {
    if (!s) return;
    map_free(&s->account_ids);
    map_free(&s->transfer_ids);
    map_free(&s->posted);
    free(s->accounts);
    free(s->transfers);
    free(s->undo);
    free(s);
}

void tbo_reset(tbo_state* s) {
    u64 acap = s->account_ids.cap, tcap = s->transfer_ids.cap;
    map_free(&s->account_ids);
    map_free(&s->transfer_ids);
    map_free(&s->posted);
    map_init(&s->account_ids, acap);
    map_init(&s->transfer_ids, tcap);
    map_init(&s->posted, 1024);
    s->accounts_len = 0;
    s->transfers_len = 0;
    s->commit_timestamp = 0;
    s->scope_open = 0;
    s->undo_len = 0;
}

int tbo_commit(tbo_state* s, uint8_t operation, uint64_t timestamp, const void* input, uint32_t input_len,
               void* output, uint32_t output_cap, uint32_t* out_len) {
    *out_len = 0;
    if (operation < OP_CREATE_ACCOUNTS || operation > OP_LOOKUP_TRANSFERS) return TBO_STATUS_INVALID;

    /* commit asserts (state_machine.zig:518-519), for every operation. */
    if (!(timestamp > s->commit_timestamp)) return TBO_STATUS_PANIC;

    if (operation == OP_LOOKUP_ACCOUNTS || operation == OP_LOOKUP_TRANSFERS) {
        /* execute_lookup_* (state_machine.zig:700-736): ids not found are skipped; results that
         * do not fit in the output are omitted. */
        if (input_len % 16 != 0) return TBO_STATUS_INVALID;
        const u32 count = input_len / 16;
        const u32 slots = output_cap / 128;
        u32 n = 0;
        for (u32 i = 0; i < count; i++) {
            u128 id;
            memcpy(&id, (const u8*)input + (u64)i * 16, 16);
            const void* rec = operation == OP_LOOKUP_ACCOUNTS ? (const void*)accounts_get(s, id)
                                                              : (const void*)transfers_get(s, id);
            if (rec && n < slots) {
                memcpy((u8*)output + (u64)n * 128, rec, 128);
                n++;
            }
        }
        *out_len = n * 128;
        return TBO_STATUS_OK;
    }

    if (input_len % 128 != 0) return TBO_STATUS_INVALID;
    const u32 count = input_len / 128;
    if ((u64)output_cap < (u64)count * 8) return TBO_STATUS_INVALID;

    result_t* results = (result_t*)output;
    if (setjmp(s->panic_jmp)) {
        s->scope_open = 0;
        s->undo_len = 0;
        return TBO_STATUS_PANIC;
    }
    const u32 n = execute(s, operation, timestamp, input, count, results);
    *out_len = n * 8;
    return TBO_STATUS_OK;
}

int tbo_set_balances(tbo_state* s, uint64_t id_lo, uint64_t id_hi, const uint64_t balances[8]) {
    const u128 id = ((u128)id_hi << 64) | id_lo;
    map_slot* m = map_find(&s->account_ids, id);
    if (!m) return TBO_STATUS_PANIC;
    account_t* a = &s->accounts[m->value];
    a->debits_pending = ((u128)balances[1] << 64) | balances[0];
    a->debits_posted = ((u128)balances[3] << 64) | balances[2];
    a->credits_pending = ((u128)balances[5] << 64) | balances[4];
    a->credits_posted = ((u128)balances[7] << 64) | balances[6];
    return TBO_STATUS_OK;
}

uint64_t tbo_commit_timestamp(const tbo_state* s) { return s->commit_timestamp; }
uint64_t tbo_account_count(const tbo_state* s) { return s->accounts_len; }
uint64_t tbo_transfer_count(const tbo_state* s) { return s->transfers_len; }

static int cmp_id(const void* a, const void* b) {
    u128 x, y;
    memcpy(&x, a, 16);
    memcpy(&y, b, 16);
    return x < y ? -1 : (x > y ? 1 : 0);
}

uint64_t tbo_export_accounts(const tbo_state* s, void* out, uint64_t cap) {
    u64 n = s->accounts_len < cap ? s->accounts_len : cap;
    account_t* tmp = (account_t*)malloc((s->accounts_len + 1) * sizeof(account_t));
    memcpy(tmp, s->accounts, s->accounts_len * sizeof(account_t));
    qsort(tmp, s->accounts_len, sizeof(account_t), cmp_id);
    memcpy(out, tmp, n * sizeof(account_t));
    free(tmp);
    return n;
}

uint64_t tbo_export_transfers(const tbo_state* s, void* out, uint64_t cap) {
    u64 n = s->transfers_len < cap ? s->transfers_len : cap;
    transfer_t* tmp = (transfer_t*)malloc((s->transfers_len + 1) * sizeof(transfer_t));
    memcpy(tmp, s->transfers, s->transfers_len * sizeof(transfer_t));
    qsort(tmp, s->transfers_len, sizeof(transfer_t), cmp_id);
    memcpy(out, tmp, n * sizeof(transfer_t));
    free(tmp);
    return n;
}

static int cmp_u64pair(const void* a, const void* b) {
    const u64* x = (const u64*)a;
    const u64* y = (const u64*)b;
    return x[0] < y[0] ? -1 : (x[0] > y[0] ? 1 : 0);
}

uint64_t tbo_export_posted(const tbo_state* s, uint64_t* out_pairs, uint64_t cap) {
    u64 n = 0;
    u64* tmp = (u64*)malloc((s->posted.count + 1) * 2 * sizeof(u64));
    for (u64 i = 0; i < s->posted.cap; i++) {
        if (s->posted.slots[i].state == SLOT_FULL) {
            tmp[2 * n] = (u64)s->posted.slots[i].key;
            tmp[2 * n + 1] = s->posted.slots[i].value;
            n++;
        }
    }
    qsort(tmp, n, 2 * sizeof(u64), cmp_u64pair);
    u64 m = n < cap ? n : cap;
    memcpy(out_pairs, tmp, m * 2 * sizeof(u64));
    free(tmp);
    return m;
}

int tbo_sum_overflows_u64(uint64_t a, uint64_t b) { return sum_overflows_u64(a, b); }

int tbo_sum_overflows_u128(uint64_t a_lo, uint64_t a_hi, uint64_t b_lo, uint64_t b_hi) {
    return sum_overflows_u128(((u128)a_hi << 64) | a_lo, ((u128)b_hi << 64) | b_lo);
}

/* ------------------------------------------------------------------------------------------ */
/* Shard test double support (tests/harness/shard_double.py): the per-rank primitives of       */
/* include/tbgpu_shard.h restated on the CPU state, so the multi-GPU router's collectives and  */
/* fallback logic can be tested with gloo on CPU.                                              */
/* ------------------------------------------------------------------------------------------ */

int tbo_commit_routed(tbo_state* s, uint64_t n, const void* events, uint8_t* codes) {
    if (setjmp(s->panic_jmp)) return TBO_STATUS_PANIC;
    for (u64 i = 0; i < n; i++) {
        transfer_t t; /* t.timestamp = the execute timestamp assigned by the source */
        memcpy(&t, (const u8*)events + i * 128, 128);
        if (t.flags & (1 | 4 | 8 | 16 | 32)) return TBO_STATUS_INVALID; /* never routed */
        if (!(t.timestamp > s->commit_timestamp)) return TBO_STATUS_PANIC;
        codes[i] = (uint8_t)create_transfer(s, &t);
    }
    return TBO_STATUS_OK;
}

int tbo_fetch_accounts(const tbo_state* s, const uint64_t* ids, uint32_t n, void* out, uint8_t* found) {
    for (u32 i = 0; i < n; i++) {
        const u128 id = ((u128)ids[2 * i + 1] << 64) | ids[2 * i];
        const account_t* a = accounts_get(s, id);
        found[i] = a != NULL;
        if (a) memcpy((u8*)out + (u64)i * 128, a, 128);
        else memset((u8*)out + (u64)i * 128, 0, 128);
    }
    return TBO_STATUS_OK;
}

int tbo_fetch_transfers(const tbo_state* s, const uint64_t* ids, uint32_t n, void* out, uint8_t* state) {
    for (u32 i = 0; i < n; i++) {
        const u128 id = ((u128)ids[2 * i + 1] << 64) | ids[2 * i];
        const transfer_t* t = transfers_get(s, id);
        if (t) {
            memcpy((u8*)out + (u64)i * 128, t, 128);
            state[i] = (uint8_t)(1 + posted_get(s, t->timestamp));
        } else {
            memset((u8*)out + (u64)i * 128, 0, 128);
            state[i] = 0;
        }
    }
    return TBO_STATUS_OK;
}

int tbo_upsert_accounts(tbo_state* s, const void* records, uint32_t n) {
    if (setjmp(s->panic_jmp)) return TBO_STATUS_PANIC;
    for (u32 i = 0; i < n; i++) {
        account_t a;
        memcpy(&a, (const u8*)records + (u64)i * 128, 128);
        map_slot* m = map_find(&s->account_ids, a.id);
        if (m) {
            account_t* cur = &s->accounts[m->value];
            cur->debits_pending = a.debits_pending;
            cur->debits_posted = a.debits_posted;
            cur->credits_pending = a.credits_pending;
            cur->credits_posted = a.credits_posted;
        } else {
            accounts_insert(s, &a);
        }
    }
    return TBO_STATUS_OK;
}

int tbo_upsert_transfers(tbo_state* s, const void* records, const uint8_t* state, uint32_t n) {
    if (setjmp(s->panic_jmp)) return TBO_STATUS_PANIC;
    for (u32 i = 0; i < n; i++) {
        transfer_t t;
        memcpy(&t, (const u8*)records + (u64)i * 128, 128);
        const transfer_t* cur = transfers_get(s, t.id);
        if (!cur) transfers_insert(s, &t);
        const u64 ts = cur ? cur->timestamp : t.timestamp;
        if (state[i] >= 2) {
            if (map_find(&s->posted, ts)) map_remove(&s->posted, ts);
            map_put(&s->posted, ts, (u64)(state[i] - 2));
        } else if (state[i] == 1 && map_find(&s->posted, ts)) {
            map_remove(&s->posted, ts);
        }
    }
    return TBO_STATUS_OK;
}

void tbo_balance_bound(const tbo_state* s, uint64_t out[2]) {
    u128 bound = 0;
    const u128 MAX = ~(u128)0;
    for (u64 i = 0; i < s->accounts_len; i++) {
        const account_t* a = &s->accounts[i];
        u128 d, c;
        if (__builtin_add_overflow(a->debits_pending, a->debits_posted, &d)) d = MAX;
        if (__builtin_add_overflow(a->credits_pending, a->credits_posted, &c)) c = MAX;
        if (d > bound) bound = d;
        if (c > bound) bound = c;
    }
    out[0] = (u64)bound;
    out[1] = (u64)(bound >> 64);
}
