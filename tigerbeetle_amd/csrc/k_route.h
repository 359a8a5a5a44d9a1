// k_route.h — multi-GPU routing of a create_transfers pass (include/tbgpu_shard.h).
//
// Partition: account records are replicated on every rank, account balances are
// per-rank partial sums, and a transfer (record, id index entry, posted state) lives on
// home(id).  A CLEAN pass — no linked / post / void / balancing event, no limit-flag account,
// global overflow certificate — is decided entirely by each event's home: id uniqueness and the
// exists checks are home-local and no free account's balance is read by create_transfer
// (state_machine.zig:779-884 reads balances only for balancing :826-846, the overflow checks
// :848-861 and the limit checks :863-868).  So a clean pass is
//   1. tb_route_classify + tb_route_offsets + tb_route_scatter on every rank: the rank's events
//      grouped by home (stable: global order survives), each carrying its execute timestamp
//      (:645) in its timestamp field — one send buffer for the all-to-all.  An event whose
//      timestamp field is non-zero fails with timestamp_must_be_zero before touching any state
//      (execute :643), so its source answers it and never routes it;
//   2. a routed commit on every home (the normal validate/resolve/replay kernels in routed mode);
//   3. tb_route_replies: the codes that came back, compacted into per-prepare sparse replies.
// Dirty passes use the prefetch/write-back kernels at the bottom (tb_fetch_*, tb_upsert_*).
#pragma once

#include "pass.h"

#define ROUTE_THREADS 256
#define ROUTE_WORLD_MAX 64
#define ROUTE_LOCAL 0xFF
#define SLOT_LOCAL 0xFFFFFFFFu
#define ROUTE_DEP 0xFE       // home of a skipped (dependent) event
#define SLOT_DEP 0xFFFFFFFEu  // its slot

enum : u32 { ROUTE_DIRTY_FLAGS = 1, ROUTE_DIRTY_LIMIT = 2 };

// home(id) / owner(id): tb_home (tb_device.h).

// Limit flags, replicated: one bit per hash bucket of ids, set for every account created or loaded
// with debits_must_not_exceed_credits / credits_must_not_exceed_debits (tigerbeetle.zig:31-39).  A
// source classifies its events with it instead of reading account records it does not hold; a false
// positive (another id in the bucket) only sequences an event that could have been routed, which is
// always exact.  The bucket hash is independent of the table position and owner bits.
__host__ __device__ static inline u64 tb_limit_bit(u64 lo, u64 hi, u64 mask) {
    return tb_mix64(tb_hash_id(lo, hi) ^ 0x9e3779b97f4a7c15ULL) & mask;
}
__device__ static inline bool tb_limit_maybe(const u64* bits, u64 mask, u64 lo, u64 hi) {
    if (tb_id_reserved(lo, hi)) return false;
    const u64 b = tb_limit_bit(lo, hi, mask);
    return (bits[b >> 6] >> (b & 63)) & 1;
}
__device__ static inline void tb_limit_set(u64* bits, u64 mask, u64 lo, u64 hi) {
    const u64 b = tb_limit_bit(lo, hi, mask);
    atomicOr((unsigned long long*)&bits[b >> 6], 1ULL << (b & 63));
}

struct RouteArgs {
    const u8* events;      // this rank's events of the pass, back to back
    u32 n;
    u32 nb;
    const u64* batch_off;  // [nb + 1]
    const u64* batch_ts;   // [nb]
    u32 world;
    u32 nblocks;
    u8* home;              // [n] home rank, or ROUTE_LOCAL (answered by the source)
    u32* block_counts;     // [nblocks][world] events of block blk for home h
    u32* block_base;       // [nblocks][world] send-buffer position of those events
    u64* words;            // [2*SUM_SHARDS] S shards, [2*SUM_SHARDS] HUGE, [+1] dirty bits, [+2..] counts
    Tables T;
    const u8* skip;        // [n] or null: non-zero = a dependent event the sequencer commits (not routed)
    // Node engines (records partitioned, node.h): limit accounts by the replicated bitmap
    // (k_node.h tb_limit_maybe), not by this shard's records; limit_any = 0: none exists.  Null:
    // records replicated (the per-process protocol), probe T.
    const u64* limbits;
    u64 limmask;
    u32 limit_any;
    // Non-null (a one-prepare block of a node call): tb_route_classify writes the block's metadata
    // {0, n, im_ts} here (= batch_off / batch_ts) from its arguments, instead of a host copy.
    u64* im_meta;
    u64 im_ts;
};
#define RW_HUGE (2 * SUM_SHARDS)
#define RW_DIRTY (2 * SUM_SHARDS + 1)
#define RW_COUNTS (2 * SUM_SHARDS + 2)
#define ROUTE_WORDS (RW_COUNTS + ROUTE_WORLD_MAX)

// Pass 1: home of every event, dirty bits, S (saturating sum of amounts: every potential
// increment of any balance), per-block home histogram.
__global__ __launch_bounds__(ROUTE_THREADS) void tb_route_classify(RouteArgs A) {
    __shared__ u32 s_cnt[ROUTE_WORLD_MAX];
    __shared__ u64 s_sum[2 * (ROUTE_THREADS / 64)];
    __shared__ u32 s_dirty;
    if (threadIdx.x < A.world) s_cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_dirty = 0;
    if (A.im_meta && blockIdx.x == 0 && threadIdx.x == 0) {  // read by the kernels after this one
        A.im_meta[0] = 0;
        A.im_meta[1] = A.n;
        A.im_meta[2] = A.im_ts;
    }
    __syncthreads();
    const u64 e = (u64)blockIdx.x * ROUTE_THREADS + threadIdx.x;
    const bool limits = A.limbits ? A.limit_any != 0 : A.T.g->limit_accounts != 0;
    u128 amount = 0;
    if (e < A.n) {
        const u64* w = (const u64*)(A.events + e * 128);
        const u64 id_lo = w[0], id_hi = w[1];
        const u16 flags = *(const u16*)(A.events + e * 128 + 118);
        if (A.skip && A.skip[e]) {
            A.home[e] = ROUTE_DEP;  // committed in order by the pass's sequencer
            amount = tb_u128(w[6], w[7]);
        } else if (w[15] != 0) {
            A.home[e] = ROUTE_LOCAL;  // timestamp_must_be_zero, answered at the source
        } else {
            const u32 h = tb_home(id_lo, id_hi, A.world);
            A.home[e] = (u8)h;
            atomicAdd(&s_cnt[h], 1u);
            amount = tb_u128(w[6], w[7]);
        }
        u32 dirty = 0;
        if (flags & (TF_LINKED | TF_POST | TF_VOID | TF_BAL_DEBIT | TF_BAL_CREDIT)) {
            dirty = ROUTE_DIRTY_FLAGS;
        } else if (limits && A.limbits) {
            if (tb_limit_maybe(A.limbits, A.limmask, w[2], w[3]) || tb_limit_maybe(A.limbits, A.limmask, w[4], w[5])) {
                dirty = ROUTE_DIRTY_LIMIT;
            }
        } else if (limits) {  // no limit account exists (C2/C5): no account probe at all
            const u32 d = tb_account_find(A.T, w[2], w[3]);
            const u32 c = tb_account_find(A.T, w[4], w[5]);
            const u16 lim = AF_DEBITS_MUST_NOT_EXCEED_CREDITS | AF_CREDITS_MUST_NOT_EXCEED_DEBITS;
            if ((d != TB_NOT_FOUND && (A.T.acct_hot[d].flags & lim)) ||
                (c != TB_NOT_FOUND && (A.T.acct_hot[c].flags & lim))) {
                dirty = ROUTE_DIRTY_LIMIT;
            }
        }
        if (dirty) atomicOr(&s_dirty, dirty);
    }
    const u128 ws = tb_wave_sum_u128(amount);
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        s_sum[2 * wave] = tb_lo(ws);
        s_sum[2 * wave + 1] = tb_hi(ws);
    }
    __syncthreads();
    if (threadIdx.x < A.world) A.block_counts[(u64)blockIdx.x * A.world + threadIdx.x] = s_cnt[threadIdx.x];
    if (threadIdx.x == 0) {
        u128 total = 0;
        for (u32 k = 0; k < ROUTE_THREADS / 64; k++) total = tb_sat_add(total, tb_u128(s_sum[2 * k], s_sum[2 * k + 1]));
        if (total != 0) {
            if (tb_hi(total) >> 36) atomicOr((unsigned long long*)&A.words[RW_HUGE], 1ULL);
            else tb_atomic_add_u128(A.words + 2 * (blockIdx.x % SUM_SHARDS), total);
        }
        if (s_dirty) atomicOr((unsigned long long*)&A.words[RW_DIRTY], (unsigned long long)s_dirty);
    }
}

// Pass 2: exclusive bases, one workgroup per home (all homes at once).  block_base[blk][h] is the
// send-buffer position of block blk's first event for home h: homes in rank order, blocks in order
// within a home.  Workgroup h scans its home's column and sums the columns of the homes before it
// (its base) in the same sweep; each thread owns a contiguous run of blocks (one contiguous span of
// counts), and the scan is a shuffle scan (two barriers).
__global__ __launch_bounds__(1024) void tb_route_offsets(RouteArgs A) {
    __shared__ u32 s_wave[1024 / 64];
    const u32 h = blockIdx.x;
    const u32 per = (A.nblocks + 1023) / 1024;
    const u32 b0 = min(A.nblocks, threadIdx.x * per), b1 = min(A.nblocks, b0 + per);
    u32 local = 0, before = 0;
    for (u32 b = b0; b < b1; b++) {
        const u32* row = A.block_counts + (u64)b * A.world;
        for (u32 k = 0; k <= h; k++) {
            const u32 v = row[k];
            if (k < h) before += v;
            else local += v;
        }
    }
    u32 home_total, base;
    const u32 run0 = tb_block_excl_sum(local, s_wave, &home_total);
    tb_block_excl_sum(before, s_wave, &base);
    u32 run = base + run0;
    for (u32 b = b0; b < b1; b++) {
        A.block_base[(u64)b * A.world + h] = run;
        run += A.block_counts[(u64)b * A.world + h];
    }
    if (threadIdx.x == 0) A.words[RW_COUNTS + h] = home_total;
}

// After a plan (node engines): its words into the source's mapped host copy, the device words
// zeroed for the plan after next of this parity (so no memset precedes a plan), then `seq` into the
// word at `done` with system scope — the host spins on it instead of waiting for the route stream.
// One wave: every load is issued before the first store into mapped memory (gfx950's vmcnt counts
// stores too), and its stores drain before the flag.
__global__ __launch_bounds__(64) void tb_route_publish(u64* words, u64* host_words, u32* done, u32 seq) {
    constexpr u32 R = (ROUTE_WORDS + 63) / 64;
    u64 v[R];
#pragma unroll
    for (u32 r = 0; r < R; r++) {
        const u32 i = r * 64 + threadIdx.x;
        v[r] = i < ROUTE_WORDS ? words[i] : 0;
    }
#pragma unroll
    for (u32 r = 0; r < R; r++) {
        const u32 i = r * 64 + threadIdx.x;
        if (i < ROUTE_WORDS) {
            host_words[i] = v[r];
            words[i] = 0;
        }
    }
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pass 3: stable scatter into the send buffer, with the execute timestamp of every event.  A tile's
// events for one home land at consecutive send positions, so the tile is written cooperatively: eight
// lanes per event, each a 16-B chunk, the events in tile order — a wave's store covers eight whole
// records, mostly contiguous (one store per lane per record would put 64 records' partial lines in
// every store instruction).
__global__ __launch_bounds__(ROUTE_THREADS) void tb_route_scatter(RouteArgs A, u8* send_events, u32* slot) {
    __shared__ __attribute__((aligned(16))) u8 stage[ROUTE_THREADS * STAGE_STRIDE];
    __shared__ u32 s_wcnt[ROUTE_THREADS / 64][ROUTE_WORLD_MAX];
    __shared__ u32 s_range[2];
    __shared__ u32 s_pos[ROUTE_THREADS];  // each event's send position (SLOT_LOCAL: not routed)
    const u64 tile0 = (u64)blockIdx.x * ROUTE_THREADS;
    const u32 count = (u32)min((u64)ROUTE_THREADS, A.n - tile0);
    tb_stage_events(A.events + tile0 * 128, count, stage);
    const u64 e = tile0 + threadIdx.x;
    const bool live = threadIdx.x < count;
    const u32 h = live ? A.home[e] : 0xFFFFFFFFu;
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 before = 0;
    for (u32 k = 0; k < A.world; k++) {
        const u64 m = __ballot(h == k);
        if (h == k) before = __popcll(m & ((1ULL << lane) - 1));
        if (lane == 0) s_wcnt[wave][k] = __popcll(m);
    }
    // Batch of every event (for its timestamp).
    if (threadIdx.x == 0) {
        s_range[0] = tb_batch_search(A.batch_off, 0, A.nb, tile0);
        s_range[1] = tb_batch_search(A.batch_off, s_range[0], A.nb, tile0 + count - 1) + 1;
    }
    __syncthreads();
    u32 pos = SLOT_LOCAL;
    if (live && (h == ROUTE_LOCAL || h == ROUTE_DEP)) {
        slot[e] = h == ROUTE_LOCAL ? SLOT_LOCAL : SLOT_DEP;
    } else if (live) {
        pos = A.block_base[(u64)blockIdx.x * A.world + h] + before;
        for (u32 w = 0; w < wave; w++) pos += s_wcnt[w][h];
        const u32 b = tb_batch_search(A.batch_off, s_range[0], s_range[1], e);
        const u64 boff = A.batch_off[b];
        const u32 L = (u32)(A.batch_off[b + 1] - boff);
        slot[e] = pos;
        *(u64*)(stage + tb_stage_off(threadIdx.x, 7) + 8) = A.batch_ts[b] - L + 1 + (e - boff);  // execute, :645
    }
    s_pos[threadIdx.x] = pos;
    __syncthreads();
#pragma unroll
    for (u32 r = 0; r < 8; r++) {
        const u32 c = threadIdx.x + r * ROUTE_THREADS;  // chunk c: event c / 8, part c % 8
        const u32 j = c >> 3, part = c & 7;
        if (j < count && s_pos[j] != SLOT_LOCAL) {
            ((u32x4*)(send_events + (u64)s_pos[j] * 128))[part] = *(const u32x4*)(stage + tb_stage_off(j, part));
        }
    }
}

// Dependency classes of every event of a dirty pass (its source's share), for the split commit
// (tigerbeetle_amd/sharded.py): a dependent event is committed in global order by the pass's
// sequencer, the others are routed to their homes as in a clean pass.  Bits: 1 member of a linked
// chain (execute :628-692: an event is in a chain if it or its predecessor in the prepare is
// linked), 2 post / void (:907-1014), 4 balancing (:826-846), 8 an account with a limit flag
// (tigerbeetle.zig:31-39), 16 an account a balancing event of the pass touches (`marked`: sorted
// {lo, hi} pairs, by hi then lo).
__device__ static inline bool tb_route_marked(const u64* marked, u32 n, u64 lo, u64 hi) {
    u32 a = 0, b = n;
    while (a < b) {
        const u32 m = (a + b) >> 1;
        const u64 mh = marked[2 * m + 1], ml = marked[2 * m];
        if (mh < hi || (mh == hi && ml < lo)) a = m + 1; else b = m;
    }
    return a < n && marked[2 * a] == lo && marked[2 * a + 1] == hi;
}

__global__ __launch_bounds__(ROUTE_THREADS) void tb_route_dependents(RouteArgs A, const u64* marked, u32 n_marked,
                                                                    u8* dep) {
    const u64 e = (u64)blockIdx.x * ROUTE_THREADS + threadIdx.x;
    if (e >= A.n) return;
    const u64* w = (const u64*)(A.events + e * 128);
    const u16 flags = *(const u16*)(A.events + e * 128 + 118);
    const u32 b = tb_batch_search(A.batch_off, 0, A.nb, e);
    u8 d = 0;
    if ((flags & TF_LINKED) || (e > A.batch_off[b] && (*(const u16*)(A.events + (e - 1) * 128 + 118) & TF_LINKED))) d |= 1;
    if (flags & (TF_POST | TF_VOID)) d |= 2;
    if (flags & (TF_BAL_DEBIT | TF_BAL_CREDIT)) d |= 4;
    if (A.T.g->limit_accounts != 0) {
        const u32 dr = tb_account_find(A.T, w[2], w[3]);
        const u32 cr = tb_account_find(A.T, w[4], w[5]);
        if ((dr != TB_NOT_FOUND && (A.T.acct_hot[dr].flags & AF_LIMITS)) ||
            (cr != TB_NOT_FOUND && (A.T.acct_hot[cr].flags & AF_LIMITS))) {
            d |= 8;
        }
    }
    if (n_marked && (tb_route_marked(marked, n_marked, w[2], w[3]) || tb_route_marked(marked, n_marked, w[4], w[5]))) {
        d |= 16;
    }
    dep[e] = d;
}

// home(id) of n {lo, hi} ids (device buffers): where a key a dependent event reads lives.
__global__ void tb_route_homes(const u64* ids, u64 n, u32 world, u8* out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (u8)tb_home(ids[2 * i], ids[2 * i + 1], world);
}

// Per-prepare sparse replies from the codes that came back (in send order): ascending index,
// non-ok only (tb_write_replies' layout).  One workgroup per prepare.
__global__ __launch_bounds__(1024) void tb_route_replies(const u64* batch_off, const u32* slot, const u8* codes,
                                                        u32* results, u32* reply_bytes) {
    __shared__ u32 s_wave[1024 / 64];
    const u32 b = blockIdx.x;
    const u64 boff = batch_off[b];
    const u32 L = (u32)(batch_off[b + 1] - boff);
    u32* out = results + 2 * boff;
    u32 running = 0;
    for (u32 c = 0; c < L; c += blockDim.x) {
        const u32 i = c + threadIdx.x;
        u32 code = R_OK;
        if (i < L) {
            const u32 s = slot[boff + i];
            code = s == SLOT_LOCAL ? R_TIMESTAMP_MUST_BE_ZERO : codes[s];
        }
        const u64 m = __ballot(code != R_OK);
        const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) s_wave[wave] = __popcll(m);
        __syncthreads();
        u32 wb = 0, tot = 0;
        for (u32 k = 0; k < blockDim.x / 64; k++) {
            wb += k < wave ? s_wave[k] : 0;
            tot += s_wave[k];
        }
        if (code != R_OK) {
            const u32 r = running + wb + __popcll(m & ((1ULL << lane) - 1));
            out[2 * r] = i;
            out[2 * r + 1] = code;
        }
        running += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) reply_bytes[b] = running * 8;
}

// ---- dirty-pass prefetch / write-back ----------------------------------------------------------

// Prefetch of transfers by id (groove get, state_machine.zig:1079-1082): record + state
// (0 absent, 1 + POSTED_* otherwise: the posted groove entry, :1084-1089).
__global__ void tb_fetch_transfers(Tables T, const u64* ids, u32 n, u8* out, u8* state) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 pos = tb_transfer_find(T, ids[2 * i], ids[2 * i + 1]);
    if (pos == TB_NOT_FOUND) {
        state[i] = 0;
        return;
    }
    *(Transfer*)(out + (u64)i * 128) = T.xlog[pos];
    state[i] = 1 + T.xposted[pos];
}

// Insert accounts verbatim (metadata + balances + timestamp), or overwrite the balances of an
// existing one.  Ids within one call are distinct.  status: bit0 table full.
// if_absent (tbgpu_load_accounts): only accounts the table does not hold are inserted; a resident
// account is newer than any copy from the forest and stays as it is.
__global__ void tb_upsert_accounts(Tables T, const u8* recs, u32 n, u32* status, u32 if_absent, BalView snap) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Account a = *(const Account*)(recs + (u64)i * 128);
    u32 slot = tb_account_find(T, tb_lo(a.id), tb_hi(a.id));
    if (slot != TB_NOT_FOUND) {
        if (if_absent) return;
        AccountBal b;
        b.debits_pending = a.debits_pending;
        b.debits_posted = a.debits_posted;
        b.credits_pending = a.credits_pending;
        b.credits_posted = a.credits_posted;
        tb_bal_store(T.bal, slot, b);
        return;
    }
    slot = tb_account_claim(T, tb_lo(a.id), tb_hi(a.id), a.timestamp);
    if (slot == TB_NOT_FOUND) {
        atomicOr(status, 1u);
        return;
    }
    tb_account_store_new(T, slot, a);
    if (snap.lo) tb_bal_store(snap, slot, tb_bal_load(T.bal, slot));  // loaded from the forest: written back already
    atomicAdd((unsigned long long*)&T.g->account_count, 1ULL);
}

// Insert transfers verbatim at the end of the log (state = 1 + POSTED_*), or set the posted state
// of an existing one (state != 0).  Ids within one call are distinct.
__global__ void tb_upsert_transfers(Tables T, const u8* recs, const u8* state, u32 n, u64 log_base, u32* counter,
                                    u32* status, u32 if_absent, u8* snap_posted) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Transfer& t = *(const Transfer*)(recs + (u64)i * 128);
    const u32 pos = tb_transfer_find(T, tb_lo(t.id), tb_hi(t.id));
    const u8 st = state[i];
    if (pos != TB_NOT_FOUND) {
        if (if_absent) return;
        if (st) T.xposted[pos] = st - 1;
        return;
    }
    const u64 lp = log_base + atomicAdd(counter, 1u);
    if (lp >= T.xlog_cap) {
        atomicOr(status, 1u);
        return;
    }
    T.xlog[lp] = t;
    T.xposted[lp] = st ? st - 1 : POSTED_NONE;
    if (snap_posted) snap_posted[lp] = T.xposted[lp];  // read through the index from the next kernel on (no fence)
    if (tb_transfer_claim_new(T, tb_lo(t.id), tb_hi(t.id), (u32)lp) == TB_NOT_FOUND) atomicOr(status, 1u);
    atomicAdd((unsigned long long*)&T.g->transfer_count, 1ULL);
}

// ---- owner-partitioned balances ------------------------------------------------------------------
// An account's balances live on owner(id) = tb_home(id, world) only (every other rank keeps zeros
// there); the immutable account fields are replicated, so every home validates with local probes.
// After a routed pass, every committed transfer's two balance deltas (state_machine.zig:870-880:
// debits_{pending,posted} of the debit account, credits_{pending,posted} of the credit account)
// become LEGS routed to the owners (all-to-all) and added there (tb_apply_owner_legs).
//   * independent events were not applied here (the pass skips tb_apply_events), so each emits both
//     legs, to whichever owner, itself included;
//   * dependent events (id collisions replayed in order by tb_flow / tb_replay) were applied to the
//     local table by the replay: a leg whose owner is another rank goes there and the local copy is
//     cancelled (adds are mod 2^128; free balances feed no check in a clean pass, so the transient
//     local value is never read).
// Leg on the wire: {account id lo, hi, amount lo, hi, field (BAL_DP .. BAL_CPOST)}.  The node engine
// (os_of set) sends the account's slot on its owner instead of its id — {slot << 2 | field, amount lo,
// hi} — so the owner adds without a probe: an owned account's slot is the home's own, an imported
// one's is what the import read (tb_node_import's os_of).
#define OWNER_LEG_WORDS 5
#define NODE_LEG_WORDS 3

struct OwnerLegArgs {
    u32 world;
    u32 self;
    u64* legs;      // [world][cap][words]: owner o's legs at legs + o * cap * words
    u64 cap;        // legs per owner region
    u64* counts;    // [world] legs written per owner (zeroed by the host before the call)
    const u32* os_of;  // node engine: [home slot] -> owner slot of an imported account (null: id legs)
    u32 words;      // OWNER_LEG_WORDS (id legs) or NODE_LEG_WORDS (slot legs)
};

// The tile's records are staged through LDS (coalesced 16-B chunks) and each thread reads the fields
// it needs (accounts, amount, flags) from there: a per-thread 128-B record load would put 64
// records' partial lines in every load instruction.
__global__ __launch_bounds__(256) void tb_owner_legs(PassArgs P, OwnerLegArgs O) {
    static_assert(VALIDATE_THREADS == 256, "tb_stage_events stages 256 records");
    __shared__ __attribute__((aligned(16))) u8 stage[256 * STAGE_STRIDE];
    __shared__ u32 s_cnt[ROUTE_WORLD_MAX];
    __shared__ u64 s_base[ROUTE_WORLD_MAX];
    if (threadIdx.x < O.world) s_cnt[threadIdx.x] = 0;
    const u32 tile0 = blockIdx.x * 256;
    tb_stage_events((const u8*)(P.T.xlog + P.log_base + tile0), (u32)min((u64)256, P.n - tile0), stage);  // (syncs)
    const u32 pe = tile0 + threadIdx.x;
    u32 owner[2] = {0, 0}, pos[2] = {0, 0}, oslot[2] = {0, 0};
    bool emit[2] = {false, false};
    u128 acct[2] = {0, 0}, amount = 0;
    u32 field0 = 0;
    if (pe < P.n && P.codes[P.e0 + pe] == R_OK) {
        const u64* c1 = (const u64*)(stage + tb_stage_off(threadIdx.x, 1));  // debit account id
        const u64* c2 = (const u64*)(stage + tb_stage_off(threadIdx.x, 2));  // credit account id
        const u64* c3 = (const u64*)(stage + tb_stage_off(threadIdx.x, 3));  // amount
        const u16 flags = *(const u16*)(stage + tb_stage_off(threadIdx.x, 7) + 6);  // @118
        acct[0] = tb_u128(c1[0], c1[1]);
        acct[1] = tb_u128(c2[0], c2[1]);
        amount = tb_u128(c3[0], c3[1]);
        const u32 info = P.info[pe];
        const bool dep = (info & HZ_DEP) != 0;
        field0 = (flags & TF_PENDING) ? 0 : 1;  // debits_pending / debits_posted (+2: credits)
#pragma unroll
        for (u32 s = 0; s < 2; s++) {
            const u128 id = acct[s];
            owner[s] = tb_home(tb_lo(id), tb_hi(id), O.world);
            emit[s] = !(dep && owner[s] == O.self);
            if (emit[s]) pos[s] = atomicAdd(&s_cnt[owner[s]], 1u);
            if (!emit[s] || (!dep && !O.os_of)) continue;
            // This shard's slot of the account (validate's, or a probe for an event it did not reach).
            const u32 slot = (info & HZ_ACCTS) ? (s ? P.cr[pe] : P.dr[pe]) : tb_account_find(P.T, tb_lo(id), tb_hi(id));
            if (slot == TB_NOT_FOUND) {  // an ok event's account is always here: invariant failure
                tb_panic(P.T.g, PANIC_ASSERT);
                oslot[s] = TB_NOT_FOUND;  // the owner skips it (its position in the region is taken)
                continue;
            }
            if (slot > P.T.account_mask) {  // guard (diagnostic panic bit 0x100)
                tb_panic(P.T.g, PANIC_ASSERT | 0x100);
                oslot[s] = TB_NOT_FOUND;
                continue;
            }
            if (O.os_of) {
                oslot[s] = owner[s] == O.self ? slot : O.os_of[slot];
                if (oslot[s] > P.T.account_mask) {  // guard (0x200): shards share one table size
                    tb_panic(P.T.g, PANIC_ASSERT | 0x200);
                    oslot[s] = TB_NOT_FOUND;
                }
            }
            if (dep) {  // cancel the replay's local add: the owner applies it
                tb_bal_add(P.T.bal, slot, field0 + 2 * s, (u128)0 - amount);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < O.world) {
        const u32 c = s_cnt[threadIdx.x];
        s_base[threadIdx.x] = c ? atomicAdd((unsigned long long*)&O.counts[threadIdx.x], (unsigned long long)c) : 0;
    }
    __syncthreads();
#pragma unroll
    for (u32 s = 0; s < 2; s++) {
        if (!emit[s]) continue;
        const u64 k = s_base[owner[s]] + pos[s];
        if (k >= O.cap) {  // the host sized every region for the whole call
            tb_panic(P.T.g, PANIC_ASSERT);
            continue;
        }
        u64* w = O.legs + ((u64)owner[s] * O.cap + k) * O.words;
        if (O.os_of) {
            w[0] = ((u64)oslot[s] << 2) | (field0 + 2 * s);
            w[1] = tb_lo(amount);
            w[2] = tb_hi(amount);
            continue;
        }
        w[0] = tb_lo(acct[s]);
        w[1] = tb_hi(acct[s]);
        w[2] = tb_lo(amount);
        w[3] = tb_hi(amount);
        w[4] = field0 + 2 * s;
    }
}

// Owner side: add every received leg to its account's balance field (the sums commute, so arrival
// order does not matter).  cert64: the router's certificate bounds every balance below 2^64 this
// pass, so the adds are low-word no-return atomics.
__global__ __launch_bounds__(256) void tb_apply_owner_legs(Tables T, const u64* legs, u64 n, u32 cert64, u32* status) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64* w = legs + i * OWNER_LEG_WORDS;
    const u32 slot = tb_account_find(T, w[0], w[1]);
    if (slot == TB_NOT_FOUND || w[4] > 3) {
        atomicOr(status, 1u);
        return;
    }
    if (cert64) tb_bal_add_lo(T.bal, slot, (u32)w[4], w[2]);
    else tb_bal_add(T.bal, slot, (u32)w[4], tb_u128(w[2], w[3]));
}
