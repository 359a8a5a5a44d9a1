// k_node.h — kernels of the multi-device engine (node.h): one process, N shards on N GPUs (or N
// logical shards on fewer), the exchange between them done by kernels reading their peers' HBM over
// xGMI (hipDeviceEnablePeerAccess) — no host staging, no collective library, one host round trip
// per pass (the route plan's counts).
//
// Partition: an account (record and balances) lives on owner(id) = tb_home(id, N)
// only, a transfer (record, id index entry, posted state) on home(id).  A clean create_transfers
// pass:
//   1. every source shard: tb_route_classify / _offsets / _scatter over its block of the pass's
//      prepares (k_route.h): its events grouped by home, each with its execute timestamp (limit
//      accounts are recognised by a replicated bitmap, tb_limit_maybe: no account probe);
//   2. every home: tb_node_gather pulls its run from every source's send buffer (global order:
//      sources in order, each source's run in event order); tb_node_import copies the hot record of
//      every foreign account the run names from its owner's table into the home's (the reference's
//      prefetch of the pass's accounts, src/state_machine.zig:345-506), then the routed commit with
//      owner legs (tb_owner_legs: every committed transfer's two balance legs, grouped by owner).
//      The imported entries stay for the next passes (account hot records never change after
//      create_account) until the import room fills or an account is inserted on the shard
//      (tb_pass_clear's import gate, tb_node_import_flush);
//   3. every owner: tb_node_apply_legs pulls its region of every home's legs and adds them;
//   4. every source: tb_node_replies reads each event's result code from its home's code array and
//      compacts the sparse replies of its prepares (tb_route_replies' layout).
#pragma once

#include "k_route.h"

#define NODE_WORLD_MAX 16

struct NodeGatherArgs {
    const u8* src[NODE_WORLD_MAX];    // source s's run for this home: its send buffer + its offset
    u64 start[NODE_WORLD_MAX + 1];    // exclusive prefix of the runs' lengths (events)
    u32 world;
    u8* recv;                         // [start[world]] events, back to back
};

// Consecutive lanes copy consecutive 16-B chunks of the records (coalesced on both sides; the source
// side crosses xGMI when the source is another GPU); each thread has GATHER_PER chunks in flight,
// their loads issued before any store.
#define GATHER_PER 4
__global__ __launch_bounds__(256) void tb_node_gather(NodeGatherArgs A) {
    const u64 n8 = A.start[A.world] * 8;
    const u64 base = (u64)blockIdx.x * 256 * GATHER_PER + threadIdx.x;
    u32x4 v[GATHER_PER];
#pragma unroll
    for (u32 q = 0; q < GATHER_PER; q++) {
        const u64 idx = base + q * 256;
        if (idx >= n8) continue;
        const u64 i = idx >> 3;
        u32 s = 0;
        while (s + 1 < A.world && A.start[s + 1] <= i) s++;
        v[q] = ((const u32x4*)(A.src[s] + (i - A.start[s]) * 128))[idx & 7];
    }
#pragma unroll
    for (u32 q = 0; q < GATHER_PER; q++) {
        const u64 idx = base + q * 256;
        if (idx < n8) ((u32x4*)A.recv)[idx] = v[q];
    }
}

struct NodeLegArgs {
    const u64* legs[NODE_WORLD_MAX];    // home h's leg region for this owner
    const u64* counts[NODE_WORLD_MAX];  // home h's leg count for this owner
    u64 region[NODE_WORLD_MAX];         // legs the region holds (a larger count is a panic at the home)
    u32 world;
    u32 cert64;                         // no balance can reach 2^64 this pass: low-word adds
};

// Owner side: every leg this shard owns, from every home, each naming the account's slot here (k_route.h
// NODE_LEG_WORDS: no probe).  The sums commute, so the order of homes and legs does not matter.  A leg
// whose slot is out of range or unknown (TB_NOT_FOUND: the home panicked) is skipped.
// Under the 64-bit certificate a workgroup takes a chunk of NAL_CHUNK legs and sums them per (slot,
// field) in an LDS table first, then adds each sum with one global atomic: a Zipf-hot account (C3: the
// hottest takes about a fifth of the legs) costs one atomic per chunk, not one per leg — atomics on
// one address serialise at its L2 channel.  A leg that finds no LDS entry within NAL_PROBES adds
// directly.  Without the certificate, one exact u128 atomic per leg.
#define NAL_PER 4
#define NAL_CHUNK (256 * NAL_PER)
#define NAL_TABLE 1024
#define NAL_PROBES 8
__global__ __launch_bounds__(256) void tb_node_apply_legs(Tables T, NodeLegArgs A) {
    __shared__ u64 start[NODE_WORLD_MAX + 1];  // exclusive prefix of the homes' leg counts
    if (threadIdx.x == 0) {
        u64 s = 0;
        for (u32 h = 0; h < A.world; h++) {
            start[h] = s;
            u64 c = *A.counts[h];
            if (c > A.region[h]) {  // guard (0x400): never read past a home's region
                tb_panic(T.g, PANIC_ASSERT | 0x400);
                c = A.region[h];
            }
            s += c;
        }
        start[A.world] = s;
    }
    __syncthreads();
    const u64 total = start[A.world];
    const u64 nslots = T.account_mask + 1;
    if (!A.cert64) {
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < total; i += (u64)gridDim.x * 256) {
            u32 h = 0;
            while (start[h + 1] <= i) h++;
            const u64* w = A.legs[h] + (i - start[h]) * NODE_LEG_WORDS;
            if ((w[0] >> 2) >= nslots || (w[0] >> 2) == TB_NOT_FOUND) {  // NOT_FOUND: the home panicked; else 0x800
                if ((w[0] >> 2) != TB_NOT_FOUND) tb_panic(T.g, PANIC_ASSERT | 0x800);
                continue;
            }
            tb_bal_add(T.bal, w[0] >> 2, (u32)(w[0] & 3), tb_u128(w[1], w[2]));
        }
        return;
    }
    __shared__ u64 s_key[NAL_TABLE];  // slot << 2 | field, ~0 = empty
    __shared__ u64 s_sum[NAL_TABLE];
    for (u64 c0 = (u64)blockIdx.x * NAL_CHUNK; c0 < total; c0 += (u64)gridDim.x * NAL_CHUNK) {
        for (u32 k = threadIdx.x; k < NAL_TABLE; k += 256) {
            s_key[k] = ~0ULL;
            s_sum[k] = 0;
        }
        __syncthreads();
        u64 key[NAL_PER], amt[NAL_PER];
#pragma unroll
        for (u32 q = 0; q < NAL_PER; q++) {  // consecutive lanes on consecutive legs
            const u64 i = c0 + q * 256 + threadIdx.x;
            key[q] = ~0ULL;
            amt[q] = 0;
            if (i < total) {
                u32 h = 0;
                while (start[h + 1] <= i) h++;
                const u64* w = A.legs[h] + (i - start[h]) * NODE_LEG_WORDS;
                key[q] = w[0];
                amt[q] = w[1];
            }
        }
#pragma unroll
        for (u32 q = 0; q < NAL_PER; q++) {
            if (key[q] != ~0ULL && (key[q] >> 2) >= nslots && (key[q] >> 2) != TB_NOT_FOUND) tb_panic(T.g, PANIC_ASSERT | 0x800);
            if ((key[q] >> 2) >= nslots || (key[q] >> 2) == TB_NOT_FOUND || amt[q] == 0) continue;
            u32 p = (u32)(tb_mix64(key[q]) & (NAL_TABLE - 1));
            bool placed = false;
            for (u32 r = 0; r < NAL_PROBES; r++) {
                const u64 prev = atomicCAS((unsigned long long*)&s_key[p], ~0ULL, (unsigned long long)key[q]);
                if (prev == ~0ULL || prev == key[q]) {
                    atomicAdd((unsigned long long*)&s_sum[p], (unsigned long long)amt[q]);
                    placed = true;
                    break;
                }
                p = (p + 1) & (NAL_TABLE - 1);
            }
            if (!placed) tb_bal_add_lo(T.bal, key[q] >> 2, (u32)(key[q] & 3), amt[q]);
        }
        __syncthreads();
        for (u32 k = threadIdx.x; k < NAL_TABLE; k += 256) {
            const u64 kk = s_key[k];
            if (kk != ~0ULL) tb_bal_add_lo(T.bal, kk >> 2, (u32)(kk & 3), s_sum[k]);
        }
        __syncthreads();
    }
}

// ---- partitioned account records ----------------------------------------------------------------
// Every limit account among n records (a load or an upsert of accounts, any owner) into this shard's
// bitmap.
__global__ void tb_limbits_from_records(const u8* recs, u32 n, u64* bits, u64 mask) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Account& a = *(const Account*)(recs + (u64)i * 128);
    if (a.flags & AF_LIMITS) tb_limit_set(bits, mask, tb_lo(a.id), tb_hi(a.id));
}

// Workgroup-level dedup of 128-bit ids in LDS (open addressing on the fingerprint; exact: a lane that
// meets its fingerprint compares the ids after the barrier).  A Zipf-hot id named by many lanes of a
// workgroup then costs one lane's global work, not one per lane: global atomics on one address
// serialise.  Every thread calls tb_wg_dedup_claim, then __syncthreads, then tb_wg_dedup_go.
#define WGD_SLOTS 1024
#define WGD_SKIP 0xFFFFFFFFu  // no id
#define WGD_FIRST 0xFFFFFFFEu // this lane placed the id (or the table had no room): it does the work
struct WgDedup {
    u64 tag[WGD_SLOTS];
    u64 lo[WGD_SLOTS], hi[WGD_SLOTS];
};

__device__ static inline void tb_wg_dedup_reset(WgDedup& d) {
    for (u32 k = threadIdx.x; k < WGD_SLOTS; k += blockDim.x) d.tag[k] = 0;
    __syncthreads();
}

// WGD_SKIP, WGD_FIRST, or the LDS slot holding the same fingerprint (compare after the barrier).
__device__ static inline u32 tb_wg_dedup_claim(WgDedup& d, bool want, u64 lo, u64 hi) {
    if (!want) return WGD_SKIP;
    const u64 fp = tb_fingerprint(lo, hi) | 1;
    u32 p = (u32)(tb_mix64(fp) & (WGD_SLOTS - 1));
    for (u32 r = 0; r < 16; r++) {
        const u64 prev = atomicCAS((unsigned long long*)&d.tag[p], 0ULL, (unsigned long long)fp);
        if (prev == 0) {
            d.lo[p] = lo;
            d.hi[p] = hi;
            return WGD_FIRST;
        }
        if (prev == fp) return p;
        p = (p + 1) & (WGD_SLOTS - 1);
    }
    return WGD_FIRST;
}

__device__ static inline bool tb_wg_dedup_go(const WgDedup& d, u32 st, u64 lo, u64 hi) {
    if (st == WGD_SKIP) return false;
    if (st == WGD_FIRST) return true;
    return !(d.lo[st] == lo && d.hi[st] == hi);  // another id with this fingerprint: not a duplicate
}

struct NodeTablesArgs {
    Tables T[NODE_WORLD_MAX];  // every shard's tables (device pointers; peers read over xGMI)
    u32 world;
};

// Home side, before a routed sub-pass: the hot record (id, ledger, code, flags, timestamp) of every
// foreign account the sub-pass's events name, from its owner's table, into this shard's table — what
// validate and the ordered fallback read of an account in a routed pass (its balances are the owner's
// and never read here: the router's certificate rules out every balance check, and limit and
// balancing events are sequenced).  Entries go into empty slots and stay: the next passes find them
// with one probe instead of importing again (a hot record never changes after create_account, and
// every insert of an account flushes the imports first).  An id no owner holds takes no entry
// (validate answers account_not_found), so the imports are at most the ledger's accounts.  An import never sits on an owned account's probe chain (owned accounts are only
// inserted while no import exists), and tb_node_import_flush restores the owned-only table exactly.
// One entry per id however many lanes name it (a Zipf-hot account is named by a large share of a
// pass): first the workgroup keeps one lane per distinct id (tb_wg_dedup: LDS, exact), then that lane
// claims an empty slot by a CAS of its timestamp word to a marker {bit 63, the id's 63-bit
// fingerprint} (real timestamps are below 2^63), and a lane that meets its own marker or its id
// already there stops — the winner alone reads the owner's record, writes the entry and puts the real
// timestamp last.  (Two ids with one 63-bit fingerprint meeting on one probe chain in one pass would
// import one of them only: about 2^-63 per pair, the sequencer's own fingerprint bet.)
// Returns whether it imported the id (false: another lane imports it, it is here already, or no
// owner holds it).
__device__ static inline bool tb_import_one(const Tables& H, const NodeTablesArgs& N, u64 lo, u64 hi, u32 o, u32* os_of) {
    const u64 mark = (1ULL << 63) | (tb_fingerprint(lo, hi) >> 1);
    u64 pos = tb_hash_id(lo, hi) & H.account_mask;
    u32 slot = TB_NOT_FOUND;
    // The owner's table is read only when this one lacks the id (an import is needed once per id and
    // kept: most lookups find the entry of an earlier pass and read nothing of the owner's).
    const Tables& O = N.T[o];
    u64 t_first = H.acct_hot[pos].timestamp;
    // The owner's verdict comes before any claim: an id no owner holds never takes a slot (a slot
    // claimed and released would leave a hole in the probe chain of an id imported past it).
    AccountHot a;
    u32 os = TB_NOT_FOUND;
    bool looked = false;
    for (u64 k = 0; k <= H.account_mask; k++) {
        // Plain (cached) reads: a stale one costs a failed CAS (which returns the truth) or a
        // duplicate entry, never a wrong one.
        u64* tw = &H.acct_hot[pos].timestamp;
        u64 t = k == 0 ? t_first : *tw;
        if (t == 0) {
            if (!looked) {
                const u64 opos = tb_hash_id(lo, hi) & O.account_mask;
                os = tb_account_find_from(O, lo, hi, opos, O.acct_hot[opos], &a);
                looked = true;
                if (os == TB_NOT_FOUND) return false;  // validate finds no entry: account_not_found
            }
            t = atomicCAS((unsigned long long*)tw, 0ULL, (unsigned long long)mark);
            if (t == 0) {
                slot = (u32)pos;
                break;
            }
        }
        if (t == mark) break;  // another lane is importing this id
        if (!(t >> 63)) {  // a complete entry: this id already?  (a stale read only costs a duplicate entry)
            const AccountHot* e = &H.acct_hot[pos];
            if (e->id_lo == lo && e->id_hi == hi) break;
        }
        pos = (pos + 1) & H.account_mask;
    }
    if (slot == TB_NOT_FOUND) return false;
    AccountHot* h = &H.acct_hot[slot];
    os_of[slot] = os;  // the owner's slot, for this pass's owner legs
    h->ledger = a.ledger;
    h->code = a.code;
    h->flags = a.flags;
    h->id_lo = lo;
    h->id_hi = hi;
    // No fence before the timestamp: a lane of this kernel that reads the entry before the fields
    // reach it only imports the id once more (a duplicate entry, equal by the end), and the
    // pass's next kernel sees everything.  (An agent-scope fence on gfx950 writes back and
    // invalidates the XCD's whole L2, per wave: it cost this kernel 1 ms a pass.)
    __hip_atomic_store(&h->timestamp, a.timestamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// count: the shard's live imports (tb_pass_clear's import gate), one add per workgroup that claimed any —
// none once the pass's accounts are all here (a counter every importing wave added to serialised at
// its L2 channel: 16K atomics on one word, ~0.3 ms of a 2-shard C2 pass).
__global__ __launch_bounds__(256) void tb_node_import(Tables H, NodeTablesArgs N, const u8* events, u64 n, u32 self,
                                                      u64* count, u32* os_of) {
    __shared__ WgDedup s_d;
    __shared__ u32 s_claimed;
    if (threadIdx.x == 0) s_claimed = 0;
    for (u64 base = (u64)blockIdx.x * 256; base < n; base += (u64)gridDim.x * 256) {  // uniform per workgroup
        tb_wg_dedup_reset(s_d);
        const u64 e = base + threadIdx.x;
        u64 lo[2] = {0, 0}, hi[2] = {0, 0};
        u32 o[2] = {0, 0}, st[2] = {WGD_SKIP, WGD_SKIP};
#pragma unroll
        for (u32 s = 0; s < 2; s++) {
            if (e < n) {
                const u64* w = (const u64*)(events + e * 128) + 2 + 2 * s;  // debit @16, credit @32
                lo[s] = w[0];
                hi[s] = w[1];
                o[s] = tb_home(lo[s], hi[s], N.world);
            }
            // owned here: present or absent in the owned table itself
            const bool want = e < n && !tb_id_reserved(lo[s], hi[s]) && o[s] != self;
            st[s] = tb_wg_dedup_claim(s_d, want, lo[s], hi[s]);
        }
        __syncthreads();
        u32 claimed = 0;
#pragma unroll
        for (u32 s = 0; s < 2; s++) {
            if (tb_wg_dedup_go(s_d, st[s], lo[s], hi[s]) && tb_import_one(H, N, lo[s], hi[s], o[s], os_of)) claimed++;
        }
        if (claimed) atomicAdd(&s_claimed, claimed);
        __syncthreads();
    }
    if (threadIdx.x == 0 && s_claimed) atomicAdd((unsigned long long*)count, (unsigned long long)s_claimed);
}

// Every import out of the table (each entry whose id another shard owns, or the tombstone of an id no
// owner held, under its marker): the owned-only table again.  flag: only if *flag (tb_pass_clear's
// import gate), null: always (before
// an account is inserted on this shard, or the table is read whole).
__global__ __launch_bounds__(256) void tb_node_import_flush(Tables H, u64 cap, u32 world, u32 self, const u32* flag) {
    if (flag && !*flag) return;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (u64)gridDim.x * blockDim.x) {
        const AccountHot& h = H.acct_hot[i];
        if (h.timestamp == 0) continue;
        // A tombstone id: an import's (its timestamp the import marker, bit 63) or a withdrawn create's
        // (a real timestamp: it stays, on an owned probe chain).
        const bool tomb = h.id_lo == ~0ULL && h.id_hi == ~0ULL;
        if (tomb ? (h.timestamp >> 63) != 0 : tb_home(h.id_lo, h.id_hi, world) != self) H.acct_hot[i] = AccountHot{};
    }
}

// What a routed commit on a node home needs to import (engine.hip enqueue_call: the gate in
// tb_pass_clear, then the flush and the import, before each of its sub-passes).
struct NodeImport {
    NodeTablesArgs N;
    u32 self;
    u64* count;    // the shard's live imports (persistent across passes)
    u64 room;      // imports the table has room for (2 x a sub-pass's events at most)
    u32* flag;     // tb_pass_clear's gate -> tb_node_import_flush
    u32* os_of;    // [account_cap] imported slot -> the account's slot on its owner
    u64* leg_counts = nullptr;  // the home's per-owner leg counts, zeroed by the sub-pass's tb_pass_clear
    u32 legs_n = 0;
    // Recorded after each sub-pass's owner legs: what the owners wait for (the legs and codes are
    // final there).  Host-side only (hipEvent_t).
    void* ev_legs = nullptr;
};

struct NodeReplyArgs {
    const u8* codes[NODE_WORLD_MAX];  // home h's result codes (one byte per received event)
    i64 delta[NODE_WORLD_MAX];        // code of an event sent to h at send slot q: codes[h][q + delta[h]]
    const u8* seq;                    // split pass: the sequencer's code of this block's event e at seq[e]
};

// Per-prepare sparse replies of a source's block (tb_route_replies with the codes read from their
// homes): ascending index, non-ok only.  One workgroup per prepare.
// A prepare (up to 8 x 1024 events) is one group: every event's home and slot are loaded first, then
// every code (one dependent round trip each, not one per 1024 events), then one barrier ranks all.
#define NR_K 8
__global__ __launch_bounds__(1024) void tb_node_replies(const u64* batch_off, const u8* home, const u32* slot,
                                                        NodeReplyArgs A, u32* results, u32* reply_bytes) {
    __shared__ u32 s_cnt[NR_K][1024 / 64];
    const u32 b = blockIdx.x;
    const u64 boff = batch_off[b];
    const u32 L = (u32)(batch_off[b + 1] - boff);
    u32* out = results + 2 * boff;
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    u32 running = 0;
    for (u32 c0 = 0; c0 < L; c0 += NR_K * blockDim.x) {
        u32 h[NR_K], sl[NR_K], code[NR_K];
#pragma unroll
        for (u32 q = 0; q < NR_K; q++) {
            const u32 i = c0 + q * blockDim.x + threadIdx.x;
            h[q] = i < L ? home[boff + i] : (u32)ROUTE_LOCAL;
            sl[q] = i < L ? slot[boff + i] : 0u;
        }
#pragma unroll
        for (u32 q = 0; q < NR_K; q++) {
            const u32 i = c0 + q * blockDim.x + threadIdx.x;
            code[q] = i >= L                 ? (u32)R_OK
                      : h[q] == ROUTE_LOCAL ? (u32)R_TIMESTAMP_MUST_BE_ZERO
                      : h[q] == ROUTE_DEP   ? (u32)A.seq[boff + i]
                                            : (u32)A.codes[h[q]][(i64)sl[q] + A.delta[h[q]]];
        }
        u64 m[NR_K];
#pragma unroll
        for (u32 q = 0; q < NR_K; q++) {
            m[q] = __ballot(code[q] != R_OK);
            if (lane == 0) s_cnt[q][wave] = __popcll(m[q]);
        }
        __syncthreads();
#pragma unroll
        for (u32 q = 0; q < NR_K; q++) {
            u32 wb = 0, tot = 0;
            for (u32 k = 0; k < nw; k++) {
                const u32 v = s_cnt[q][k];
                wb += k < wave ? v : 0;
                tot += v;
            }
            if (code[q] != R_OK) {
                const u32 r = running + wb + __popcll(m[q] & ((1ULL << lane) - 1));
                out[2 * r] = c0 + q * blockDim.x + threadIdx.x;
                out[2 * r + 1] = code[q];
            }
            running += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) reply_bytes[b] = running * 8;
}

// Ledger summary (tbgpu_bench_ledger_summary): u128 sums of the balance fields over every live
// slot (block-reduced, then one u128 atomic per field and block), live accounts, and slots whose
// owner under `world` is not `self` but hold a non-zero balance (world 0: no owner check).
__global__ __launch_bounds__(256) void tb_ledger_summary(Tables T, u64 cap, u32 world, u32 self, u64* out) {
    __shared__ u64 s_red[4][2][256 / 64];
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    u128 v[4] = {0, 0, 0, 0};
    u64 live = 0, stray = 0;
    if (i < cap) {
        const AccountHot& h = T.acct_hot[i];
        if (h.timestamp != 0 && !tb_id_reserved(h.id_lo, h.id_hi)) {
            const AccountBal b = tb_bal_load(T.bal, i);
            v[0] = b.debits_pending;
            v[1] = b.debits_posted;
            v[2] = b.credits_pending;
            v[3] = b.credits_posted;
            const bool owned = !world || tb_home(h.id_lo, h.id_hi, world) == self;
            live = owned ? 1 : 0;  // (a node home's imports are not its accounts)
            if (!owned && (v[0] | v[1] | v[2] | v[3]) != 0) stray = 1;
        }
    }
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int f = 0; f < 4; f++) {
        const u128 w = tb_wave_sum_u128(v[f]);
        if (lane == 0) {
            s_red[f][0][wave] = tb_lo(w);
            s_red[f][1][wave] = tb_hi(w);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        live += __shfl_xor((unsigned long long)live, off);
        stray += __shfl_xor((unsigned long long)stray, off);
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        u128 t = 0;
        for (u32 w = 0; w < 256 / 64; w++) t += tb_u128(s_red[threadIdx.x][0][w], s_red[threadIdx.x][1][w]);
        if (t != 0) tb_atomic_add_u128(out + 2 * threadIdx.x, t);
    }
    if (lane == 0 && live) atomicAdd((unsigned long long*)&out[8], (unsigned long long)live);
    if (lane == 0 && stray) atomicAdd((unsigned long long*)&out[9], (unsigned long long)stray);
}

// ---- dirty passes: the dependent subsequence, sequenced on the devices ----------------------------
// A pass with linked / post / void / balancing events or limit accounts is SPLIT (node.h
// node_split_pass): every source classifies its events; the independent ones are routed and committed
// by their homes exactly as in a clean pass; the dependent ones (and every event whose id a dependent
// event reads) are committed in order by the SEQUENCER, a scratch engine on the first device that
// holds exactly the state they read (the reference's prefetch -> commit split,
// src/state_machine.zig:345-506), and what they changed is written back to homes and owners.
//
// Dependence (the per-process protocol's rule, tigerbeetle_amd/sharded.py, and DESIGN.md §5b): a
// member of a linked chain (it or its predecessor in the prepare is linked, execute :628-692), a
// post / void (:907-1014), a balancing event (:826-846), an event on a limit-flag account
// (tigerbeetle.zig:31-39) or on an account a balancing event of the pass touches, and — so that no
// routed event creates an id a dependent event reads — every event whose id is the id or pending id
// of a dependent event.

struct NodeDepArgs {
    u8* dep1;          // [n] primary classes (0: none)
    u8* dep;           // [n] final: 1 = sequenced (the route plan's skip mask)
    u64* keys;         // [2n][2] ids and pending ids of primary-dependent events
    u64* bal;          // [2n][2] accounts of balancing events
    u64* counts;       // [0] keys, [1] balancing accounts, [2] sequenced events, [3] (host),
                       // [NODE_DC_HOME + h] sequenced events whose id is homed on h (log room there)
    u32 all;           // 1: every event is sequenced (no global certificate)
};
#define NODE_DC_HOME 4
#define NODE_DC_WORDS (NODE_DC_HOME + NODE_WORLD_MAX)

__global__ __launch_bounds__(ROUTE_THREADS) void tb_node_classify1(RouteArgs A, NodeDepArgs D) {
    const u64 e = (u64)blockIdx.x * ROUTE_THREADS + threadIdx.x;
    if (e >= A.n) return;
    const u64* w = (const u64*)(A.events + e * 128);
    const u16 flags = *(const u16*)(A.events + e * 128 + 118);
    const u32 b = tb_batch_search(A.batch_off, 0, A.nb, e);
    u8 d = D.all ? 32 : 0;
    if ((flags & TF_LINKED) || (e > A.batch_off[b] && (*(const u16*)(A.events + (e - 1) * 128 + 118) & TF_LINKED))) d |= 1;
    if (flags & (TF_POST | TF_VOID)) d |= 2;
    if (flags & (TF_BAL_DEBIT | TF_BAL_CREDIT)) d |= 4;
    if (A.limit_any && (tb_limit_maybe(A.limbits, A.limmask, w[2], w[3]) ||
                        tb_limit_maybe(A.limbits, A.limmask, w[4], w[5]))) {
        d |= 8;
    }
    D.dep1[e] = d;
    if (d) {  // the ids it reads: its own, and its pending transfer's
        const bool pv = (flags & (TF_POST | TF_VOID)) != 0;
        const u64 k = tb_wave_claim12(true, pv, &D.counts[0]);
        D.keys[2 * k] = w[0];
        D.keys[2 * k + 1] = w[1];
        if (pv) {
            D.keys[2 * k + 2] = w[8];
            D.keys[2 * k + 3] = w[9];
        }
    }
    if (flags & (TF_BAL_DEBIT | TF_BAL_CREDIT)) {
        const u64 k = tb_wave_claim(true, &D.counts[1], 2);
        D.bal[2 * k] = w[2];
        D.bal[2 * k + 1] = w[3];
        D.bal[2 * k + 2] = w[4];
        D.bal[2 * k + 3] = w[5];
    }
}

// Every source's keys or balancing accounts (whichever set is given) into this device's 64-bit key set
// (a false match only makes one more event sequenced, which is always exact).  Grid-stride over the
// lists' lengths, read from the sources' count words (peer reads: no host round trip).
struct NodeSetArgs {
    const u64* keys[NODE_WORLD_MAX];
    const u64* bal[NODE_WORLD_MAX];
    const u64* counts[NODE_WORLD_MAX];
    u32 world;
    u64* keyset;      // null: skip the keys
    u64 keyset_mask;
    u64* markset;     // null: skip the balancing accounts
    u64 markset_mask;
};

__global__ __launch_bounds__(256) void tb_node_sets(NodeSetArgs S) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u32 s = 0; s < S.world; s++) {
        const u64 nk = S.keyset ? S.counts[s][0] : 0, nb = S.markset ? S.counts[s][1] : 0;
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < nk; i += stride) {
            (void)tb_dedup_insert(S.keyset, S.keyset_mask, tb_dedup_key(S.keys[s][2 * i], S.keys[s][2 * i + 1]));
        }
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < nb; i += stride) {
            (void)tb_dedup_insert(S.markset, S.markset_mask, tb_dedup_key(S.bal[s][2 * i], S.bal[s][2 * i + 1]));
        }
    }
}

// An event on an account some balancing event of the pass touches is primary-dependent too, and its
// id joins the keys (before the key set is built): every sequenced event's id is then a key.
__global__ __launch_bounds__(ROUTE_THREADS) void tb_node_classify_marked(RouteArgs A, NodeDepArgs D, const u64* markset,
                                                                         u64 markset_mask) {
    const u64 e = (u64)blockIdx.x * ROUTE_THREADS + threadIdx.x;
    if (e >= A.n || D.dep1[e] != 0) return;
    const u64* w = (const u64*)(A.events + e * 128);
    if (tb_dedup_is_dup_or_present(markset, markset_mask, tb_dedup_key(w[2], w[3])) ||
        tb_dedup_is_dup_or_present(markset, markset_mask, tb_dedup_key(w[4], w[5]))) {
        D.dep1[e] = 16;
        const u64 k = tb_wave_claim(true, &D.counts[0]);
        D.keys[2 * k] = w[0];
        D.keys[2 * k + 1] = w[1];
    }
}

// Final: sequenced = primary-dependent, or its id is a key (the id or pending id of a primary one).
__global__ __launch_bounds__(ROUTE_THREADS) void tb_node_classify2(RouteArgs A, NodeDepArgs D, const u64* keyset, u64 keyset_mask) {
    __shared__ u32 s_home[NODE_WORLD_MAX + 1];  // per home, then the block's sequenced events
    if (threadIdx.x <= A.world) s_home[threadIdx.x] = 0;
    __syncthreads();
    const u64 e = (u64)blockIdx.x * ROUTE_THREADS + threadIdx.x;
    bool seq = false;
    if (e < A.n) {
        const u64* w = (const u64*)(A.events + e * 128);
        seq = D.dep1[e] != 0 || tb_dedup_is_dup_or_present(keyset, keyset_mask, tb_dedup_key(w[0], w[1]));
        D.dep[e] = seq ? 1 : 0;
        // The sequencer may create this event's transfer on its home: reserve a log position there
        // (counted per block in LDS, one global add per home and block).
        if (seq) atomicAdd(&s_home[tb_home(w[0], w[1], A.world)], 1u);
    }
    const u64 m = __ballot(seq);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_home[A.world], (u32)__popcll(m));
    __syncthreads();
    if (threadIdx.x <= A.world && s_home[threadIdx.x]) {
        const u32 slot = threadIdx.x == A.world ? 2 : NODE_DC_HOME + threadIdx.x;
        atomicAdd((unsigned long long*)&D.counts[slot], (unsigned long long)s_home[threadIdx.x]);
    }
}

// The sequencer's prefetch sets: 64-bit fingerprints of 128-bit ids with the id stored by the thread
// that claimed the entry.  A thread that finds its fingerprint already claimed does not wait for the
// id (two lanes of one wave must never spin on each other): it files itself on the `dups` list, and
// tb_seq_verify compares the ids once every claim is published — distinct ids with one 64-bit
// fingerprint (never seen; about 2^-64 per pair) stop the pass with PANIC_ASSERT rather than drop an
// object.
struct SeqEntry {
    u64 tag;       // fingerprint, 0 = empty
    u64 lo, hi;
    u32 x;         // its slot / log position in the sequencer (TB_NOT_FOUND: absent everywhere)
    u32 home;      // its slot / log position on its owner / home shard
};

#define SEQ_NEW 0xFFFFFFFEu  // SeqEntry.home: an account the sequencer created this pass

struct SeqSet {
    SeqEntry* e;
    u64 mask;
    u32* list;     // claimed entries, in claim order
    u64* count;    // [0] claimed, [1] dups
    u64* dups;     // [cap][3] {entry, lo, hi} of the threads that found their fingerprint claimed
};

__device__ static inline void tb_seq_insert(const SeqSet& S, u64 lo, u64 hi) {
    if (tb_id_reserved(lo, hi)) return;
    const u64 tag = tb_fingerprint(lo, hi);
    u64 pos = tb_mix64(tag) & S.mask;
    for (u64 n = 0; n <= S.mask; n++) {
        SeqEntry* q = &S.e[pos];
        // Plain (cached) reads: a Zipf-hot id is inserted by a large share of the lanes, and reads of
        // one address that bypass the cache serialise.  A stale 0 costs a CAS that returns the truth;
        // stale id words send the lane to the dups list (tb_seq_verify), never to a wrong answer.
        u64 cur = q->tag;
        if (cur == 0) cur = atomicCAS((unsigned long long*)&q->tag, 0ULL, (unsigned long long)tag);
        if (cur == 0) {
            q->lo = lo;
            q->hi = hi;
            q->x = TB_NOT_FOUND;
            q->home = TB_NOT_FOUND;
            S.list[tb_wave_claim(true, &S.count[0])] = (u32)pos;
            return;
        }
        if (cur == tag) {
            // The claimant's id, once published, settles it here (tb_seq_clear zeroed both words, and
            // an id is never 0): only a claim still in flight goes to the list for tb_seq_verify.
            if (q->lo == lo && q->hi == hi) return;
            const u64 k = tb_wave_claim(true, &S.count[1]);
            S.dups[3 * k] = pos;
            S.dups[3 * k + 1] = lo;
            S.dups[3 * k + 2] = hi;
            return;
        }
        pos = (pos + 1) & S.mask;
    }
}

__global__ void tb_seq_verify(SeqSet S, u64* panic) {
    const u64 n = S.count[1];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const SeqEntry& q = S.e[S.dups[3 * i]];
        if (q.lo != S.dups[3 * i + 1] || q.hi != S.dups[3 * i + 2]) atomicOr((unsigned long long*)panic, PANIC_ASSERT);
    }
}

// The pass as the sequencer commits it: only its sequenced events, in pass order (block-major =
// prepare order), each prepare keeping its place as the run of its own sequenced events.  Every
// chain member is sequenced and a chain never leaves its prepare, so chains stay consecutive, and a
// chain open at its prepare's end ends its compacted prepare; each event carries its execute
// timestamp (:645) in `out_ts` (PassArgs.ev_ts).  Three kernels: per-256-event counts, one scan,
// the stable scatter (wave ballots) — plus the compacted prepare offsets.  The ids the sequenced
// events read go to the transfer set.
struct SeqCompactArgs {
    const u8* src[NODE_WORLD_MAX];    // source s's block of the pass
    const u8* dep[NODE_WORLD_MAX];    // its sequenced mask
    const u64* meta[NODE_WORLD_MAX];  // its block's prepare offsets [nb + 1], then timestamps [nb]
    u32 nb[NODE_WORLD_MAX];
    u64 start[NODE_WORLD_MAX + 1];    // block starts in the pass (events)
    u32 pstart[NODE_WORLD_MAX + 1];   // block starts in the pass (prepares)
    u32 world;
    u32* blk;                         // [n_pass / 256 + 1]: sequenced events per 256-event block, then
                                      // their exclusive prefix (tb_seq_scan), blk[nblk] = the total
    u32 nblk;
    u8* out;                          // the sequencer's staging
    u64* out_ts;                      // [n_seq] execute timestamps
    u32* map;                         // [n_pass] compacted index of a sequenced event, else ~0
    u64* xmeta;                       // the sequencer's call meta: [nb_pass + 1] compacted offsets, [nb_pass] timestamps
};

__device__ static inline u32 tb_seq_source(const SeqCompactArgs& A, u64 g) {
    u32 s = 0;
    while (s + 1 < A.world && A.start[s + 1] <= g) s++;
    return s;
}

__global__ __launch_bounds__(256) void tb_seq_count(SeqCompactArgs A) {
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    bool d = false;
    if (g < A.start[A.world]) {
        const u32 s = tb_seq_source(A, g);
        d = A.dep[s][g - A.start[s]] != 0;
    }
    __shared__ u32 s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const u64 m = __ballot(d);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_cnt, (u32)__popcll(m));
    __syncthreads();
    if (threadIdx.x == 0) A.blk[blockIdx.x] = s_cnt;
}

__global__ __launch_bounds__(1024) void tb_seq_scan(SeqCompactArgs A) {
    __shared__ u32 s_wave[1024 / 64];
    const u32 n = A.nblk;
    const u32 per = (n + 1023) / 1024;
    const u32 k0 = min(n, threadIdx.x * per), k1 = min(n, k0 + per);
    u32 local = 0;
    for (u32 k = k0; k < k1; k++) local += A.blk[k];
    u32 total;
    u32 run = tb_block_excl_sum(local, s_wave, &total);
    for (u32 k = k0; k < k1; k++) {
        const u32 c = A.blk[k];
        A.blk[k] = run;
        run += c;
    }
    if (threadIdx.x == 0) A.blk[n] = total;
}

__global__ __launch_bounds__(256) void tb_seq_compact(SeqCompactArgs A, SeqSet tset) {
    __shared__ u32 s_wave[256 / 64];
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    const bool live = g < A.start[A.world];
    u32 s = 0;
    u64 e = 0;
    bool d = false;
    if (live) {
        s = tb_seq_source(A, g);
        e = g - A.start[s];
        d = A.dep[s][e] != 0;
    }
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 m = __ballot(d);
    if (lane == 0) s_wave[wave] = (u32)__popcll(m);
    __syncthreads();
    u32 before = 0;
    for (u32 w = 0; w < wave; w++) before += s_wave[w];
    if (!live) return;
    if (!d) {
        A.map[g] = 0xFFFFFFFFu;
        return;
    }
    const u32 r = A.blk[blockIdx.x] + before + (u32)__popcll(m & ((1ULL << lane) - 1));
    A.map[g] = r;
    const u64* off = A.meta[s];
    const u32 b = tb_batch_search(off, 0, A.nb[s], e);
    const u64 L = off[b + 1] - off[b];
    A.out_ts[r] = off[A.nb[s] + 1 + b] - L + 1 + (e - off[b]);  // execute, :645
    const u32x4* in = (const u32x4*)(A.src[s] + e * 128);
    u32x4 v[8];
#pragma unroll
    for (u32 k = 0; k < 8; k++) v[k] = in[k];
    u32x4* dst = (u32x4*)(A.out + (u64)r * 128);
#pragma unroll
    for (u32 k = 0; k < 8; k++) dst[k] = v[k];
    const u64* w = (const u64*)v;
    tb_seq_insert(tset, w[0], w[1]);
    if (((const u16*)v)[59] & (TF_POST | TF_VOID)) tb_seq_insert(tset, w[8], w[9]);
}

// The compacted prepare offsets: prepare k of the pass starts where its first event's compacted rank
// would be (the sequenced events before it), and ends where prepare k + 1 starts.
__global__ void tb_seq_meta(SeqCompactArgs A) {
    const u32 nbp = A.pstart[A.world];
    for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k <= nbp; k += gridDim.x * blockDim.x) {
        u64 g;
        u64 ts = 0;
        if (k == nbp) {
            g = A.start[A.world];
        } else {
            u32 s = 0;
            while (s + 1 < A.world && A.pstart[s + 1] <= k) s++;
            const u32 b = k - A.pstart[s];
            g = A.start[s] + A.meta[s][b];
            ts = A.meta[s][A.nb[s] + 1 + b];
        }
        const u64 blk = g >> 8;
        u32 r = A.blk[blk];
        for (u64 q = blk << 8; q < g; q++) {
            const u32 s = tb_seq_source(A, q);
            r += A.dep[s][q - A.start[s]] != 0;
        }
        A.xmeta[k] = r;
        if (k < nbp) A.xmeta[nbp + 1 + k] = ts;
    }
}

// The sequencer's dense codes back at their pass positions (for tb_node_replies, ROUTE_DEP).
__global__ void tb_seq_expand(SeqCompactArgs A, const u8* xcodes, u8* codes) {
    const u64 n = A.start[A.world];
    for (u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (u64)gridDim.x * blockDim.x) {
        const u32 r = A.map[g];
        if (r != 0xFFFFFFFFu) codes[g] = xcodes[r];
    }
}

// What the sequencer's pass leaves in its globals, into the first shard's (on that shard's stream, so
// nothing else writes them meanwhile): its panic bits, its latest ok timestamp, and its balance growth
// (the node's bound is the sum of the shards').  The first shard's reply arena then carries them.
__global__ void tb_seq_fold(const Globals* xg, Globals* g0, u64 bound0_lo, u64 bound0_hi) {
    if (blockIdx.x || threadIdx.x) return;
    g0->panic |= xg->panic;
    if (xg->commit_timestamp > g0->commit_timestamp) g0->commit_timestamp = xg->commit_timestamp;
    const u128 grow = tb_u128(xg->bound_lo, xg->bound_hi) - tb_u128(bound0_lo, bound0_hi);
    const u128 b = tb_sat_add(tb_u128(g0->bound_lo, g0->bound_hi), grow);
    g0->bound_lo = tb_lo(b);
    g0->bound_hi = tb_hi(b);
}

// The transfers the sequenced events read, from their homes: record, posted state, into the
// sequencer's log at [0, loaded) and its index.  Their accounts go to the account set (a post / void
// reads its pending transfer's accounts).
__global__ void tb_seq_load_transfers(NodeTablesArgs N, SeqSet tset, Tables X, u64* loaded, SeqSet aset) {
    const u64 n = tset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        SeqEntry& q = tset.e[tset.list[i]];
        const Tables& H = N.T[tb_home(q.lo, q.hi, N.world)];
        const u32 pos = tb_transfer_find(H, q.lo, q.hi);
        if (pos == TB_NOT_FOUND) continue;
        const Transfer t = H.xlog[pos];
        const u32 xp = (u32)tb_wave_claim(true, loaded);
        X.xlog[xp] = t;
        X.xposted[xp] = H.xposted[pos];
        q.x = xp;
        q.home = pos;
        // No fence: nothing in this kernel reads the record through the index (the ids are distinct);
        // the next kernel sees it.
        if (tb_transfer_claim_new(X, q.lo, q.hi, xp) == TB_NOT_FOUND) continue;  // PANIC_TABLE_FULL set
        tb_seq_insert(aset, tb_lo(t.debit_account_id), tb_hi(t.debit_account_id));
        tb_seq_insert(aset, tb_lo(t.credit_account_id), tb_hi(t.credit_account_id));
    }
}

// The accounts every sequenced event names, to the account set.
// (one lane per distinct id of the workgroup: Zipf-hot accounts are most of the names)
__global__ __launch_bounds__(256) void tb_seq_event_accounts(const u8* events, u64 n, SeqSet aset) {
    __shared__ WgDedup s_d;
    tb_wg_dedup_reset(s_d);
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    // a placeholder (or a reserved-flag event: no state read) names nothing
    const bool live = g < n && !(((const u16*)(events + g * 128))[59] & 0x8000);
    u64 lo[2] = {0, 0}, hi[2] = {0, 0};
    u32 st[2];
#pragma unroll
    for (u32 s = 0; s < 2; s++) {
        if (live) {
            const u64* w = (const u64*)(events + g * 128) + 2 + 2 * s;
            lo[s] = w[0];
            hi[s] = w[1];
        }
        st[s] = tb_wg_dedup_claim(s_d, live && !tb_id_reserved(lo[s], hi[s]), lo[s], hi[s]);
    }
    __syncthreads();
#pragma unroll
    for (u32 s = 0; s < 2; s++) {
        if (tb_wg_dedup_go(s_d, st[s], lo[s], hi[s])) tb_seq_insert(aset, lo[s], hi[s]);
    }
}

// The accounts, into the sequencer: record and balances from the owner (the only copy); the balances
// as loaded are kept (bal0[i]) so the write-back adds the sequencer's changes as deltas — the routed
// part of the pass may be adding legs to the same (free) accounts meanwhile.
__global__ void tb_seq_load_accounts(NodeTablesArgs N, SeqSet aset, Tables X, AccountBal* bal0) {
    const u64 n = aset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        SeqEntry& q = aset.e[aset.list[i]];
        const Tables& O = N.T[tb_home(q.lo, q.hi, N.world)];
        const u32 os = tb_account_find(O, q.lo, q.hi);
        if (os == TB_NOT_FOUND) continue;  // no such account
        const Account a = tb_account_load(O, os);
        if (bal0) {
            // The balances as loaded, not read again: the routed part may be adding legs to this
            // (free) account meanwhile, and the write-back's deltas must be against what the
            // sequencer started from (a second read could include a leg the first did not — and
            // the delta would cancel it).
            AccountBal b;
            b.debits_pending = a.debits_pending;
            b.debits_posted = a.debits_posted;
            b.credits_pending = a.credits_pending;
            b.credits_posted = a.credits_posted;
            bal0[i] = b;
        }
        const u32 xs = tb_account_claim(X, q.lo, q.hi, a.timestamp);
        if (xs == TB_NOT_FOUND) continue;  // PANIC_TABLE_FULL set
        tb_account_store_new(X, xs, a);
        q.x = xs;
        q.home = os;
    }
}

// Write-back, on home h: the transfers the sequencer created (its log at [base, base + n), live in its
// index) whose home is h, appended to h's log at h_base + (a per-home counter); and the posted state of
// every loaded transfer of h that the pass posted or voided.
__global__ void tb_seq_writeback_transfers(Tables X, u64 base, u64 n, SeqSet tset, Tables H, u32 self, u32 world,
                                           u64 h_base, u64* h_count) {
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const Transfer& t = X.xlog[base + i];
        if (t.timestamp == 0 || tb_home(tb_lo(t.id), tb_hi(t.id), world) != self) continue;
        if (tb_transfer_find(X, tb_lo(t.id), tb_hi(t.id)) != (u32)(base + i)) continue;  // withdrawn
        const u64 lp = h_base + tb_wave_claim(true, h_count);
        if (lp >= H.xlog_cap) {
            tb_panic(H.g, PANIC_TABLE_FULL);
            continue;
        }
        H.xlog[lp] = t;
        H.xposted[lp] = X.xposted[base + i];  // read through the index from the next kernel on (no fence)
        if (tb_transfer_claim_new(H, tb_lo(t.id), tb_hi(t.id), (u32)lp) == TB_NOT_FOUND) continue;
        (void)tb_wave_claim(true, &H.g->transfer_count);
    }
    const u64 m = tset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const SeqEntry& q = tset.e[tset.list[i]];
        if (q.x == TB_NOT_FOUND || tb_home(q.lo, q.hi, world) != self) continue;
        const u8 st = X.xposted[q.x];
        if (H.xposted[q.home] != st) H.xposted[q.home] = st;
    }
}

// Write-back, on owner o: what the sequencer changed in the balances of every account it held that o
// owns, added as u128 deltas (mod 2^128, exact in aggregate): sums commute with the routed part's
// legs on the same free accounts; a constrained account's balance only the sequencer touches.
__global__ void tb_seq_writeback_accounts(Tables X, SeqSet aset, Tables O, u32 self, u32 world, const AccountBal* bal0) {
    const u64 n = aset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const SeqEntry& q = aset.e[aset.list[i]];
        if (q.x == TB_NOT_FOUND || q.home == SEQ_NEW || tb_home(q.lo, q.hi, world) != self) continue;
        const AccountBal x = tb_bal_load(X.bal, q.x), b = bal0[i];
        if (x.debits_pending != b.debits_pending) tb_bal_add(O.bal, q.home, BAL_DP, x.debits_pending - b.debits_pending);
        if (x.debits_posted != b.debits_posted) tb_bal_add(O.bal, q.home, BAL_DPOST, x.debits_posted - b.debits_posted);
        if (x.credits_pending != b.credits_pending) tb_bal_add(O.bal, q.home, BAL_CP, x.credits_pending - b.credits_pending);
        if (x.credits_posted != b.credits_posted) tb_bal_add(O.bal, q.home, BAL_CPOST, x.credits_posted - b.credits_posted);
    }
}

// create_accounts on the sequencer (node.h node_commit_accounts): every event's id to the account set
// (its existing record is loaded from its owner: create_account_exists, state_machine.zig:767-777).
__global__ __launch_bounds__(256) void tb_seq_account_ids(const u8* events, u64 n, SeqSet aset) {
    const u64 g = (u64)blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    const u64* w = (const u64*)(events + g * 128);
    tb_seq_insert(aset, w[0], w[1]);
}

// After the sequencer's create_accounts pass: the accounts its table holds that were not loaded were
// created by the pass (a rolled-back insert is a tombstone, never found by id).
__global__ void tb_seq_locate_new(SeqSet aset, Tables X) {
    const u64 n = aset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        SeqEntry& q = aset.e[aset.list[i]];
        if (q.x != TB_NOT_FOUND) continue;
        const u32 xs = tb_account_find(X, q.lo, q.hi);
        if (xs == TB_NOT_FOUND) continue;
        q.x = xs;
        q.home = SEQ_NEW;
    }
}

// Write-back, on shard `self`: the accounts the sequencer created that it owns, inserted verbatim
// (timestamp as assigned, zero balances); every created limit account into its limit bitmap.
__global__ void tb_seq_writeback_new_accounts(Tables X, SeqSet aset, Tables O, u32 self, u32 world, u64* limbits,
                                              u64 limmask) {
    const u64 n = aset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const SeqEntry& q = aset.e[aset.list[i]];
        if (q.home != SEQ_NEW) continue;
        const Account a = tb_account_load(X, q.x);
        if (a.flags & AF_LIMITS) tb_limit_set(limbits, limmask, q.lo, q.hi);
        if (tb_home(q.lo, q.hi, world) != self) continue;
        const u32 slot = tb_account_claim(O, q.lo, q.hi, a.timestamp);
        if (slot == TB_NOT_FOUND) continue;  // PANIC_TABLE_FULL set
        tb_account_store_new(O, slot, a);
        (void)tb_wave_claim(true, &O.g->account_count);
    }
}

// The sequencer's transfer index emptied entry by entry instead of by a whole-table memset (64 MB at
// C3's pass size, 0.13 ms a split pass): every entry of X's index was claimed for one of its log
// positions under that position's id — a loaded transfer at [0, loaded) (tb_seq_load_transfers), a
// sequenced event at [base, base + n) (validate, the ordered run; a withdrawn claim is tombstoned,
// never emptied) — so scanning each id's chain for the entries naming its position finds them all.
// Pass 1 lists them with the chains intact; pass 2 empties them, their collision marks and the
// positions' posted states.  A list past `cap` (it holds 2 entries per position) makes pass 2 empty
// the whole index instead.
__global__ void tb_seq_xidx_list(Tables X, const u64* loaded, const u8* events, u64 base, u64 n, u32* list, u64* count,
                                 u64 cap) {
    const u64 L = *loaded, total = L + n;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (u64)gridDim.x * blockDim.x) {
        u64 lo, hi, pos;
        if (i < L) {
            lo = tb_lo(X.xlog[i].id);
            hi = tb_hi(X.xlog[i].id);
            pos = i;
        } else {
            const u64* w = (const u64*)(events + (i - L) * 128);
            lo = w[0];
            hi = w[1];
            pos = base + (i - L);
        }
        if (tb_id_reserved(lo, hi)) continue;  // no claim: the event failed before its id check
        const u64 fp = tb_fp32(lo, hi);
        u64 p = tb_hash_id(lo, hi) & X.xidx_mask;
        for (u64 k = 0; k <= X.xidx_mask; k++) {
            const u64 e = X.xidx[p];
            if (e == 0) break;
            if ((e >> 32) == fp && (e & XI_POS_MASK) == pos + 1) {
                const u64 at = atomicAdd((unsigned long long*)&count[0], 1ULL);
                if (at < cap) list[at] = (u32)p;
            }
            p = (p + 1) & X.xidx_mask;
        }
    }
}

__global__ void tb_seq_xidx_zero(Tables X, const u32* list, const u64* count, const u64* loaded, u64 base, u64 n,
                                 u64 cap) {
    const u64 stride = (u64)gridDim.x * blockDim.x, t0 = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 m = count[0];
    if (m > cap) {  // the list overflowed: the whole index
        for (u64 i = t0; i <= X.xidx_mask; i += stride) {
            X.xidx[i] = 0;
            X.xdup[i] = 0;
        }
    } else {
        for (u64 i = t0; i < m; i += stride) {
            X.xidx[list[i]] = 0;
            X.xdup[list[i]] = 0;
        }
    }
    const u64 L = *loaded;
    for (u64 i = t0; i < L; i += stride) X.xposted[i] = 0;
    for (u64 i = t0; i < n; i += stride) X.xposted[base + i] = 0;
}

// Empties what the pass put in the sequencer's account table and both sets (by their lists).
__global__ void tb_seq_clear(SeqSet tset, SeqSet aset, Tables X) {
    const u64 stride = (u64)gridDim.x * blockDim.x;
    const u64 na = aset.count[0], nt = tset.count[0];
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) {
        SeqEntry& q = aset.e[aset.list[i]];
        if (q.x != TB_NOT_FOUND) X.acct_hot[q.x] = AccountHot{};
        q.tag = q.lo = q.hi = 0;
    }
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += stride) {
        SeqEntry& q = tset.e[tset.list[i]];
        q.tag = q.lo = q.hi = 0;
    }
}
