// pass.h — one device pass = N consecutive prepares (batches) of one create operation.
//
// Kernels of a pass (all on the engine stream, no host synchronisation between them):
//   1. tb_{transfers,accounts}_validate  one event per lane: stateless checks in the reference's
//      code order, hash probes of the HBM tables, the event's intrinsic result, hazard bits,
//      dedup-set inserts, balancing marks and the overflow-certificate sum S.
//   2. tb_resolve<op>                     one workgroup per prepare: dependence classification,
//      linked-chain resolution, in-place apply of independent ok events, sparse replies.
//   2b. tb_apply_legs                     one workgroup per account bucket: the legs of the
//      independent ok transfers summed per account (k_apply.h).
//   3. tb_flow (create_transfers)         the ordered fallback in parallel over the co-resident
//      grid (k_flow.h); tb_replay<op> (one workgroup) replays create_accounts passes and engines
//      whose balances were set directly.  Either writes the replies of the prepares that had
//      dependent events.
#pragma once

#include "tb_device.h"

// info word per event: [7:0] result code, [31:8] hazard bits (event flags live in eflags[]).
enum : u32 {
    HZ_KEYS = 1u << 8,       // create_accounts: inserted its id into the pass dedup set
    HZ_LIMIT = 1u << 9,      // touches an account with a limit flag (tigerbeetle.zig:31-39)
    HZ_BAL = 1u << 10,       // balancing_debit / balancing_credit event
    HZ_ACCTS = 1u << 11,     // dr/cr slots valid (marks + certificate apply)
    HZ_POSTVOID = 1u << 12,  // post_pending_transfer / void_pending_transfer
    HZ_DEP = 1u << 13,       // dependent: resolved by the ordered replay
    HZ_EVAL_OK = 1u << 14,   // returned ok when evaluated (feeds commit_timestamp)
    HZ_SPEC = 1u << 15,      // index entry rs[] claimed, record written at log_base + event
    HZ_SELFDEP = 1u << 16,   // kernel 1 already knows the event is dependent (id collision)
    HZ_PV_KEY = 1u << 17,    // post/void: pending id registered in the pass pending set
    HZ_AMT_HI = 1u << 18,    // amt_hi[] holds the amount's high word (else it is zero, not written)
    HZ_REC = 1u << 19,       // kernel 1 wrote the event's record (timestamped, amount as given) at
                             // log_base + event, under its claimed entry rs[]
    HZ_LATE = 1u << 20,      // tb_resolve: an independent ok create_transfers event that is not a
                             // balance leg — tb_apply_events applies exactly these
    HZ_INPLACE = 1u << 21,   // in-place pass (PassArgs.inplace): the event at log_base + event is its
                             // record, and kernel 1 wrote its timestamp there (read back as 0 by the
                             // ordered path, which re-evaluates the event)
};

#define SUM_SHARDS 64
#define FLOW_WORDS 16  // tb_flow's per-pass counters (k_flow.h FW_*)
#define VALIDATE_THREADS 256
#define RESOLVE_THREADS 1024
#define REPLAY_THREADS 256
#define BATCH_EVENTS_MAX 8191
#define BATCH_LDS 8192

struct PassArgs {
    u8 op;
    u32 epoch;             // pass number (never 0): balancing marks
    u32 b0, b1;            // batches [b0, b1) of the call
    u64 e0;                // first event of the pass (call-relative)
    u32 n;                 // events in the pass
    const u64* batch_off;  // [nb_call + 1] call-relative event offsets
    const u64* batch_ts;   // [nb_call] prepare timestamps
    const u8* events;      // call events (128 B each)
    const u8* events_src;  // != null: kernel 1 reads the events here (registered host memory, over
                           // PCIe) and writes them through to `events` for the later kernels
    u32* results;          // call reply area: batch k at results + 2*batch_off[k]
    u32* reply_bytes;      // [nb_call]
    // scratch, pass-relative
    u32* info;
    u16* eflags;           // event flags
    u32* dr;
    u32* cr;
    u32* ps;               // log position of the pending transfer (post/void)
    u32* rs;               // index entry claimed by the speculative insert
    u64* amt;              // amount applied, low word
    u64* amt_hi;           // high word, written only when non-zero (HZ_AMT_HI)
    u64* kid;              // create_accounts: dedup key of the id (create_transfers: recomputed from the event)
    u64* kpid;
    u32* dep_list;         // pass-relative: batch k's dependent events at dep_list + (off[k]-e0)
    u32* dep_count;        // per batch (call-relative index - b0)
    u64* dedup;
    u64 dedup_mask;
    u64* sum_shards;       // [SUM_SHARDS][2] then the pass words (PW_*)
    u64* pass_words;       // == sum_shards
    u64 log_base;          // transfer-log position of event 0 of the pass
    Tables T;
    u32 ablate;            // timing-only ablation bits (TBGPU_TIMING_KNOBS builds only: TB_ABL)
    // Routed mode (tbgpu_commit_routed_async, a shard of a multi-GPU pass): the events are this
    // shard's share of the global pass, in global order, with no linked/post/void/balancing event.
    u32 routed;            // 1: each event carries its execute timestamp in its timestamp field
    u8* codes;             // call-relative dense result codes instead of sparse replies (or null)
    u32 cert_ext;          // 0: certificate from this engine's bound; CERT_EXT_*: given by the caller
    u32 seq_pv;            // 1: balances were set directly (tbgpu_test_set_balances / upserts): every
                           // post / void is dependent, so the replay checks its pending-balance `-=`
    // Compacted prepares (a node's sequencer, node.h node_split_pass): each event's execute
    // timestamp, call-relative, instead of batch_ts - L + 1 + i — a prepare holds only its sequenced
    // events, in order, so positions no longer give timestamps.  Their own timestamp fields are the
    // caller's (timestamp_must_be_zero still applies).  Null: from batch_ts (or routed).
    const u64* ev_ts;
    // In-place pass (tbgpu_log_window): the events already sit at their transfer-log positions
    // (events + (e0 + pe) * 128 == &T.xlog[log_base + pe]).  Kernel 1 writes the timestamp of each
    // create that may commit (HZ_INPLACE: its record is the event) and no post / void record;
    // tb_resolve composes the record of each independent ok post / void over its event; the ordered
    // path stores its records as always.  No kernel reads an event's bytes after its record is
    // written, except its id and pending id, which a record keeps, and an HZ_INPLACE event's
    // timestamp, which the ordered path takes as the 0 kernel 1 checked.
    u32 inplace;
    // Balance legs (k_apply.h): with the 64-bit certificate, the balance deltas of independent ok
    // create_transfer events are written as legs, bucketed by account slot per prepare, and summed
    // per account by tb_apply_legs instead of being added with one global atomic per leg.
    u32 legs;              // 1: the legs path is enabled for this pass (the host checked the sizes)
    u32 apply_late;        // 1: no legs; tb_apply_events applies the independent ok transfers (small passes)
    u32 late_in_flow;      // 1: tb_flow applies them (tb_apply_events' work) before its own; no separate launch
    u32 leg_shift;         // bucket of an account slot = slot >> leg_shift (2^leg_shift slots each)
    u32* leg_tot;          // [leg_buckets + 1] legs per bucket in the pass (tb_emit_legs; zeroed by tb_pass_clear),
                           // then the number of buckets that reached APPLY_SPLIT_MIN
    u32 leg_buckets;       // account_cap >> leg_shift
    u32* resolve_slow;     // [pass prepares] or null: 1 = the prepare is tb_resolve's (tb_resolve_lean did not
                           // resolve it); null: tb_resolve resolves every prepare
    u64* leg_w;            // [2 * pass events] the same leg words grouped by bucket per prepare

    u32* leg_off;          // [prepares of the pass][leg_buckets + 1] bucket starts in the prepare's legs
    u32* flow_words;       // tb_flow's per-pass counters (k_flow.h, FLOW_WORDS), zeroed by tb_resolve (or null)
    u64* kclock;           // profiling (or null): this pass's launch spans, {first start, last end} of
                           // validate, resolve and apply (device wall clock), set up by tb_pass_clear
};

// Launch span of a profiled kernel (tbgpu_stats.span_ms).  Resolve and apply: the first workgroup of
// each XCD lowers the start word to its start, and every workgroup raises one of KCLOCK_ENDS end
// words (one 128-B line each, by workgroup) to its end; the host takes the maximum after the pass.
// Both are no-return atomics, so no wave waits on them.  Validate carries no stamp at all: any
// stamping code in it — even one store by one workgroup — measured 10 % slower in same-box A/B runs
// (its SGPRs already spill); its span is from the end of tb_pass_clear (the kernel before it on the
// stream, stamped by its workgroup 0 into validate's start word) to the start of tb_resolve (the one
// after it, kernel 1's start word): the two launch gaps inside were below the kernel trace's
// resolution (profiles/r04).
#define KCLOCK_ENDS 16
#define KCLOCK_LINE 16                                   // u64 words per 128-B line
#define KCLOCK_STRIDE (KCLOCK_LINE * (1 + KCLOCK_ENDS))  // per kernel: [0] start, [(1 + q) * KCLOCK_LINE] end q
#define KCLOCK_WORDS (3 * KCLOCK_STRIDE)                 // per pass: kernel 0 validate, 1 resolve, 2 apply
__device__ static inline void tb_kclock_stamp_end(u64* kernel_words) {
    atomicMax((unsigned long long*)(kernel_words + (1 + blockIdx.x % KCLOCK_ENDS) * KCLOCK_LINE),
              (unsigned long long)wall_clock64());
}
__device__ static inline void tb_kclock_start(const PassArgs& P, u32 k) {
    if (P.kclock && blockIdx.x < 8 && threadIdx.x == 0) {
        atomicMin((unsigned long long*)(P.kclock + k * KCLOCK_STRIDE), (unsigned long long)wall_clock64());
    }
}
// Every thread of the workgroup calls it (a barrier, then thread 0 stamps).
__device__ static inline void tb_kclock_end(const PassArgs& P, u32 k) {
    if (!P.kclock) return;
    __syncthreads();
    if (threadIdx.x == 0) tb_kclock_stamp_end(P.kclock + k * KCLOCK_STRIDE);
}

enum : u32 { CERT_EXT_U128 = 1, CERT_EXT_U64 = 2 };

// Legs limits: a bucket's accumulators live in LDS (4 fields x 8 B per slot), the per-prepare
// bucket histogram in the resolve workgroup's LDS, the per-prepare segment table in the apply
// workgroup's LDS.
#ifndef LEG_SLOTS_MAX
#define LEG_SLOTS_MAX 1024
#endif
#ifndef LEG_BUCKETS_PREF  // -DLEG_BUCKETS_PREF=... builds an A/B variant
#define LEG_BUCKETS_PREF 2048
#endif
#define LEG_BUCKETS_MAX 4096  // u16 counters: 8 KB of tb_resolve's LDS (under 80 KB: two workgroups per CU)
#define LEG_PREPARES_MAX 1024
#define LEG_SPLIT_MIN 65536  // tb_apply_legs splits a bucket with at least this many legs in the pass
#define LEGS_MIN_EVENTS (1u << 18)  // smaller passes apply balances with atomics (engine.hip)
#ifndef APPLY_THREADS  // -DAPPLY_THREADS=... builds an A/B variant (tools/gpu/r04_ab.sh)
#define APPLY_THREADS 256
#endif
// Leg word: ((slot within its bucket) << 2 | balance field (BAL_OFF / 16)) << LEG_AMT_BITS | amount.
// An amount of 2^LEG_AMT_BITS or more is applied by the resolve kernel with an atomic instead.
#ifndef LEG_AMT_BITS
#define LEG_AMT_BITS 52  // leaves 12 bits: slot-in-bucket (<= 10, LEG_SLOTS_MAX) + field (2)
#endif
#define LEG_AMT_MASK ((1ULL << LEG_AMT_BITS) - 1)
static_assert((1u << (64 - LEG_AMT_BITS - 2)) >= LEG_SLOTS_MAX, "leg word: slot-in-bucket field too narrow");

// Timestamp of event i of batch b (execute, state_machine.zig:645).  A routed event carries the
// timestamp its source assigned (the source answered timestamp_must_be_zero itself and never
// routed such an event).
__device__ static inline u64 tb_event_ts(const PassArgs& P, u32 b, u64 boff, u32 L, u32 i) {
    if (P.ev_ts) return P.ev_ts[boff + i];
    return P.routed ? *(const u64*)(P.events + (boff + i) * 128 + 120) : P.batch_ts[b] - L + 1 + i;
}
// Timestamps not from the prepare's position (routed, or compacted prepares).
__device__ static inline bool tb_ts_carried(const PassArgs& P) { return P.routed || P.ev_ts; }

// Timing-only ablations (A/B experiments with tools/gpu/ab.sh) exist only in a build with
// -DTBGPU_TIMING_KNOBS; in the product build every check folds to false, so no environment
// variable can switch off a validation step.
#ifdef TBGPU_TIMING_KNOBS
#define TB_ABL(P, bits) ((((P).ablate) & (bits)) != 0)
#else
#define TB_ABL(P, bits) false
#endif
enum : u32 { ABL_DEDUP = 1, ABL_SPEC = 2, ABL_ACCTS = 4, ABL_XFIND = 8, ABL_STAGE = 16, ABL_RECORD = 32, ABL_CAS = 64, EXP_NT = 128,
             ABL_LEGS = 256, ABL_LEG_STORES = 512, ABL_LEG_WORK = 1024,  // ABL_LEG_*: timing only (wrong balances)
             ABL_FLOW = 2048 };  // sequential replay instead of the parallel flow path (exact either way)

// Batch of a call-relative event index: binary search over batch_off[lo..hi) (off[lo] <= e < off[hi]).
__device__ static inline u32 tb_batch_search(const u64* off, u32 lo, u32 hi, u64 e) {
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (off[mid] <= e) lo = mid; else hi = mid;
    }
    return lo;
}

// Batch of every event of a VALIDATE_THREADS tile: one lane searches for the tile's first and last
// events, then each lane searches only that (usually one- or two-batch) range.
__device__ static inline u32 tb_tile_batch(const PassArgs& P, u64 e_first, u32 count, u64 e, u32* s_range) {
    if (threadIdx.x == 0) {
        s_range[0] = tb_batch_search(P.batch_off, P.b0, P.b1, e_first);
        s_range[1] = tb_batch_search(P.batch_off, s_range[0], P.b1, e_first + count - 1) + 1;
    }
    __syncthreads();
    return tb_batch_search(P.batch_off, s_range[0], s_range[1], e);
}

// Batch of every event of a wave: the wave's first and last events are wave-uniform, so their
// searches run on the scalar unit (s_load, no LDS, no barrier); each lane then searches only that
// (usually one- or two-batch) range.  `count` = events of the workgroup's tile.
__device__ static inline u32 tb_wave_batch(const u64* off, u32 lo, u32 hi, u64 tile_e0, u32 count, u64 e) {
    const u32 w0 = (u32)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 64;
    if (w0 >= count) return lo;
    const u64 first = tile_e0 + w0, last = tile_e0 + min(count, w0 + 64) - 1;
    const u32 a = tb_batch_search(off, lo, hi, first);
    const u32 z = tb_batch_search(off, a, hi, last) + 1;
    return tb_batch_search(off, a, z, e);
}

// Stage VALIDATE_THREADS 128-byte events through LDS with 16-byte coalesced loads.  Rows are 128 B
// with the 16-B chunks of row r XOR-swizzled by r & 7, so the per-lane ds_read_b128 of one record
// spreads over the banks without padding (32 KB per 256 events: five validate workgroups per CU).
#define STAGE_STRIDE 128
__device__ static inline u32 tb_stage_off(u32 row, u32 chunk) { return row * STAGE_STRIDE + ((chunk ^ (row & 7)) << 4); }
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ static inline void tb_stage_events(const u8* src, u32 count, u8* lds, bool nt = false, u8* copy = nullptr) {
    const u32 t = threadIdx.x;
#pragma unroll
    for (u32 r = 0; r < 8; r++) {
        const u32 c = t + r * VALIDATE_THREADS;  // 16-byte chunk index within the tile
        const u32 ev = c >> 3, part = c & 7;
        if (ev < count) {
            const u32x4* g = (const u32x4*)(src + (u64)c * 16);
            const u32x4 v = nt ? __builtin_nontemporal_load(g) : *g;
            *(u32x4*)(lds + tb_stage_off(ev, part)) = v;
            if (copy) *(u32x4*)(copy + (u64)c * 16) = v;
        }
    }
    __syncthreads();
}

// Kernel 1's tile: from the call's events, or (SRC, a separate instantiation so the HBM path's
// code is untouched) read through from registered host memory.
template <bool SRC>
__device__ static inline void tb_stage_tile(const PassArgs& P, u32 tile0, u32 count, u8* lds, bool nt = false) {
    const u64 off = (P.e0 + tile0) * 128;
    if (SRC) tb_stage_events(P.events_src + off, count, lds, false, const_cast<u8*>(P.events) + off);
    else tb_stage_events(P.events + off, count, lds, nt);
}

template <typename R>
__device__ static inline R tb_read_staged(const u8* lds) {
    R r;
#pragma unroll
    for (u32 k = 0; k < 8; k++) ((uint4*)&r)[k] = *(const uint4*)(lds + tb_stage_off(threadIdx.x, k));
    return r;
}

// Positions from one shared counter, one atomic per wave instead of one per lane (a counter every lane
// of a kernel adds to is a single L2 address: its atomics serialise).  The lanes of the wave that are
// active here with `take` set get consecutive positions, `k` each (a call from divergent code is
// fine: the ballot sees only the active lanes, and the leader is one of them).
__device__ static inline u64 tb_wave_claim(bool take, u64* count, u64 k = 1) {
    const u64 m = __ballot(take);
    if (!m) return 0;
    const u32 lane = threadIdx.x & 63;
    const u32 leader = __ffsll((long long)m) - 1;
    u64 base = 0;
    if (lane == leader) base = atomicAdd((unsigned long long*)count, (unsigned long long)(k * __popcll(m)));
    base = __shfl(base, leader);
    return base + k * __popcll(m & ((1ULL << lane) - 1));
}

// The same with a weight of 1 or 2 per lane (two = `two` set).
__device__ static inline u64 tb_wave_claim12(bool take, bool two, u64* count) {
    const u64 m = __ballot(take), m2 = __ballot(take && two);
    if (!m) return 0;
    const u32 lane = threadIdx.x & 63;
    const u32 leader = __ffsll((long long)m) - 1;
    u64 base = 0;
    if (lane == leader) base = atomicAdd((unsigned long long*)count, (unsigned long long)(__popcll(m) + __popcll(m2)));
    base = __shfl(base, leader);
    const u64 lt = (1ULL << lane) - 1;
    return base + __popcll(m & lt) + __popcll(m2 & lt);
}

// Wave-level sum of a u128 (64 lanes).
__device__ static inline u128 tb_wave_sum_u128(u128 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const u64 lo = __shfl_xor((unsigned long long)tb_lo(v), off);
        const u64 hi = __shfl_xor((unsigned long long)tb_hi(v), off);
        v = tb_sat_add(v, tb_u128(lo, hi));
    }
    return v;
}

// Add a block's partial S into one of SUM_SHARDS shards (no single hot word).  A partial at or
// above 2^100 sets the HUGE word instead, which keeps every shard total below 2^124 (at most 2^24
// blocks per pass) so the mod-2^128 shard atomics never wrap.
// Pass words after the shards: HUGE (S >= 2^100 somewhere), DUP (an id or pending-id collision
// happened), BAL (a tentatively-ok balancing event exists), PV (a post/void event registered its
// pending id), LATE (an independent ok transfer of a legs pass is not a leg: tb_apply_events applies
// it).  Written with idempotent stores.
#define PW_HUGE (2 * SUM_SHARDS)
#define PW_DUP (2 * SUM_SHARDS + 1)
#define PW_BAL (2 * SUM_SHARDS + 2)
#define PW_PV (2 * SUM_SHARDS + 3)
#define PW_LATE (2 * SUM_SHARDS + 4)
#define SUM_WORDS (2 * SUM_SHARDS + 5)
__device__ static inline void tb_sum_publish(const PassArgs& P, u128 block_sum) {
    if (block_sum == 0) return;
    if (tb_hi(block_sum) >> 36) {
        atomicOr((unsigned long long*)&P.sum_shards[PW_HUGE], 1ULL);
        return;
    }
    tb_atomic_add_u128(P.sum_shards + 2 * (blockIdx.x % SUM_SHARDS), block_sum);
}

// The pass dedup set is cleared lazily: a pass that inserts records its epoch and extent, and the
// next pass's tb_pass_clear zeroes that extent only then (a pass without post/void or
// create_accounts events leaves the set clean, and the next clear is a no-op).
__device__ static inline void tb_dedup_mark(const PassArgs& P) {
    P.T.g->dedup_dirty = ((u64)P.epoch << 8) | (u64)(64 - __clzll((long long)P.dedup_mask));
}

// Before kernel 1 of pass `epoch`: zero the S shards and pass words, and the dedup entries the
// previous pass may have written (all `cap` entries when `force`).
// meta (optional): a one-prepare call's metadata {offset 0, offset 1, timestamp}, carried here as
// kernel arguments instead of a copy ahead of the pass (the replica's one-prepare commits).
// zero_b (optional): counters of the caller zeroed here instead of by a copy each (a node home's leg
// counts, k_node.h).  imp (optional): a node home's import gate (k_node.h tb_node_import_flush):
// when its live imports plus what this sub-pass may add would pass the room, flag the flush and
// restart the count.
struct ImportGate {
    u64* count;
    u64 room, need;
    u32* flag;
};
__global__ __launch_bounds__(256) void tb_pass_clear(u64* dedup, u64 cap, u64* sum_shards, const Globals* g, u32 epoch,
                                                     u32 force, u32* leg_tot, u32 leg_buckets, u64* meta, u64 m0, u64 m1,
                                                     u64 m2, u64* kclock, ImportGate imp, u64* zero_b = nullptr,
                                                     u32 zero_b_n = 0) {
    const u64 w = g->dedup_dirty;  // before the stores (a load after them waits for them)
    if (blockIdx.x == 0 && threadIdx.x < SUM_WORDS) sum_shards[threadIdx.x] = 0;
    if (imp.count && blockIdx.x == 0 && threadIdx.x == 0) {
        const bool full = *imp.count + imp.need > imp.room;
        *imp.flag = full ? 1u : 0u;
        if (full) *imp.count = 0;
    }
    if (zero_b && blockIdx.x == 0 && threadIdx.x < zero_b_n) zero_b[threadIdx.x] = 0;
    if (kclock && blockIdx.x == 0) {
        for (u32 k = threadIdx.x; k < KCLOCK_WORDS; k += 256) kclock[k] = k % KCLOCK_STRIDE ? 0 : ~0ULL;
    }
    if (meta && blockIdx.x == 0 && threadIdx.x == 0) {
        meta[0] = m0;
        meta[1] = m1;
        meta[2] = m2;
    }
    if (blockIdx.x == 0 && leg_tot) {
        for (u32 k = threadIdx.x; k <= leg_buckets; k += 256) leg_tot[k] = 0;
    }
    u64 n = 0;
    if (force) n = cap;
    else if ((u32)(w >> 8) == epoch - 1 && w != 0) n = min(cap, 1ULL << (w & 255));
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const v4 z = {0, 0, 0, 0};
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; 2 * i < n; i += (u64)gridDim.x * 256) ((v4*)dedup)[i] = z;
    if (kclock && blockIdx.x == 0) {  // validate's span starts where this kernel ends (see KCLOCK_STRIDE)
        __syncthreads();
        if (threadIdx.x == 0) kclock[0] = wall_clock64();
    }
}

__device__ static inline u128 tb_sum_total(const u64* shards) {
    if (shards[PW_HUGE]) return TB_U128_MAX;
    u128 s = 0;
    for (int i = 0; i < SUM_SHARDS; i++) s = tb_sat_add(s, tb_u128(shards[2 * i], shards[2 * i + 1]));
    return s;
}

// The same sum over the lanes of a wave: lane l loads shard l and a butterfly of saturating adds
// leaves the total in every lane.  Saturating addition of non-negative values is exact up to the
// first carry out of 128 bits and sticky after it, so any order gives min(true sum, maxInt) as the
// sequential loop does.  Every lane of the wave must call it (all 64 active).  It replaces 64
// dependent u128 adds on the scalar unit per wave (one scalar unit serves all 16 waves of a
// 1024-thread workgroup's CU).
__device__ static inline u128 tb_sum_total_wave(const u64* shards) {
    static_assert(SUM_SHARDS == 64, "one shard per lane");
    if (shards[PW_HUGE]) return TB_U128_MAX;
    const u32 lane = threadIdx.x & 63;
    u64 lo = shards[2 * lane], hi = shards[2 * lane + 1];
    u32 sat = 0;
#pragma unroll
    for (u32 off = 1; off < 64; off <<= 1) {
        const u64 olo = __shfl_xor((unsigned long long)lo, off), ohi = __shfl_xor((unsigned long long)hi, off);
        sat |= __shfl_xor(sat, off);
        u128 r;
        sat |= tb_add_overflows(tb_u128(lo, hi), tb_u128(olo, ohi), &r) ? 1u : 0u;
        lo = tb_lo(r);
        hi = tb_hi(r);
    }
    // Equal in every lane: take lane 0's words as wave-uniform (scalar) values.
    const u32 l0 = __builtin_amdgcn_readfirstlane((u32)lo), l1 = __builtin_amdgcn_readfirstlane((u32)(lo >> 32));
    const u32 h0 = __builtin_amdgcn_readfirstlane((u32)hi), h1 = __builtin_amdgcn_readfirstlane((u32)(hi >> 32));
    if (__builtin_amdgcn_readfirstlane(sat)) return TB_U128_MAX;
    return tb_u128(((u64)l1 << 32) | l0, ((u64)h1 << 32) | h0);
}

// The pass's overflow certificate (k_resolve.h header).  Every kernel of the pass between validate
// and replay computes the same answer: S is final after validate and `bound` only moves at the end
// of the replay kernel.
//   cert_global: bound + S fits in u128 — no overflow check of create_transfer can fire;
//   cert64:      bound + S < 2^64 — no balance word can carry this pass.
// Every lane of the calling wave must call it (tb_sum_total_wave).
__device__ static inline void tb_pass_cert(const PassArgs& P, u128& S, bool& cert_global, bool& cert64) {
    S = tb_sum_total_wave(P.sum_shards);
    u128 r;
    // S saturates at maxInt(u128) (and the HUGE word reads as maxInt): such an S is a lower bound
    // of the true sum, not an upper one, so it certifies nothing.
    cert_global = S != TB_U128_MAX && !tb_add_overflows(tb_u128(P.T.g->bound_lo, P.T.g->bound_hi), S, &r);
    cert64 = cert_global && tb_hi(r) == 0;
    if (P.cert_ext) {  // routed shard: the router certified the global bound + S
        cert_global = true;
        cert64 = P.cert_ext == CERT_EXT_U64;
    }
}

// Exclusive prefix sum of one u32 per thread over the workgroup; *total = the sum.  Every thread
// calls it; s_wave holds blockDim.x / 64 words.
__device__ static inline u32 tb_block_excl_sum(u32 v, u32* s_wave, u32* total) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    u32 x = v;
#pragma unroll
    for (u32 off = 1; off < 64; off <<= 1) {
        const u32 o = __shfl_up(x, off);
        if (lane >= off) x += o;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    u32 before = 0, tot = 0;
    for (u32 k = 0; k < nwaves; k++) {
        const u32 c = s_wave[k];
        before += k < wave ? c : 0;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

// In-place exclusive scan of s[0, n) in LDS, s[n] = the total (which must fit T).  Every thread
// calls it.
template <typename T>
__device__ static inline void tb_block_scan_lds(T* s, u32 n, u32* s_wave) {
    const u32 per = (n + blockDim.x - 1) / blockDim.x;
    const u32 k0 = min(n, threadIdx.x * per), k1 = min(n, k0 + per);
    u32 local = 0;
    for (u32 k = k0; k < k1; k++) local += s[k];
    u32 total;
    u32 run = tb_block_excl_sum(local, s_wave, &total);
    for (u32 k = k0; k < k1; k++) {
        const u32 c = s[k];
        s[k] = (T)run;
        run += c;
    }
    if (threadIdx.x == 0) s[n] = (T)total;
    __syncthreads();
}
