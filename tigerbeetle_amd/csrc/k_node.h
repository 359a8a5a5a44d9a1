// k_node.h — kernels of the multi-device engine (node.h): one process, N shards on N GPUs (or N
// logical shards on fewer), the exchange between them done by kernels reading their peers' HBM over
// xGMI (hipDeviceEnablePeerAccess) — no host staging, no collective library, one host round trip
// per pass (the route plan's counts).
//
// Partition (as the per-process protocol of tigerbeetle_amd/sharded.py): account
// records replicated on every shard, an account's balances on owner(id) = tb_home(id, N) only, a
// transfer (record, id index entry, posted state) on home(id).  A clean create_transfers pass:
//   1. every source shard: tb_route_classify / _offsets / _scatter over its block of the pass's
//      prepares (k_route.h): its events grouped by home, each with its execute timestamp;
//   2. every home: tb_node_gather pulls its run from every source's send buffer (global order:
//      sources in order, each source's run in event order), then the routed commit with owner
//      legs (tb_owner_legs: every committed transfer's two balance legs, grouped by owner);
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

// One 16-B chunk per thread: consecutive lanes copy consecutive chunks of a record (coalesced on
// both sides; the source side crosses xGMI when the source is another GPU).
__global__ __launch_bounds__(256) void tb_node_gather(NodeGatherArgs A) {
    const u64 n = A.start[A.world];
    const u64 idx = (u64)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n * 8) return;
    const u64 i = idx >> 3;
    const u32 c = (u32)(idx & 7);
    u32 s = 0;
    while (s + 1 < A.world && A.start[s + 1] <= i) s++;
    const u32x4* in = (const u32x4*)(A.src[s] + (i - A.start[s]) * 128) + c;
    ((u32x4*)(A.recv + i * 128))[c] = *in;
}

struct NodeLegArgs {
    const u64* legs[NODE_WORLD_MAX];    // home h's leg region for this owner
    const u64* counts[NODE_WORLD_MAX];  // home h's leg count for this owner
    u32 world;
    u32 cert64;                         // no balance can reach 2^64 this pass: low-word adds
};

// Owner side: every leg this shard owns, from every home (tb_apply_owner_legs' arithmetic).  The
// sums commute, so the order of homes and legs does not matter.  A leg for an account this shard
// lacks is an invariant failure (accounts are replicated): PANIC_ASSERT.
__global__ __launch_bounds__(256) void tb_node_apply_legs(Tables T, NodeLegArgs A) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u32 h = 0; h < A.world; h++) {
        const u64 n = *A.counts[h];
        const u64* legs = A.legs[h];
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
            const u64* w = legs + i * OWNER_LEG_WORDS;
            const u64 id_lo = w[0], id_hi = w[1], a_lo = w[2], a_hi = w[3], field = w[4];
            const u32 slot = tb_account_find(T, id_lo, id_hi);
            if (slot == TB_NOT_FOUND || field > 3) {
                tb_panic(T.g, PANIC_ASSERT);
                continue;
            }
            u8* f = (u8*)&T.acct_bal[slot] + 16 * field;
            if (A.cert64) tb_atomic_add_lo_noret(f, a_lo);
            else tb_atomic_add_u128(f, tb_u128(a_lo, a_hi));
        }
    }
}

struct NodeReplyArgs {
    const u8* codes[NODE_WORLD_MAX];  // home h's result codes (one byte per received event)
    i64 delta[NODE_WORLD_MAX];        // code of an event sent to h at send slot q: codes[h][q + delta[h]]
};

// Per-prepare sparse replies of a source's block (tb_route_replies with the codes read from their
// homes): ascending index, non-ok only.  One workgroup per prepare.
__global__ __launch_bounds__(1024) void tb_node_replies(const u64* batch_off, const u8* home, const u32* slot,
                                                        NodeReplyArgs A, u32* results, u32* reply_bytes) {
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
            const u32 h = home[boff + i];
            code = h == ROUTE_LOCAL ? (u32)R_TIMESTAMP_MUST_BE_ZERO
                                    : (u32)A.codes[h][(i64)slot[boff + i] + A.delta[h]];
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
            const AccountBal b = T.acct_bal[i];
            v[0] = b.debits_pending;
            v[1] = b.debits_posted;
            v[2] = b.credits_pending;
            v[3] = b.credits_posted;
            live = 1;
            if (world && tb_home(h.id_lo, h.id_hi, world) != self && (v[0] | v[1] | v[2] | v[3]) != 0) stray = 1;
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
