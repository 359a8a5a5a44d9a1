// k_evict.h — bounded HBM residency of the transfer store (include/tbgpu.h tbgpu_evict_transfers,
// tbgpu_transfers_maybe_cold).
//
// The reference keeps every transfer reachable through its groove: the object cache first, then the
// LSM levels on disk, loaded by prefetch before commit (src/lsm/groove.zig:602-898,
// src/state_machine.zig:419-467).  Here the transfer log is HBM and finite, so a replica that
// outlives it drops the records its forest already holds (written back, §7b of DESIGN.md) and loads
// them again when a prepare names them — the same prefetch -> commit split:
//   * eviction (at a bar boundary, the stream drained): every live record before the cut goes into a
//     Bloom filter of evicted ids; the records after it slide to the front of the log (their posted
//     states with them) and the id index is rebuilt from them — so the index never holds tombstones
//     of what left, and positions, capacity and probe lengths are those of a log of the kept records;
//   * prefetch: an id the index does not hold that the filter may hold is COLD — the caller loads it
//     from its forest (tbgpu_load_transfers) before the commit, or knows it absent.  A false positive
//     costs one forest lookup, never a wrong result.
#pragma once

#include "pass.h"

#define BLOOM_K 3

__host__ __device__ static inline u64 tb_bloom_bit(u64 lo, u64 hi, u32 k, u64 mask) {
    return tb_mix64(tb_fingerprint(lo, hi) + 0x9e3779b97f4a7c15ULL * (k + 1)) & mask;
}

__device__ static inline void tb_bloom_add(u64* bits, u64 mask, u64 lo, u64 hi) {
#pragma unroll
    for (u32 k = 0; k < BLOOM_K; k++) {
        const u64 b = tb_bloom_bit(lo, hi, k, mask);
        atomicOr((unsigned long long*)&bits[b >> 6], 1ULL << (b & 63));
    }
}

__device__ static inline bool tb_bloom_maybe(const u64* bits, u64 mask, u64 lo, u64 hi) {
#pragma unroll
    for (u32 k = 0; k < BLOOM_K; k++) {
        const u64 b = tb_bloom_bit(lo, hi, k, mask);
        if (!((bits[b >> 6] >> (b & 63)) & 1)) return false;
    }
    return true;
}

// Every log position below n: a live record (the index holds it at that position) before `cut` is
// evicted (its id into the filter, counted), one at or after it is kept (live[pos - cut] = 1).
__global__ void tb_evict_scan(Tables T, u64 cut, u64 n, u64* bloom, u64 mask, u8* live, u64* evicted) {
    u64 mine = 0;
    for (u64 pos = (u64)blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += (u64)gridDim.x * blockDim.x) {
        const Transfer& t = T.xlog[pos];
        const u64 lo = tb_lo(t.id), hi = tb_hi(t.id);
        const bool alive = t.timestamp != 0 && !tb_id_reserved(lo, hi) && tb_transfer_find(T, lo, hi) == (u32)pos;
        if (pos < cut) {
            if (alive) {
                tb_bloom_add(bloom, mask, lo, hi);
                mine++;
            }
        } else {
            live[pos - cut] = alive ? 1 : 0;
        }
    }
    for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor((unsigned long long)mine, off);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd((unsigned long long*)evicted, (unsigned long long)mine);
}

// The index of the kept records at their new positions (the index was cleared; the records moved).
__global__ void tb_evict_reindex(Tables T, u64 n, const u8* live) {
    for (u64 pos = (u64)blockIdx.x * blockDim.x + threadIdx.x; pos < n; pos += (u64)gridDim.x * blockDim.x) {
        if (!live[pos]) continue;
        const Transfer& t = T.xlog[pos];
        (void)tb_transfer_claim_new(T, tb_lo(t.id), tb_hi(t.id), (u32)pos);
    }
}

// Which of n ids are cold: not in the index, maybe evicted.
__global__ void tb_cold_query(Tables T, const u64* bloom, u64 mask, const u64* ids, u32 n, u8* out) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 lo = ids[2 * i], hi = ids[2 * i + 1];
    out[i] = !tb_id_reserved(lo, hi) && tb_transfer_find(T, lo, hi) == TB_NOT_FOUND && tb_bloom_maybe(bloom, mask, lo, hi);
}
