// k_apply.h — kernel 2b of a create_transfers pass: per-account sums of the balance legs.
//
// An independent ok create_transfer adds its amount to one balance field of its debit account and
// one of its credit account (state_machine.zig:870-880).  Adding them with one global atomic per
// leg runs at the memory-side atomic rate (≈20 G random 8-B atomics/s on MI355X).
// Instead, under the 64-bit certificate (no balance word can carry this pass), the resolve kernel
// writes each leg as one 8-B word {slot-in-bucket << 2 | field, amount < 2^52} into its prepare's
// leg region grouped by bucket (bucket = slot >> leg_shift) and publishes the bucket starts
// (tb_emit_legs); a larger amount is added with an atomic there instead.  This kernel
// — one workgroup per bucket — gathers the bucket's segment of every prepare of the pass, sums the
// legs per (slot, field) in LDS, and adds each sum to its balance word with one plain
// read-modify-write: the workgroup owns the bucket's slots, so no global atomic is needed.  The
// sums are exact (mod 2^64 with no carry, by the certificate) and independent of leg order, so the
// result is the same as the reference's sequential adds.
#pragma once

#include "k_resolve.h"

// Gather of one bucket's legs: consecutive legs of a segment go to consecutive lanes (coalesced
// reads), Q legs per thread in flight before their LDS adds (a heavy, Zipf-hot bucket keeps more in
// flight).  A thread's legs j only grow, so the prepare holding j is searched for only past the
// last one, and not at all while j stays in it (one LDS read: the common case in a heavy bucket,
// whose binary searches per leg serialised the loads).
template <u32 Q>
__device__ static inline void tb_gather_legs(const PassArgs& P, u32 total, u32 nb_, const u32* s_start, const u32* s_pref,
                                             u64* s_acc, u32 hot_key = 0xFFFFFFFFu, u64* hot = nullptr) {
    u32 lo = 0;  // the last prepare whose segment starts at or before this thread's current leg
    for (u32 j0 = 0; j0 < total; j0 += Q * APPLY_THREADS) {
        u64 w[Q];
#pragma unroll
        for (u32 q = 0; q < Q; q++) {
            const u32 j = j0 + q * APPLY_THREADS + threadIdx.x;
            w[q] = 0;
            if (j < total) {
                if (s_pref[lo + 1] <= j) {  // past this prepare: binary search in the ones after it
                    u32 b = nb_;
                    lo++;
                    while (b - lo > 1) {
                        const u32 mid = (lo + b) >> 1;
                        if (s_pref[mid] <= j) lo = mid; else b = mid;
                    }
                }
                w[q] = P.leg_w[(u64)s_start[lo] + (j - s_pref[lo])];
            }
        }
#pragma unroll
        for (u32 q = 0; q < Q; q++) {
            if (!w[q]) continue;
            const u32 key = (u32)(w[q] >> LEG_AMT_BITS);
            if (hot && key == hot_key) *hot += w[q] & LEG_AMT_MASK;  // registers: LDS atomics on one word serialise
            else atomicAdd((unsigned long long*)&s_acc[key], (unsigned long long)(w[q] & LEG_AMT_MASK));
        }
    }
}

__global__ __launch_bounds__(APPLY_THREADS) void tb_apply_legs(PassArgs P) {
    extern __shared__ u64 s_acc[];                  // [4 << leg_shift] per (slot, field) sum (dynamic)
    __shared__ u32 s_start[LEG_PREPARES_MAX];       // the bucket's first leg in each prepare
    __shared__ u32 s_pref[LEG_PREPARES_MAX + 1];    // exclusive prefix of the segment lengths
    __shared__ u32 s_wave[APPLY_THREADS / 64];

    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);
    if (!cert64 || TB_ABL(P, ABL_LEG_WORK)) return;  // the resolve kernel applied every leg with u128 atomics

    const u32 g = blockIdx.x;
    const u32 W = 1u << P.leg_shift;
    const u32 nb = P.b1 - P.b0;
    const u32 stride = P.leg_buckets + 1;
    for (u32 k = threadIdx.x; k < 4 * W; k += APPLY_THREADS) s_acc[k] = 0;

    // Segment of this bucket in every prepare of the pass; each thread owns a run of prepares.
    const u32 per = (nb + APPLY_THREADS - 1) / APPLY_THREADS;
    const u32 p0 = min(nb, threadIdx.x * per), p1 = min(nb, p0 + per);
    u32 local = 0;
    for (u32 p = p0; p < p1; p++) {
        const u32* row = P.leg_off + (u64)p * stride;
        const u32 a = row[g], len = row[g + 1] - a;
        s_start[p] = (u32)(2 * (P.batch_off[P.b0 + p] - P.e0)) + a;
        s_pref[p] = len;
        local += len;
    }
    u32 total;
    u32 run = tb_block_excl_sum(local, s_wave, &total);
    for (u32 p = p0; p < p1; p++) {
        const u32 len = s_pref[p];
        s_pref[p] = run;
        run += len;
    }
    if (threadIdx.x == 0) s_pref[nb] = total;
    __syncthreads();

    // Gather (tb_gather_legs).
    if (total < 16 * 4 * APPLY_THREADS) {
        tb_gather_legs<4>(P, total, nb, s_start, s_pref, s_acc);
        __syncthreads();
    } else {
        // A heavy bucket: its most frequent (slot, field) word among 256 legs spread over it (counted
        // in s_acc, still zero) is summed in registers, then added once.
        __shared__ u64 s_red[APPLY_THREADS / 64];
        const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
        const u32 j = (u32)((u64)tid * total / APPLY_THREADS);
        u32 p = 0;
        while (s_pref[p + 1] <= j) p++;
        const u32 key = (u32)(P.leg_w[(u64)s_start[p] + (j - s_pref[p])] >> LEG_AMT_BITS);
        atomicAdd((unsigned long long*)&s_acc[key], 1ULL);
        __syncthreads();
        u64 best = (s_acc[key] << 32) | key;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) best = max(best, (u64)__shfl_xor((unsigned long long)best, off));
        if (lane == 0) s_red[wave] = best;
        __syncthreads();
        best = 0;
        for (u32 k = 0; k < APPLY_THREADS / 64; k++) best = max(best, s_red[k]);
        s_acc[key] = 0;
        __syncthreads();
        const u32 hot_key = (u32)best;
        u64 hot = 0;
        tb_gather_legs<16>(P, total, nb, s_start, s_pref, s_acc, hot_key, &hot);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) hot += __shfl_xor((unsigned long long)hot, off);
        if (lane == 0) s_red[wave] = hot;
        __syncthreads();
        if (tid == 0) {
            u64 v = 0;
            for (u32 k = 0; k < APPLY_THREADS / 64; k++) v += s_red[k];
            s_acc[hot_key] += v;
        }
        __syncthreads();
    }

    // Write back: thread k -> (slot k/4, field k%4), consecutive threads on consecutive 16-B fields.
    u8* bal = (u8*)(P.T.acct_bal + (u64)g * W);
    for (u32 k = threadIdx.x; k < 4 * W; k += APPLY_THREADS) {
        const u64 v = s_acc[k];
        if (v != 0) *(u64*)(bal + (u64)k * 16) += v;  // low word: no carry under the certificate
    }
}

// Kernel 2b of a small pass (no legs): the balance effects of every independent ok transfer, one
// event per lane.  The resolve kernel has one workgroup per prepare; left there, a one-prepare
// pass (the replica's commit) would issue all 16K atomics of its prepare from a single CU.
__global__ __launch_bounds__(256) void tb_apply_events(PassArgs P) {
    const u32 pe = blockIdx.x * 256 + threadIdx.x;
    if (pe >= P.n) return;
    const u32 info = P.info[pe];
    if ((info & HZ_DEP) || (info & 0xFF) != R_OK || !(info & HZ_ACCTS)) return;
    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);
    tb_apply_transfer(P, pe, info, P.eflags[pe], cert64);
}
