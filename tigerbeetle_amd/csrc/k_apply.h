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

    // Gather: consecutive legs of a segment go to consecutive lanes (coalesced reads), four legs
    // per thread in flight before their LDS adds.  A thread's legs j only grow, so the prepare
    // holding j is found by walking forward from the last one (s_pref[nb] = total stops the walk):
    // about one LDS read per leg, instead of a binary search whose dependent reads serialised the
    // loads of a heavy (Zipf-hot) bucket.
    u32 lo = 0;  // the last prepare whose segment starts at or before this thread's current leg
    for (u32 j0 = 0; j0 < total; j0 += 4 * APPLY_THREADS) {
        u64 w[4];
#pragma unroll
        for (u32 q = 0; q < 4; q++) {
            const u32 j = j0 + q * APPLY_THREADS + threadIdx.x;
            w[q] = 0;
            if (j < total) {
                while (s_pref[lo + 1] <= j) lo++;
                w[q] = P.leg_w[(u64)s_start[lo] + (j - s_pref[lo])];
            }
        }
#pragma unroll
        for (u32 q = 0; q < 4; q++) {
            if (w[q]) atomicAdd((unsigned long long*)&s_acc[w[q] >> LEG_AMT_BITS], (unsigned long long)(w[q] & LEG_AMT_MASK));
        }
    }
    __syncthreads();

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
