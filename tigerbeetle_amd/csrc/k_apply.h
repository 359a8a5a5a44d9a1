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

#define APPLY_HEAVY (16 * 4 * APPLY_THREADS)  // a range this long: 16 loads in flight, hot word in registers
#define APPLY_PART 32768                      // legs per part of a split bucket
#define APPLY_SPLIT_MIN LEG_SPLIT_MIN         // buckets at least this heavy are split (2 parts)
#define APPLY_EXTRA 64                        // extra workgroups of tb_apply_legs for the parts

// Gather of one bucket's legs: consecutive legs of a segment go to consecutive lanes (coalesced
// reads), Q legs per thread in flight before their LDS adds (a heavy, Zipf-hot bucket keeps more in
// flight).  A thread's legs j only grow, so the prepare holding j is searched for only past the
// last one, and not at all while j stays in it (one LDS read: the common case in a heavy bucket,
// whose binary searches per leg serialised the loads).
template <u32 Q>
__device__ static inline void tb_gather_legs(const PassArgs& P, u32 jb, u32 je, u32 nb_, const u32* s_start, const u32* s_pref,
                                             u64* s_acc, u32 hot_key = 0xFFFFFFFFu, u64* hot = nullptr) {
    u32 lo = 0;  // the last prepare whose segment starts at or before this thread's current leg
    for (u32 j0 = jb; j0 < je; j0 += Q * APPLY_THREADS) {
        u64 w[Q];
#pragma unroll
        for (u32 q = 0; q < Q; q++) {
            const u32 j = j0 + q * APPLY_THREADS + threadIdx.x;
            w[q] = 0;
            if (j < je) {
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

// Legs [jb, je) of the bucket into s_acc.  A heavy range's most frequent (slot, field) word among 256
// legs spread over it (counted in s_acc, still zero) is summed in registers, then added once: LDS
// atomics on one word serialise.
__device__ static inline void tb_gather_range(const PassArgs& P, u32 jb, u32 je, u32 nb, const u32* s_start,
                                              const u32* s_pref, u64* s_acc, u64* s_red) {
    if (je - jb < APPLY_HEAVY) {
        tb_gather_legs<4>(P, jb, je, nb, s_start, s_pref, s_acc);
        __syncthreads();
        return;
    }
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 j = jb + (u32)((u64)tid * (je - jb) / APPLY_THREADS);
    u32 p = 0;
    while (s_pref[p + 1] <= j) p++;
    const u32 key = (u32)(P.leg_w[(u64)s_start[p] + (j - s_pref[p])] >> LEG_AMT_BITS);
    const u64 before = s_acc[key];  // an earlier range's sum (the counts are taken off again below)
    __syncthreads();
    atomicAdd((unsigned long long*)&s_acc[key], 1ULL);
    __syncthreads();
    u64 best = ((s_acc[key] - before) << 32) | key;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) best = max(best, (u64)__shfl_xor((unsigned long long)best, off));
    if (lane == 0) s_red[wave] = best;
    __syncthreads();
    best = 0;
    for (u32 k = 0; k < APPLY_THREADS / 64; k++) best = max(best, s_red[k]);
    atomicAdd((unsigned long long*)&s_acc[key], ~0ULL);  // take this thread's count off again
    __syncthreads();
    const u32 hot_key = (u32)best;
    u64 hot = 0;
    tb_gather_legs<16>(P, jb, je, nb, s_start, s_pref, s_acc, hot_key, &hot);
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

// Extra legs of a heavy bucket b (one of APPLY_PART legs beyond its first part), counted over the
// buckets before it: the extra workgroups take them in this order.
__device__ static inline u32 tb_bucket_extras(u32 total) {
    return total >= APPLY_SPLIT_MIN ? (total - 1) / APPLY_PART : 0u;
}

// grid = leg_buckets + APPLY_EXTRA.  Workgroup g < leg_buckets owns bucket g.  A bucket with at least
// APPLY_SPLIT_MIN legs (a Zipf-hot account's) is cut into parts of APPLY_PART legs: its owner takes
// part 0, the extra workgroups take the others in bucket order (the owner also takes any the
// extras cannot), and every workgroup of a split bucket adds its sums with atomics (no carry under
// the certificate).  Every other bucket is summed by its owner alone and written back with plain
// read-modify-writes.
__device__ static inline void tb_apply_legs_body(const PassArgs& P, u64* s_acc);

// Dynamic LDS: [4 << leg_shift] per (slot, field) sums, then the bucket's first leg in each prepare of
// the pass and the exclusive prefix of the segment lengths (sized by the pass's prepares, not
// LEG_PREPARES_MAX: at 2048 buckets of 1024 slots that keeps a workgroup under 40 KB, four per CU).
__host__ __device__ static inline u32 tb_apply_lds_bytes(u32 leg_shift, u32 nb) {
    return (4u << leg_shift) * 8 + (2 * nb + 1) * 4;
}

__global__ __launch_bounds__(APPLY_THREADS) void tb_apply_legs(PassArgs P) {
    extern __shared__ u64 s_acc[];
    tb_kclock_start(P, 2);
    tb_apply_legs_body(P, s_acc);
    tb_kclock_end(P, 2);
}

__device__ static inline void tb_apply_legs_body(const PassArgs& P, u64* s_acc) {
    const u32 W = 1u << P.leg_shift;
    const u32 nb = P.b1 - P.b0;
    u32* s_start = (u32*)(s_acc + 4 * W);           // [nb] the bucket's first leg in each prepare
    u32* s_pref = s_start + nb;                     // [nb + 1] exclusive prefix of the segment lengths
    __shared__ u32 s_wave[APPLY_THREADS / 64];
    __shared__ u64 s_red[APPLY_THREADS / 64];
    __shared__ u32 s_pick[3];                       // extra workgroup: bucket, part; owner: its first extra index

    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);
    // Without the 64-bit certificate the resolve kernel emitted no leg: every independent ok event is
    // HZ_LATE and tb_apply_events adds it with u128 atomics.
    if (!cert64 || TB_ABL(P, ABL_LEG_WORK)) return;

    const u32 NBK = P.leg_buckets;
    const bool owner = blockIdx.x < NBK;
    if (!owner && P.leg_tot[NBK] == 0) return;  // no bucket of this pass is split
    u32 g = blockIdx.x, part = 0, first_extra = 0;
    const u32 tot_g = owner ? P.leg_tot[g] : 0u;
    if (!owner || tb_bucket_extras(tot_g)) {
        // Extra-part numbering over the buckets in order: a block scan of each bucket's extras.
        const u32 per = (NBK + APPLY_THREADS - 1) / APPLY_THREADS;
        const u32 k0 = min(NBK, threadIdx.x * per), k1 = min(NBK, k0 + per);
        u32 local = 0;
        for (u32 k = k0; k < k1; k++) local += tb_bucket_extras(P.leg_tot[k]);
        u32 all;
        u32 run = tb_block_excl_sum(local, s_wave, &all);
        const u32 e = blockIdx.x - NBK;  // this extra workgroup's part index (when !owner)
        if (threadIdx.x == 0) s_pick[0] = 0xFFFFFFFFu;
        __syncthreads();
        for (u32 k = k0; k < k1; k++) {
            const u32 x = tb_bucket_extras(P.leg_tot[k]);
            if (owner && k == g) s_pick[2] = run;
            if (!owner && e >= run && e < run + x) {
                s_pick[0] = k;
                s_pick[1] = e - run + 1;
            }
            run += x;
        }
        __syncthreads();
        if (!owner) {
            if (s_pick[0] == 0xFFFFFFFFu) return;  // more extra workgroups than extra parts
            g = s_pick[0];
            part = s_pick[1];
        } else {
            first_extra = s_pick[2];
        }
    }

    const u32 stride = NBK + 1;
    for (u32 k = threadIdx.x; k < 4 * W; k += APPLY_THREADS) s_acc[k] = 0;

    // Segment of bucket g in every prepare of the pass; each thread owns a run of prepares.
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

    const u32 extras = tb_bucket_extras(total);
    if (!extras) {
        tb_gather_range(P, 0, total, nb, s_start, s_pref, s_acc, s_red);
        // Write back into the low plane (tb_device.h BalView): word k of the bucket is (slot k/4, field
        // k%4), so consecutive threads read-modify-write consecutive 8-B words — whole lines, four
        // accounts each, and no high word (no carry under the certificate).  Every load of the
        // thread's words is issued before any store: on gfx950 a load waits for the wave's earlier
        // stores (vmcnt counts both), so a read-modify-write per word in turn was one memory round
        // trip per word.
        constexpr u32 PER = 4 * LEG_SLOTS_MAX / APPLY_THREADS;
        u64* __restrict__ bal = P.T.bal.lo + 4 * (u64)g * W;
        u64 v[PER], old[PER];
#pragma unroll
        for (u32 q = 0; q < PER; q++) {
            const u32 k = threadIdx.x + q * APPLY_THREADS;
            v[q] = k < 4 * W ? s_acc[k] : 0;
        }
#pragma unroll
        for (u32 q = 0; q < PER; q++) old[q] = v[q] ? bal[threadIdx.x + q * APPLY_THREADS] : 0;
#pragma unroll
        for (u32 q = 0; q < PER; q++) {
            if (v[q]) bal[threadIdx.x + q * APPLY_THREADS] = old[q] + v[q];  // low word: no carry (certificate)
        }
        return;
    }
    // A split bucket: this workgroup's parts, then atomic adds of its sums.
    for (u32 q = 0; q <= extras; q++) {
        const bool mine = owner ? (q == 0 || first_extra + q - 1 >= APPLY_EXTRA) : q == part;
        if (!mine) continue;
        tb_gather_range(P, q * APPLY_PART, min(total, (q + 1) * APPLY_PART), nb, s_start, s_pref, s_acc, s_red);
    }
    u64* bal = P.T.bal.lo + 4 * (u64)g * W;
    for (u32 k = threadIdx.x; k < 4 * W; k += APPLY_THREADS) {
        const u64 v = s_acc[k];
        if (v != 0) tb_atomic_add_lo_noret(bal + k, v);
    }
}

// Kernel 2b: the balance effects of every independent ok transfer that is not a leg, grid-stride,
// one event per lane — every one in a small pass (no legs: the resolve kernel has one workgroup per
// prepare, and a one-prepare pass, the replica's commit, would issue all 16K atomics of its prepare
// from a single CU), the post / voids and the wide amounts in a legs pass (none at all when the pass
// word says so: the launch exits at once).  The resolve kernel applies nothing itself, so its
// classification reads the pre-pass balances.
// The body, shared with tb_flow (PassArgs.late_in_flow): every thread of the grid calls it.
__device__ static inline void tb_apply_late(const PassArgs& P) {
    if (P.legs && !P.pass_words[PW_LATE]) return;
    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);  // every lane (a wave-wide sum)
    for (u32 pe = blockIdx.x * blockDim.x + threadIdx.x; pe < P.n; pe += gridDim.x * blockDim.x) {
        const u32 info = P.info[pe];
        // Exactly the events the resolve kernel marked: independent, ok, and not a balance leg (the
        // legs went to tb_apply_legs) — one decision, made once, so no event is applied twice or never.
        if (!(info & HZ_LATE) || (info & HZ_DEP) || (info & 0xFF) != R_OK || !(info & HZ_ACCTS)) continue;
        tb_apply_transfer(P, pe, info, P.eflags[pe], cert64);
    }
}

__global__ __launch_bounds__(256) void tb_apply_events(PassArgs P) { tb_apply_late(P); }
