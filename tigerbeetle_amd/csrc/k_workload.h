// k_workload.h — synthetic workload generators for bench.py (BASELINE.json configs), on device so
// 100M-transfer inputs are produced in HBM without a host round trip.
//
// Shapes follow the reference benchmark client (src/benchmark.zig:223-327): ids from
// IdPermutation.inversion (src/testing/id.zig:31: id = maxInt(u128) - data, data = index + 1),
// ledger 2, account code 1, transfer code = random u16 +| 1, amount = Exp(mean 10 000) +| 1,
// random user_data, dr != cr uniform.  The PRNG is a counter-based splitmix64 (the exact Zig
// DefaultPrng stream is not reproduced).
#pragma once

#include "tb_device.h"

__host__ __device__ static inline u64 tb_splitmix(u64 x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

__device__ static inline u64 tb_rand(u64 seed, u64 index, u64 stream) {
    return tb_splitmix(tb_splitmix(seed ^ (stream * 0xd1b54a32d192ed03ULL)) + index);
}

__device__ static inline u64 tb_range(u64 r, u64 n) { return (u64)(((u128)r * n) >> 64); }

struct WorkloadParams {
    u64 seed;
    u64 account_count;
    u64 first_index;      // transfer index of element 0
    u32 kind;             // WK_UNIFORM (C2), WK_ZIPF_LIMITS (C3), WK_TWO_PHASE (C4)
    u32 limit_permille;   // accounts with debits_must_not_exceed_credits, per mille (account 0 never)
    double zipf_s;        // C3: Zipf exponent over account ranks
    u64 perm_a, perm_b;   // C3: rank r -> account (perm_a * r + perm_b) mod account_count (gcd = 1)
    u32 hot_limited;      // C3: ranks [0, hot_limited) are limit accounts too (account 0 never)
};

enum : u32 { WK_UNIFORM = 0, WK_ZIPF_LIMITS = 1, WK_TWO_PHASE = 2 };

// C3 funding amount: bank (account 0) -> each limit account, as the first transfers of the stream.
#define WK_FUND_AMOUNT 1000000ULL
// C4 mix, per mille.
#define WK_CHAIN_BLOCK_PERMILLE 320   // blocks of 8 events that open a chain (2..8 members): ~20% of events
#define WK_CHAIN_INVALID_PERMILLE 50  // chain members with ledger 0 (chain-breaking)
#define WK_POST_VOID_PERMILLE 150     // events that post or void an earlier transfer
#define WK_PENDING_PERMILLE 300       // other events that are pending (timeout 0 or 1..10 s)
#define WK_BALANCING_PERMILLE 5       // other events with balancing_debit / balancing_credit

__device__ static inline u128 tb_wk_account_id(u64 idx) { return TB_U128_MAX - (u128)(idx + 1); }
__device__ static inline u128 tb_wk_transfer_id(u64 k) { return TB_U128_MAX - (u128)(k + 1); }

__device__ static inline bool tb_wk_limited(const WorkloadParams& W, u64 idx) {
    if (idx == 0) return false;
    for (u32 r = 0; r < W.hot_limited; r++) {
        if ((u64)(((u128)W.perm_a * r + W.perm_b) % W.account_count) == idx) return true;
    }
    return W.limit_permille && tb_range(tb_rand(W.seed, idx, 17), 1000) < W.limit_permille;
}

// Exp(mean 10 000) +| 1 (benchmark.zig:309): u in (0, 1].
__device__ static inline u64 tb_wk_amount(const WorkloadParams& W, u64 k) {
    const double u = ((double)(tb_rand(W.seed, k, 8) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
    return (u64)(-log(u) * 10000.0) + 1;
}

__device__ static inline double tb_u01(u64 r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }

// Zipf(s) over ranks 1..N by rejection-inversion (Hörmann & Derflinger 1996), exact for s != 1.
__device__ static inline double tb_zipf_H(double x, double s) {  // ∫ t^-s, shifted so H(1) = 0
    const double lx = log(x), t = (1.0 - s) * lx;
    return fabs(t) > 1e-8 ? expm1(t) / t * lx : lx * (1.0 + 0.5 * t);
}
__device__ static inline double tb_zipf_Hinv(double y, double s) {
    double t = y * (1.0 - s);
    if (t < -1.0) t = -1.0;
    return exp(fabs(t) > 1e-8 ? log1p(t) / t * y : y * (1.0 - 0.5 * t));
}
__device__ static inline u64 tb_zipf(const WorkloadParams& W, u64 k, u64 stream) {
    const double s = W.zipf_s, n = (double)W.account_count;
    const double hx1 = tb_zipf_H(1.5, s) - 1.0, hn = tb_zipf_H(n + 0.5, s);
    const double sq = 2.0 - tb_zipf_Hinv(tb_zipf_H(2.5, s) - pow(2.0, -s), s);
    for (u64 it = 0;; it++) {
        const double u = hn + tb_u01(tb_rand(W.seed, k, stream + 64 * it)) * (hx1 - hn);
        const double x = tb_zipf_Hinv(u, s);
        double r = floor(x + 0.5);
        r = r < 1.0 ? 1.0 : (r > n ? n : r);
        if (r - x <= sq || u >= tb_zipf_H(r + 0.5, s) - pow(r, -s) || it == 63) {
            const u64 rank = (u64)r - 1;  // 0 = hottest
            return (u64)(((u128)W.perm_a * rank + W.perm_b) % W.account_count);
        }
    }
}

// C4 helpers: is transfer k a post/void event; is it created pending (used by later post/voids).
__device__ static inline bool tb_wk_post_void(const WorkloadParams& W, u64 k, bool chained) {
    return !chained && tb_range(tb_rand(W.seed, k, 10), 1000) < WK_POST_VOID_PERMILLE;
}
__device__ static inline bool tb_wk_chained(const WorkloadParams& W, u64 k, bool* linked) {
    const u64 g = k >> 3, pos = k & 7;
    const bool chain = tb_range(tb_rand(W.seed, g, 20), 1000) < WK_CHAIN_BLOCK_PERMILLE;
    const u64 len = 2 + tb_range(tb_rand(W.seed, g, 21), 7);
    *linked = chain && pos + 1 < len;
    return chain && pos < len;
}
__device__ static inline bool tb_wk_pending(const WorkloadParams& W, u64 k) {
    bool linked;
    const bool chained = tb_wk_chained(W, k, &linked);
    return !tb_wk_post_void(W, k, chained) && tb_range(tb_rand(W.seed, k, 12), 1000) < WK_PENDING_PERMILLE;
}

__global__ void tb_gen_accounts(u8* out, u64 first, u64 count, WorkloadParams W) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 idx = first + i;
    Account a = {};
    a.id = tb_wk_account_id(idx);
    a.ledger = 2;
    a.code = 1;
    if (tb_wk_limited(W, idx)) a.flags = AF_DEBITS_MUST_NOT_EXCEED_CREDITS;
    *(Account*)(out + i * 128) = a;
}

__global__ void tb_gen_transfers(u8* out, u64 count, WorkloadParams W) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 k = W.first_index + i;
    const u64 n = W.account_count;
    u64 dr, cr;
    if (W.kind == WK_ZIPF_LIMITS) {
        dr = tb_zipf(W, k, 1);
        cr = tb_zipf(W, k, 2);
    } else {
        dr = tb_range(tb_rand(W.seed, k, 1), n);
        cr = tb_range(tb_rand(W.seed, k, 2), n);
    }
    if (dr == cr) cr = (cr + 1) % n;
    Transfer t = {};
    t.id = tb_wk_transfer_id(k);
    t.debit_account_id = tb_wk_account_id(dr);
    t.credit_account_id = tb_wk_account_id(cr);
    t.user_data_128 = tb_u128(tb_rand(W.seed, k, 3), tb_rand(W.seed, k, 4));
    t.user_data_64 = tb_rand(W.seed, k, 5);
    t.user_data_32 = (u32)tb_rand(W.seed, k, 6);
    t.ledger = 2;
    const u32 code = (u32)(tb_rand(W.seed, k, 7) & 0xFFFF) + 1;
    t.code = (u16)(code > 0xFFFF ? 0xFFFF : code);
    t.amount = (u128)tb_wk_amount(W, k);

    if (W.kind == WK_ZIPF_LIMITS && k < n && tb_wk_limited(W, k)) {
        // Pre-funding: created accounts have zero balances (:751-754), so the bank credits each
        // limit account first.
        t.debit_account_id = tb_wk_account_id(0);
        t.credit_account_id = tb_wk_account_id(k);
        t.amount = WK_FUND_AMOUNT;
    } else if (W.kind == WK_TWO_PHASE) {
        bool linked;
        const bool chained = tb_wk_chained(W, k, &linked);
        if (tb_wk_post_void(W, k, chained)) {
            // Post or void an earlier transfer: half within the last prepare (same pass), half up to
            // 2M events back (earlier passes, across expiry gaps).  The target may not be pending
            // (-> pending_transfer_not_pending) or may already be posted/voided (-> already_*).
            const u64 near = tb_rand(W.seed, k, 13);
            const u64 back = 1 + ((near & 1) ? tb_range(near, 8190) : tb_range(near, 2000000));
            if (back <= k) {
                const u64 j = k - back;
                const u64 r = tb_rand(W.seed, k, 14);
                t.pending_id = tb_wk_transfer_id(j);
                t.debit_account_id = 0;
                t.credit_account_id = 0;
                t.ledger = 0;
                t.code = 0;
                if (tb_range(r, 3) < 2) {
                    t.flags = TF_POST;
                    const u64 pa = tb_wk_amount(W, j);
                    t.amount = (r >> 40) & 1 ? (u128)(pa / 2 + 1) : (u128)0;  // partial or full
                } else {
                    t.flags = TF_VOID;
                    t.amount = 0;
                }
                if (!tb_wk_pending(W, j) && ((r >> 41) & 1)) t.user_data_64 = 0;  // vary exists checks
            }
        } else {
            if (linked) t.flags |= TF_LINKED;
            if (chained && tb_range(tb_rand(W.seed, k, 15), 1000) < WK_CHAIN_INVALID_PERMILLE) t.ledger = 0;
            if (tb_wk_pending(W, k)) {
                t.flags |= TF_PENDING;
                const u64 r = tb_rand(W.seed, k, 16);
                t.timeout = (r & 1) ? (u32)(1 + tb_range(r, 10)) : 0;
            } else {
                const u64 r = tb_rand(W.seed, k, 18);
                if (tb_range(r, 1000) < WK_BALANCING_PERMILLE) {
                    t.flags |= (r >> 40) & 1 ? TF_BAL_DEBIT : TF_BAL_CREDIT;
                    if ((r >> 41) & 1) t.amount = 0;  // balance as much as possible
                }
            }
        }
    }
    *(Transfer*)(out + i * 128) = t;
}

// ---- the memory-access mix of tb_transfers_validate (bench only) ---------------------------------
// tbgpu_bench_access_mix: the accesses kernel 1 makes per transfer, without its logic, on scratch
// buffers sized like the engine's tables — what the hardware does for this pattern is the kernel's
// practical bound.  STREAM: the 128-B event in, the 128-B record and 26 B of
// per-event results out (info, flags, dr, cr, rs, amount low word); PROBE: two random 32-B rows of an account-table-sized array; CAS: one
// random 8-B CAS into an index-sized array.
enum : u32 { MIX_STREAM = 1, MIX_PROBE = 2, MIX_CAS = 4 };
struct MixArgs {
    const uint4* events;
    uint4* records;
    u32* s4;             // 4 arrays of n u32 (info, dr, cr, rs)
    unsigned short* s2;  // flags
    u64* s8;             // n u64 (amount low word)
    const uint4* rows;   // 32-B rows
    u64 row_mask;
    u64* index;
    u64 index_mask;
    u64 n;
    u64* sink;
};

template <u32 M>
__global__ __launch_bounds__(256) void tb_access_mix(MixArgs A) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.n) return;
    u64 acc = 0;
    uint4 ev[8];
    const u64 h = tb_mix64(i * 0x9e3779b97f4a7c15ULL + 7);
    if (M & MIX_STREAM) {
#pragma unroll
        for (int w = 0; w < 8; w++) ev[w] = A.events[8 * i + w];
        acc ^= ev[0].x ^ ev[7].w;
    }
    if (M & MIX_PROBE) {
        const u64 d = tb_mix64(h ^ 1) & A.row_mask, c = tb_mix64(h ^ 2) & A.row_mask;
        const uint4 a0 = A.rows[2 * d], a1 = A.rows[2 * d + 1];
        const uint4 b0 = A.rows[2 * c], b1 = A.rows[2 * c + 1];
        acc ^= a0.x ^ a1.w ^ b0.y ^ b1.z ^ (d + c);
    }
    if (M & MIX_CAS) acc ^= atomicCAS((unsigned long long*)(A.index + (h & A.index_mask)), 0ULL, i + 1);
    if (M & MIX_STREAM) {
#pragma unroll
        for (int w = 0; w < 8; w++) A.records[8 * i + w] = ev[w];
        A.s4[i] = (u32)acc;
        A.s4[A.n + i] = (u32)h;
        A.s4[2 * A.n + i] = (u32)(h >> 8);
        A.s4[3 * A.n + i] = (u32)(h >> 16);
        A.s2[i] = (unsigned short)h;
        A.s8[i] = h ^ acc;
    } else if (acc == 0x123456789ULL) {
        A.sink[0] = acc;
    }
}
