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
    u32 kind;             // 0 uniform (C2), 1 zipf (C3)
    u32 limit_permille;   // C3: permille of accounts with debits_must_not_exceed_credits
    double zipf_s;
};

__global__ void tb_gen_accounts(u8* out, u64 first, u64 count, WorkloadParams W) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 idx = first + i;
    Account a = {};
    a.id = TB_U128_MAX - (u128)(idx + 1);
    a.ledger = 2;
    a.code = 1;
    if (W.limit_permille && tb_range(tb_rand(W.seed, idx, 17), 1000) < W.limit_permille) {
        a.flags = AF_DEBITS_MUST_NOT_EXCEED_CREDITS;
    }
    *(Account*)(out + i * 128) = a;
}

__global__ void tb_gen_transfers(u8* out, u64 count, WorkloadParams W) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const u64 k = W.first_index + i;
    const u64 n = W.account_count;
    u64 dr = tb_range(tb_rand(W.seed, k, 1), n);
    u64 cr = tb_range(tb_rand(W.seed, k, 2), n);
    if (dr == cr) cr = (cr + 1) % n;
    Transfer t = {};
    t.id = TB_U128_MAX - (u128)(k + 1);
    t.debit_account_id = TB_U128_MAX - (u128)(dr + 1);
    t.credit_account_id = TB_U128_MAX - (u128)(cr + 1);
    t.user_data_128 = tb_u128(tb_rand(W.seed, k, 3), tb_rand(W.seed, k, 4));
    t.user_data_64 = tb_rand(W.seed, k, 5);
    t.user_data_32 = (u32)tb_rand(W.seed, k, 6);
    t.ledger = 2;
    const u32 code = (u32)(tb_rand(W.seed, k, 7) & 0xFFFF) + 1;
    t.code = (u16)(code > 0xFFFF ? 0xFFFF : code);
    // Exp(mean 10 000) +| 1 (benchmark.zig:309): u in (0, 1].
    const double u = ((double)(tb_rand(W.seed, k, 8) >> 11) + 1.0) * (1.0 / 9007199254740992.0);
    const u64 e = (u64)(-log(u) * 10000.0);
    t.amount = (u128)(e + 1);
    *(Transfer*)(out + i * 128) = t;
}
