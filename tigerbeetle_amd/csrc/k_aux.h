// k_aux.h — lookups (execute_lookup_accounts / _transfers, state_machine.zig:700-736), parity
// export, and the table-test `setup` action (state_machine.zig:1398-1407).
#pragma once

#include "tb_device.h"

// One id per lane; found records are written at out[i] and found[i] = 1.  The host keeps input
// order and skips not-found ids, exactly like the reference.
template <bool ACCOUNTS>
__global__ void tb_lookup(Tables T, const u64* ids, u32 n, u8* out, u8* found) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 lo = ids[2 * i], hi = ids[2 * i + 1];
    u32 slot;
    if (ACCOUNTS) slot = tb_account_find(T, lo, hi);
    else slot = tb_transfer_find(T, lo, hi);
    found[i] = slot != TB_NOT_FOUND;
    if (slot != TB_NOT_FOUND) {
        const uint4* src = ACCOUNTS ? (const uint4*)&T.accounts[slot] : (const uint4*)&T.transfers[slot];
        uint4* dst = (uint4*)(out + (u64)i * 128);
#pragma unroll
        for (int k = 0; k < 8; k++) dst[k] = src[k];
    }
}

// Compact every live record (timestamp != 0, id != 0) into out (order unspecified; the host
// sorts by id).  For transfers, also emit the posted groove as {pending timestamp, fulfillment}.
template <bool ACCOUNTS>
__global__ void tb_export(Tables T, u64 cap_slots, u8* out, u64* count, u64* posted_out, u64* posted_count) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap_slots) return;
    const u8* rec = ACCOUNTS ? (const u8*)&T.accounts[i] : (const u8*)&T.transfers[i];
    const u64 ts = *(const u64*)(rec + 120);
    const u64* idw = (const u64*)rec;
    if (ts == 0 || (idw[0] == 0 && idw[1] == 0) || (idw[0] == ~0ULL && idw[1] == ~0ULL)) return;
    const u64 k = atomicAdd((unsigned long long*)count, 1ULL);
    uint4* dst = (uint4*)(out + k * 128);
#pragma unroll
    for (int w = 0; w < 8; w++) dst[w] = ((const uint4*)rec)[w];
    if (!ACCOUNTS && T.posted[i] != POSTED_NONE) {
        const u64 q = atomicAdd((unsigned long long*)posted_count, 1ULL);
        posted_out[2 * q] = ts;
        posted_out[2 * q + 1] = T.posted[i] == POSTED_POSTED ? 0 : 1;
    }
}

// setup: overwrite the four balances of an existing account; keep `bound` an upper bound of
// every account's dp+dpost and cp+cpost (saturating).
__global__ void tb_set_balances(Tables T, u64 lo, u64 hi, u64 dp_lo, u64 dp_hi, u64 dpo_lo, u64 dpo_hi,
                                u64 cp_lo, u64 cp_hi, u64 cpo_lo, u64 cpo_hi, u32* status) {
    const u32 slot = tb_account_find(T, lo, hi);
    if (slot == TB_NOT_FOUND) {
        *status = 1;
        return;
    }
    Account* a = &T.accounts[slot];
    a->debits_pending = tb_u128(dp_lo, dp_hi);
    a->debits_posted = tb_u128(dpo_lo, dpo_hi);
    a->credits_pending = tb_u128(cp_lo, cp_hi);
    a->credits_posted = tb_u128(cpo_lo, cpo_hi);
    const u128 d = tb_sat_add(a->debits_pending, a->debits_posted);
    const u128 c = tb_sat_add(a->credits_pending, a->credits_posted);
    u128 bound = tb_u128(T.g->bound_lo, T.g->bound_hi);
    if (d > bound) bound = d;
    if (c > bound) bound = c;
    T.g->bound_lo = tb_lo(bound);
    T.g->bound_hi = tb_hi(bound);
    *status = 0;
}

// Bench reset between steps: zero every live account's balances, drop the transfer count and the
// balance bound (the transfer table itself is cleared with a memset).
__global__ void tb_zero_balances(Tables T, u64 cap) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        T.g->transfer_count = 0;
        T.g->bound_lo = 0;
        T.g->bound_hi = 0;
    }
    if (i >= cap) return;
    Account* a = &T.accounts[i];
    if (a->timestamp == 0) return;
    a->debits_pending = 0;
    a->debits_posted = 0;
    a->credits_pending = 0;
    a->credits_posted = 0;
}
