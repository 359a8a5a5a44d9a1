// k_resolve.h — kernel 2 of a pass: one 1024-thread workgroup per prepare (batch).
//
//  a. classify: an event is DEPENDENT when its intrinsic result (kernel 1, pre-pass state) may
//     differ from the sequential result: its id / pending id collides with another event of the
//     pass; or it would change or read the balance of a constrained account (limit flags
//     tigerbeetle.zig:31-39, a balancing event's account :826-846, or an account whose balances
//     could overflow u128 this pass — the certificate below); or it is a balancing event.
//  b. linked chains (execute, state_machine.zig:628-692): a chain with a dependent member is
//     dependent as a whole; an independent chain resolves from its first failing member: that
//     member keeps its result, every other member becomes linked_event_failed (the last event of
//     the batch keeps linked_event_chain_open).
//  c. apply: independent ok events are inserted into the HBM transfer/account table and their
//     balance deltas added with exact u128 atomics (sums commute, so the order does not matter).
//  d. replies: non-ok results of a batch with no dependent event, ascending index (the reference's
//     FIFO back-fill of linked_event_failed also yields ascending order).  Batches with dependent
//     events are answered by the replay kernel.
//
// Overflow certificate: with S = Σ of every potential debit/credit increment of the pass and
// `bound` >= dp+dpost, cp+cpost of every account, no overflow check of create_transfer
// (:848-861) can fire in this pass if bound + S fits in u128.  Otherwise each account is checked
// individually (its own sums + S).
#pragma once

#include "k_validate.h"

// Ordered compaction helper: position of this thread's element among the true predicates of the
// block (ascending threadIdx), and the block total.  Every thread of the block must call it.
__device__ static inline u32 tb_block_rank(bool pred, u32* s_wave, u32& total) {
    const u64 m = __ballot(pred);
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    const u32 before = __popcll(m & ((1ULL << lane) - 1));
    if (lane == 0) s_wave[wave] = __popcll(m);
    __syncthreads();
    u32 wb = 0, tot = 0;
    for (u32 k = 0; k < nwaves; k++) {
        const u32 c = s_wave[k];
        wb += (k < wave) ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return wb + before;
}

__device__ static inline bool tb_account_cert_fails(const AccountBal& a, u128 S) {
    if (S == TB_U128_MAX) return true;  // saturated: the true S is unknown (tb_pass_cert)
    u128 d, c, r;
    if (tb_add_overflows(a.debits_pending, a.debits_posted, &d)) return true;
    if (tb_add_overflows(a.credits_pending, a.credits_posted, &c)) return true;
    if (tb_add_overflows(d, S, &r)) return true;
    if (tb_add_overflows(c, S, &r)) return true;
    return false;
}

// Write the sparse reply of batch b from LDS codes.
// n_fail: the number of non-ok codes (0: the reply is empty, no compaction needed).
__device__ static inline void tb_write_replies(const PassArgs& P, u32 b, u32 L, const u8* s_code, u32* s_wave,
                                               u32 n_fail = ~0u) {
    if (n_fail == 0 && !P.codes) {
        if (threadIdx.x == 0) P.reply_bytes[b] = 0;
        return;
    }
    if (P.codes) {  // routed mode: dense per-event codes, the router compacts them per prepare
        u8* dst = P.codes + P.batch_off[b];
        for (u32 i = threadIdx.x; i < L; i += blockDim.x) dst[i] = s_code[i];
        return;
    }
    u32* out = P.results + 2 * P.batch_off[b];
    u32 running = 0;
    for (u32 c = 0; c < L; c += blockDim.x) {
        const u32 i = c + threadIdx.x;
        const u32 code = i < L ? s_code[i] : R_OK;
        u32 total;
        const u32 r = tb_block_rank(code != R_OK, s_wave, total);
        if (code != R_OK) {
            out[2 * (running + r)] = i;
            out[2 * (running + r) + 1] = code;
        }
        running += total;
    }
    if (threadIdx.x == 0) P.reply_bytes[b] = running * 8;
}

// Apply the balance effects of one independent ok transfer whose record kernel 1 already wrote
// (create_transfer :870-880, post_or_void :987-1010).  With the 64-bit certificate (no balance
// can reach 2^64 this pass) the adds are fire-and-forget low-word atomics.
__device__ static inline void tb_apply_transfer(const PassArgs& P, u32 pe, u32 info, u16 flags, bool cert64) {
    const Tables& T = P.T;
    const u32 dr = P.dr[pe], cr = P.cr[pe];
    const u128 amount = tb_u128(P.amt[pe], (info & HZ_AMT_HI) ? P.amt_hi[pe] : 0ULL);
    if (info & HZ_POSTVOID) {
        const u32 pslot = P.ps[pe];
        const u128 pamount = T.xlog[pslot].amount;
        T.xposted[pslot] = (flags & TF_POST) ? POSTED_POSTED : POSTED_VOIDED;
        const u128 neg = (u128)0 - pamount;  // dp -= p.amount (mod 2^128, exact in aggregate)
        tb_bal_add(T.bal, dr, BAL_DP, neg);
        tb_bal_add(T.bal, cr, BAL_CP, neg);
        if (flags & TF_POST) {
            tb_bal_add(T.bal, dr, BAL_DPOST, amount);
            tb_bal_add(T.bal, cr, BAL_CPOST, amount);
        }
        return;
    }
    const u32 fd = (flags & TF_PENDING) ? BAL_DP : BAL_DPOST;
    const u32 fc = (flags & TF_PENDING) ? BAL_CP : BAL_CPOST;
    if (cert64) {
        tb_bal_add_lo(T.bal, dr, fd, tb_lo(amount));
        tb_bal_add_lo(T.bal, cr, fc, tb_lo(amount));
    } else {
        tb_bal_add(T.bal, dr, fd, amount);
        tb_bal_add(T.bal, cr, fc, amount);
    }
}

// Legs of this workgroup's prepare (see k_apply.h): s_hist holds the legs per bucket.  Publish the
// bucket starts (exclusive scan) as the prepare's leg_off row, then write every leg of an
// independent ok create_transfer into the prepare's leg region [2*pbase, 2*pbase + 2L), grouped by
// bucket: debit side into debits_pending / debits_posted, credit side into credits_pending /
// credits_posted (:870-880).  The order inside a bucket is unspecified: the sums commute.
// A leg word never leaves the registers of the thread that classified its event until it is stored
// in bucket order: each leg takes its sorted position from its bucket's LDS cursor (the counting
// sort), and the words go out through an LDS window of LEG_WIN words (the dead s_key array), each
// window stored coalesced.  (Round 5 wrote the words in event order to a global array and gathered
// them back through a 2-B LDS permutation: 32 B of traffic per transfer more.)
// Per-bucket leg counter of a prepare: 16 bits each, two per LDS word (a prepare has at most
// 16382 legs), so 4096 buckets fit in 8 KB.  Returns the counter's previous value.
__device__ static inline u32 tb_hist16_inc(u32* s_hist, u32 bucket) {
    const u32 sh = 16 * (bucket & 1);
    return (atomicAdd(&s_hist[bucket >> 1], 1u << sh) >> sh) & 0xFFFF;
}

#define RESOLVE_K (BATCH_LDS / RESOLVE_THREADS)  // events per thread of a prepare
#define LEG_WIN (BATCH_LDS / 2)                  // u64 words of the store window (s_key's 32 KB)

__device__ static inline u64 tb_leg_word(u32 slot, u32 leg_shift, u32 side, bool pending, u64 amount) {
    const u32 mask = (1u << leg_shift) - 1;
    return ((((u64)(slot & mask) << 2) | (side << 1) | (pending ? 0u : 1u)) << LEG_AMT_BITS) | amount;
}

// r_amt null: the legs' amounts are loaded again from the prepare's scratch row once the positions
// are known (tb_resolve_lean: its 64 VGPRs hold no amounts through the classification; the row was
// just read by this workgroup).
__device__ static inline void tb_emit_legs(const PassArgs& P, u32 pbase, u32 legmask, u32 pendmask, const u32* r_dr,
                                           const u32* r_cr, const u64* r_amt, u32* s_hist, u64* s_win, u32* s_wave) {
    if (TB_ABL(P, ABL_LEG_WORK)) return;
    __syncthreads();  // every count is in
    tb_block_scan_lds((u16*)s_hist, P.leg_buckets, s_wave);
    const u16* h = (const u16*)s_hist;
    const u32 nlegs = h[P.leg_buckets];
    u32* row = P.leg_off + (u64)blockIdx.x * (P.leg_buckets + 1);
    for (u32 k = threadIdx.x; k <= P.leg_buckets; k += blockDim.x) {
        row[k] = h[k];
        // The pass's legs per bucket: tb_apply_legs splits a Zipf-heavy bucket over workgroups.
        if (k < P.leg_buckets && h[k + 1] != h[k]) {
            const u32 add = h[k + 1] - h[k];
            const u32 was = atomicAdd(&P.leg_tot[k], add);
            if (was < LEG_SPLIT_MIN && was + add >= LEG_SPLIT_MIN) atomicAdd(&P.leg_tot[P.leg_buckets], 1u);
        }
    }
    __syncthreads();  // the row is read before the starts advance as cursors
    u32 r_pos[RESOLVE_K];  // sorted positions: debit leg in the low half, credit leg in the high half
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        r_pos[k] = 0;
        if (!((legmask >> k) & 1)) continue;
        r_pos[k] = tb_hist16_inc(s_hist, r_dr[k] >> P.leg_shift) | (tb_hist16_inc(s_hist, r_cr[k] >> P.leg_shift) << 16);
    }
    if (TB_ABL(P, ABL_LEG_STORES)) return;
    u64* __restrict__ w = P.leg_w + 2ULL * pbase;
    // The amounts, all loaded together (one round trip) once the classification's registers are free.
    u64 amt[RESOLVE_K];
    const u64* __restrict__ amt_b = P.amt + pbase;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        amt[k] = r_amt ? r_amt[k] : ((legmask >> k) & 1) ? amt_b[k * RESOLVE_THREADS + threadIdx.x] : 0ULL;
    }
    for (u32 w0 = 0; w0 < nlegs; w0 += LEG_WIN) {
        __syncthreads();  // the window is free (the previous one stored; before the first: s_key is dead)
#pragma unroll
        for (u32 k = 0; k < RESOLVE_K; k++) {
            if (!((legmask >> k) & 1)) continue;
            const bool pend = (pendmask >> k) & 1;
            const u32 pd = (r_pos[k] & 0xFFFF) - w0, pc = (r_pos[k] >> 16) - w0;
            if (pd < LEG_WIN) s_win[pd] = tb_leg_word(r_dr[k], P.leg_shift, 0, pend, amt[k]);
            if (pc < LEG_WIN) s_win[pc] = tb_leg_word(r_cr[k], P.leg_shift, 1, pend, amt[k]);
        }
        __syncthreads();
        const u32 m = min((u32)LEG_WIN, nlegs - w0);
        for (u32 j = threadIdx.x; j < m; j += blockDim.x) w[w0 + j] = s_win[j];
    }
}

// In-place pass: an independent ok post / void's record is composed here over its event (kernel 1
// did not write it, so the ordered path could still read the event as given).  A create's record is
// its event, stamped by kernel 1 (HZ_INPLACE).
__device__ static inline void tb_inplace_record(const PassArgs& P, u32 pe, u32 info, u64 ts) {
    if (!(info & HZ_POSTVOID)) return;
    Transfer* rec = &P.T.xlog[P.log_base + pe];
    const Transfer t = *rec;
    *rec = tb_compose_post_void(t, P.T.xlog[P.ps[pe]], ts);
}

// Apply one independent ok account (create_account :762, groove insert).
__device__ static inline void tb_apply_account(const PassArgs& P, u32 pe, u64 ts) {
    Account a = *(const Account*)(P.events + (P.e0 + pe) * 128);
    a.timestamp = ts;
    const u32 slot = tb_account_claim(P.T, tb_lo(a.id), tb_hi(a.id), ts);
    if (slot == TB_NOT_FOUND) return;
    tb_account_store_new(P.T, slot, a);
}

// Is an event dependent (see the header)?  Kernel 1's intrinsic result `code` is trusted otherwise.
template <u8 OP>
__device__ static inline bool tb_classify(const PassArgs& P, u32 pe, u32 info, u32 code, u128 S, bool cert_global,
                                          bool any_dup, bool any_bal, bool any_pv) {
    const Tables& T = P.T;
    if (OP == OP_CREATE_ACCOUNTS) {
        return any_dup && (info & HZ_KEYS) && tb_dedup_is_dup(P.dedup, P.dedup_mask, P.kid[pe]);
    }
    if (info & HZ_SELFDEP) return true;
    // The independent apply of a post / void trusts pending balances to cover its pending transfer
    // (true of every state a commit sequence builds); after a direct balance write the ordered
    // replay checks the reference's `-=` asserts instead (state_machine.zig:991-992).
    if (P.seq_pv && (P.eflags[pe] & (TF_POST | TF_VOID))) return true;
    if (any_dup) {
        if ((info & HZ_SPEC) && T.xdup[P.rs[pe]]) return true;
        if ((info & HZ_PV_KEY) && tb_dedup_is_dup(P.dedup, P.dedup_mask, P.kpid[pe])) return true;
    }
    if (any_pv) {
        // Some post/void of this pass names a pending id: an event whose id is one of them, or a
        // post/void whose pending transfer was created in this pass, is dependent.
        // The id's dedup key, for an event that reached the id check (kernel 1 set HZ_ACCTS or
        // HZ_PV_KEY right before it), recomputed from the event.
        if (info & (HZ_ACCTS | HZ_PV_KEY)) {
            const Transfer* ev = (const Transfer*)(P.events + (P.e0 + pe) * 128);
            const u64 kid = tb_dedup_key(tb_lo(ev->id), tb_hi(ev->id));
            if (tb_dedup_is_dup_or_present(P.dedup, P.dedup_mask, kid)) return true;
        }
        if (info & HZ_PV_KEY) {
            const Transfer* ev = (const Transfer*)(P.events + (P.e0 + pe) * 128);
            if (tb_transfer_claimed_in_pass(T, tb_lo(ev->pending_id), tb_hi(ev->pending_id), P.log_base)) return true;
        }
    }
    if ((info & HZ_ACCTS) && (code == R_OK || code == CT_OVERFLOWS_TIMEOUT)) {
        const u32 drs = P.dr[pe], crs = P.cr[pe];
        if (code == R_OK) {
            if (info & (HZ_BAL | HZ_LIMIT)) return true;
            if (any_bal && (T.account_mark[drs] == P.epoch || T.account_mark[crs] == P.epoch)) return true;
        }
        if (!cert_global && (tb_account_cert_fails(tb_bal_load(T.bal, drs), S) || tb_account_cert_fails(tb_bal_load(T.bal, crs), S))) {
            return true;
        }
    }
    return false;
}

template <u8 OP>
__global__ __launch_bounds__(RESOLVE_THREADS) void tb_resolve(PassArgs P) {
    __shared__ u8 s_code[BATCH_LDS];
    __shared__ u8 s_fl[BATCH_LDS];   // bit0 linked, bit1 dependent
    __shared__ u16 s_seg[BATCH_LDS]; // segment (chain) start
    __shared__ __attribute__((aligned(8))) u32 s_key[BATCH_LDS]; // per segment start: min over members (0 = dependent member)
    __shared__ u32 s_wave[RESOLVE_THREADS / 64];
    __shared__ u64 s_tsmax[RESOLVE_THREADS / 64];
    __shared__ u32 s_applied;
    __shared__ u32 s_failed;  // non-ok final results of independent events
    __shared__ u32 s_hist[OP == OP_CREATE_TRANSFERS ? LEG_BUCKETS_MAX / 2 + 1 : 1];  // legs per bucket (u16 pairs)

    if (P.resolve_slow && !P.resolve_slow[blockIdx.x]) return;  // tb_resolve_lean resolved this prepare
    const Tables& T = P.T;
    const u32 b = P.b0 + blockIdx.x;
    const u64 boff = P.batch_off[b];
    const u32 L = (u32)(P.batch_off[b + 1] - boff);
    const u32 pbase = (u32)(boff - P.e0);
    tb_kclock_start(P, 1);

    u128 S = 0;
    bool cert_global = true, cert64 = true;
    const bool any_dup = P.pass_words[PW_DUP] != 0;
    const bool any_bal = P.pass_words[PW_BAL] != 0;
    const bool any_pv = P.pass_words[PW_PV] != 0;
    if (OP == OP_CREATE_TRANSFERS) tb_pass_cert(P, S, cert_global, cert64);
    const bool use_legs = OP == OP_CREATE_TRANSFERS && P.legs && cert64;
    if (use_legs) {
        for (u32 k = threadIdx.x; k <= P.leg_buckets / 2; k += RESOLVE_THREADS) s_hist[k] = 0;
    }

    if (threadIdx.x == 0) {
        s_applied = 0;
        s_failed = 0;
    }
    // The prepare's first timestamp, loaded before any global store of this kernel: on gfx950 a
    // load waits for every earlier store of its wave to complete (vmcnt counts both), so a load
    // left between the per-event stores below would serialise them.
    const u64 ts0 = tb_ts_carried(P) ? 0 : P.batch_ts[b] - L + 1;
    // a. classify.  Each thread owns events tid + k*RESOLVE_THREADS; their scratch words are loaded
    // for every k before any is used (one memory round trip instead of one per k).  The event
    // flags the kernel needs are kept as bit masks over k (linked, pending): at 1024 threads a
    // workgroup, 64 VGPRs a lane is what lets two prepares share a CU (one round of workgroups
    // for a 512-prepare pass instead of two).
    u32 r_info[RESOLVE_K];
    u32 linkmask = 0, pendmask = 0;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        r_info[k] = i < L ? P.info[pbase + i] : 0u;
        const u16 fl = i < L ? P.eflags[pbase + i] : (u16)0;
        linkmask |= (fl & 1u) << k;
        pendmask |= ((fl & TF_PENDING) ? 1u : 0u) << k;
    }
    bool local_dep = false;
    const bool local_linked = linkmask != 0;
    // With every pass-wide condition of tb_classify off (uniform), what is left of it is a test of
    // the event's own bits, computed without branches (a 1024-thread workgroup's divergent branches
    // cost scalar instructions on its CU's one scalar unit).  Lanes past L hold info 0: not
    // dependent, not linked, and their LDS words (i < BATCH_LDS) are never read.
    const bool fast_cls = OP == OP_CREATE_TRANSFERS && !P.seq_pv && !any_dup && !any_pv && !any_bal && cert_global;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        if (!fast_cls && i >= L) continue;
        const u32 pe = pbase + i;
        const u32 info = r_info[k];
        const u32 code = info & 0xFF;
        const bool dep = fast_cls ? ((info & HZ_SELFDEP) != 0) |
                                        (((info & HZ_ACCTS) != 0) & (code == R_OK) & ((info & (HZ_BAL | HZ_LIMIT)) != 0))
                                  : tb_classify<OP>(P, pe, info, code, S, cert_global, any_dup, any_bal, any_pv);
        const bool linked = (linkmask >> k) & 1;
        local_dep |= dep;
        s_code[i] = (u8)code;
        s_fl[i] = (linked ? 1 : 0) | (dep ? 2 : 0);
        s_key[i] = 0xFFFFFFFFu;
    }
    const bool any_linked = __syncthreads_or(local_linked);
    // A chain is dependent only through a dependent member, so no classified dependent means none.
    const bool any_dep = __syncthreads_or(local_dep);

    // b. linked chains
    if (any_linked) {
        u32 carry = 0;
        for (u32 c = 0; c < L; c += RESOLVE_THREADS) {
            const u32 i = c + threadIdx.x;
            u32 v = 0;
            if (i < L) v = (i == 0 || !(s_fl[i - 1] & 1)) ? i : 0;
            const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
            for (u32 off = 1; off < 64; off <<= 1) {
                const u32 o = __shfl_up(v, off);
                if (lane >= off) v = max(v, o);
            }
            if (lane == 63) s_wave[wave] = v;
            __syncthreads();
            u32 prefix = carry;
            for (u32 k = 0; k < wave; k++) prefix = max(prefix, s_wave[k]);
            v = max(v, prefix);
            if (i < L) s_seg[i] = (u16)v;
            __syncthreads();
            carry = s_seg[min(c + RESOLVE_THREADS, L) - 1];
            __syncthreads();
        }
        for (u32 i = threadIdx.x; i < L; i += RESOLVE_THREADS) {
            const u32 s = s_seg[i];
            if (s_fl[s] & 1) {  // member of a chain
                const u32 key = (s_fl[i] & 2) ? 0u : (s_code[i] != R_OK ? i + 1 : 0xFFFFFFFFu);
                if (key != 0xFFFFFFFFu) atomicMin(&s_key[s], key);
            }
        }
        __syncthreads();
    }

    // Final results, dependent list, apply.  The account slots and amounts of every event of the
    // thread are loaded up front as well (the amount's high word only as "non-zero": a leg needs
    // an amount below 2^LEG_AMT_BITS).
    u32 r_dr[RESOLVE_K], r_cr[RESOLVE_K];
    u64 r_amt[RESOLVE_K];
    u32 wide = 0;  // bit k: event k's amount has a non-zero high word
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        const bool want = OP == OP_CREATE_TRANSFERS && i < L && (r_info[k] & HZ_ACCTS);
        const u32 pe = pbase + i;
        r_dr[k] = want ? P.dr[pe] : 0u;
        r_cr[k] = want ? P.cr[pe] : 0u;
        r_amt[k] = want ? P.amt[pe] : 0ULL;
        wide |= (want && (r_info[k] & HZ_AMT_HI) ? 1u : 0u) << k;  // HZ_AMT_HI: the high word is non-zero
    }
    u32 ndep = 0, n_app = 0, n_fail = 0;  // per thread, summed per wave below (one LDS atomic per wave)
    u32 legmask = 0;  // bit k: this thread's event k contributes two legs
    u32 last_ok = ~0u;  // the thread's last event (largest i) that returned ok when evaluated
    // An independent ok transfer that is not a leg is applied by tb_apply_events after this kernel:
    // no balance changes while any workgroup classifies, so the per-account certificate checks read
    // the pre-pass balances and the classification is a function of the input alone.
    bool late = false;
    u32* dep_out = P.dep_list + pbase;
    // No chain and no dependent event (uniform): every final result is the intrinsic code, already
    // in s_code; the loop below without its chain and dependent cases, branch-light.  Only a late
    // event's info word is rewritten (tb_apply_events reads HZ_LATE; the code byte is unchanged).
    if (OP == OP_CREATE_TRANSFERS && !any_linked && !any_dep) {
        u32 panic = 0;
#pragma unroll
        for (u32 k = 0; k < RESOLVE_K; k++) {
            const u32 i = k * RESOLVE_THREADS + threadIdx.x;
            const bool valid = i < L;
            const u32 pe = pbase + i;
            const u32 info = r_info[k];
            const u32 code = info & 0xFF;
            const bool ok = valid & (code == R_OK);
            panic |= code == TB_CODE_PANIC;
            const bool leg = use_legs && !(info & HZ_POSTVOID) && !((wide >> k) & 1) && r_amt[k] <= LEG_AMT_MASK;
            if (ok && !leg) P.info[pe] = info | HZ_EVAL_OK | HZ_LATE;
            last_ok = ok ? i : last_ok;
            n_app += ok;
            n_fail += valid & !ok;
            if (ok && P.inplace && (info & HZ_POSTVOID)) {
                tb_inplace_record(P, pe, info, tb_ts_carried(P) ? tb_event_ts(P, b, boff, L, i) : ts0 + i);
            }
            if (ok) {
                if (leg) {
                    if (!TB_ABL(P, ABL_LEG_WORK)) {
                        tb_hist16_inc(s_hist, r_dr[k] >> P.leg_shift);
                        tb_hist16_inc(s_hist, r_cr[k] >> P.leg_shift);
                    }
                    legmask |= 1u << k;
                } else {
                    late = true;
                }
            } else if (valid && (info & HZ_SPEC)) {
                tb_xindex_tombstone(T, P.rs[pe]);  // a failed event's speculative record
            }
        }
        if (panic) tb_panic(T.g, PANIC_ASSERT);
    } else {
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        bool dep = false, eval_ok = false;
        u32 fin = R_OK;
        if (i < L) {
            const u32 code = s_code[i];
            dep = (s_fl[i] & 2) != 0;
            fin = code;
            const u32 s = any_linked ? s_seg[i] : i;
            if (any_linked && (s_fl[s] & 1)) {
                const u32 key = s_key[s];
                if (key == 0) {
                    dep = true;
                } else if (key == 0xFFFFFFFFu) {
                    fin = R_OK;
                    eval_ok = true;
                } else {
                    const u32 ff = key - 1;
                    if (i == ff) {
                        fin = code;
                    } else if (i < ff) {
                        fin = R_LINKED_EVENT_FAILED;
                        eval_ok = true;
                    } else {
                        fin = ((s_fl[i] & 1) && i == L - 1) ? R_LINKED_EVENT_CHAIN_OPEN : R_LINKED_EVENT_FAILED;
                    }
                }
            } else {
                eval_ok = code == R_OK;
            }
            const u32 pe = pbase + i;
            const u32 info = r_info[k];
            if (!dep) {
                if (fin == TB_CODE_PANIC) tb_panic(T.g, PANIC_ASSERT);
                s_code[i] = (u8)fin;
                const bool leg = OP == OP_CREATE_TRANSFERS && use_legs && !(info & HZ_POSTVOID) && !((wide >> k) & 1) &&
                                 r_amt[k] <= LEG_AMT_MASK;
                const bool late_ev = OP == OP_CREATE_TRANSFERS && fin == R_OK && !leg;
                P.info[pe] = (info & 0xFFFFFF00u) | fin | (eval_ok ? HZ_EVAL_OK : 0) | (late_ev ? HZ_LATE : 0);
                if (eval_ok) last_ok = i;  // increasing in i
                if (fin == R_OK) {
                    if (OP == OP_CREATE_TRANSFERS) {
                        if (P.inplace && (info & HZ_POSTVOID)) {
                            tb_inplace_record(P, pe, info, tb_ts_carried(P) ? tb_event_ts(P, b, boff, L, i) : ts0 + i);
                        }
                        if (leg) {
                            if (!TB_ABL(P, ABL_LEG_WORK)) {
                                tb_hist16_inc(s_hist, r_dr[k] >> P.leg_shift);
                                tb_hist16_inc(s_hist, r_cr[k] >> P.leg_shift);
                            }
                            legmask |= 1u << k;
                        } else {
                            late = true;
                        }
                    } else {
                        tb_apply_account(P, pe, tb_ts_carried(P) ? tb_event_ts(P, b, boff, L, i) : ts0 + i);
                    }
                    n_app++;
                } else {
                    n_fail++;
                }
            } else {
                P.info[pe] = info | HZ_DEP;
            }
            // Withdraw a speculative record whose event did not commit here (failed, rolled back,
            // or left to the ordered replay, which inserts it itself in order).
            if (OP == OP_CREATE_TRANSFERS && (info & HZ_SPEC) && (dep || fin != R_OK)) {
                tb_xindex_tombstone(T, P.rs[pe]);
            }
        }
        if (any_dep) {
            u32 total;
            const u32 r = tb_block_rank(dep, s_wave, total);
            if (dep) dep_out[ndep + r] = i;
            ndep += total;
        }
    }
    }

    if (P.legs && __ballot(late) && (threadIdx.x & 63) == 0) P.pass_words[PW_LATE] = 1;
    // commit_timestamp: max over events that returned ok when evaluated (:763, :882, :1012) — the
    // timestamps increase with the event index, so each thread's last such event holds its maximum.
    u64 m = last_ok == ~0u ? 0 : tb_ts_carried(P) ? tb_event_ts(P, b, boff, L, last_ok) : ts0 + last_ok;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        m = max(m, (u64)__shfl_xor((unsigned long long)m, off));
        n_app += __shfl_xor(n_app, off);
        n_fail += __shfl_xor(n_fail, off);
    }
    if ((threadIdx.x & 63) == 0) {
        s_tsmax[threadIdx.x >> 6] = m;
        if (n_app) atomicAdd(&s_applied, n_app);
        if (n_fail) atomicAdd(&s_failed, n_fail);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (blockIdx.x == 0) {  // the replay kernel's per-pass counters (k_flow.h), after every load
            for (u32 k = 0; k < FL_BAR_WORDS; k++) T.g->flow_bar[FL_BAR_STRIDE * k] = 0;
            if (P.flow_words) for (u32 k = 0; k < FLOW_WORDS; k++) P.flow_words[k] = 0;
        }
        u64 mm = 0;
        for (u32 k = 0; k < RESOLVE_THREADS / 64; k++) mm = max(mm, s_tsmax[k]);
        if (mm) atomicMax((unsigned long long*)&T.g->commit_timestamp, (unsigned long long)mm);
        if (s_applied) {
            atomicAdd((unsigned long long*)(OP == OP_CREATE_TRANSFERS ? &T.g->transfer_count : &T.g->account_count),
                      (unsigned long long)s_applied);
        }
        P.dep_count[blockIdx.x] = ndep;
        if (ndep) atomicAdd((unsigned long long*)&T.g->dependent_total, (unsigned long long)ndep);
    }
    if (use_legs) tb_emit_legs(P, pbase, legmask, pendmask, r_dr, r_cr, r_amt, s_hist, (u64*)s_key, s_wave);  // s_key is dead here
    if (ndep == 0) tb_write_replies(P, b, L, s_code, s_wave, s_failed);
    tb_kclock_end(P, 1);
}

// tb_resolve's common case on a legs pass, in a lean kernel: no pass-wide condition (no
// duplicate id, post / void or balancing event in the pass, the 64-bit certificate) and, in the
// prepare, no linked chain and no dependent event.  Every final result is then the intrinsic code,
// and what is left is the legs' counting sort, the commit timestamp and the sparse reply.  Holding
// only what that needs (64 VGPRs a lane: the info words, the slots and amounts, the legs' sorted
// positions) lets two 1024-thread workgroups share a CU, so a 512-prepare pass is one round of
// workgroups; tb_resolve needs 128 VGPRs (one workgroup a CU: two rounds).  A prepare outside the
// common case is flagged in P.resolve_slow and tb_resolve, launched after this kernel, resolves it
// whole (this kernel changed nothing for it); the others tb_resolve skips.
__global__ __launch_bounds__(RESOLVE_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void tb_resolve_lean(PassArgs P) {
    __shared__ u8 s_code[BATCH_LDS];
    __shared__ __attribute__((aligned(8))) u64 s_win[LEG_WIN];
    __shared__ u32 s_wave[RESOLVE_THREADS / 64];
    __shared__ u64 s_tsmax[RESOLVE_THREADS / 64];
    __shared__ u32 s_applied;
    __shared__ u32 s_failed;
    __shared__ u32 s_hist[LEG_BUCKETS_MAX / 2 + 1];

    const Tables& T = P.T;
    const u32 b = P.b0 + blockIdx.x;
    const u64 boff = P.batch_off[b];
    const u32 L = (u32)(P.batch_off[b + 1] - boff);
    const u32 pbase = (u32)(boff - P.e0);
    tb_kclock_start(P, 1);
    u128 S = 0;
    bool cert_global = true, cert64 = true;
    tb_pass_cert(P, S, cert_global, cert64);
    const bool lean = P.legs && !P.seq_pv && P.pass_words[PW_DUP] == 0 && P.pass_words[PW_PV] == 0 &&
                      P.pass_words[PW_BAL] == 0 && cert_global && cert64;
    if (!lean) {  // uniform: the whole pass goes to tb_resolve
        if (threadIdx.x == 0) P.resolve_slow[blockIdx.x] = 1;
        return;
    }
    for (u32 k = threadIdx.x; k <= P.leg_buckets / 2; k += RESOLVE_THREADS) s_hist[k] = 0;
    if (threadIdx.x == 0) {
        s_applied = 0;
        s_failed = 0;
    }
    const u64 ts0 = tb_ts_carried(P) ? 0 : P.batch_ts[b] - L + 1;
    // The prepare's scratch rows from workgroup-uniform bases: a lane's address is a 32-bit offset
    // from a scalar base (no 64-bit address per event held in VGPRs across the kernel).
    u32* __restrict__ info_b = P.info + pbase;
    const u16* __restrict__ fl_b = P.eflags + pbase;
    const u32* __restrict__ dr_b = P.dr + pbase;
    const u32* __restrict__ cr_b = P.cr + pbase;
    const u64* __restrict__ amt_b = P.amt + pbase;
    const u32* __restrict__ rs_b = P.rs + pbase;
    u32 r_info[RESOLVE_K];
    u32 linkmask = 0, pendmask = 0;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        r_info[k] = i < L ? info_b[i] : 0u;
        const u16 fl = i < L ? fl_b[i] : (u16)0;
        linkmask |= (fl & 1u) << k;
        pendmask |= ((fl & TF_PENDING) ? 1u : 0u) << k;
    }
    // Dependent events, and post / voids (an in-place one composes its record here: tb_resolve's), send
    // the prepare to tb_resolve.
    bool local_dep = false;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 info = r_info[k];
        local_dep |= ((info & (HZ_SELFDEP | HZ_POSTVOID)) != 0) |
                     (((info & HZ_ACCTS) != 0) & ((info & 0xFF) == R_OK) & ((info & (HZ_BAL | HZ_LIMIT)) != 0));
    }
    const bool any_linked = __syncthreads_or(linkmask != 0);
    const bool any_dep = __syncthreads_or(local_dep);
    if (any_linked || any_dep) {  // uniform
        if (threadIdx.x == 0) P.resolve_slow[blockIdx.x] = 1;
        return;
    }
    if (threadIdx.x == 0) P.resolve_slow[blockIdx.x] = 0;
    // The slots stay in registers until the legs are stored; an amount is needed here only against
    // LEG_AMT_MASK (tb_emit_legs loads it again from the row when it stores the word).
    u32 r_dr[RESOLVE_K], r_cr[RESOLVE_K];
    u32 wide = 0;  // bit k: event k's amount is not a leg amount (a non-zero high word, or >= 2^LEG_AMT_BITS)
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        const bool want = i < L && (r_info[k] & HZ_ACCTS);
        r_dr[k] = want ? dr_b[i] : 0u;
        r_cr[k] = want ? cr_b[i] : 0u;
        const u64 a = want ? amt_b[i] : 0ULL;
        wide |= (want && ((r_info[k] & HZ_AMT_HI) || a > LEG_AMT_MASK) ? 1u : 0u) << k;  // HZ_AMT_HI: high word non-zero
    }
    u32 n_app = 0, n_fail = 0, legmask = 0, last_ok = ~0u, panic = 0;
    bool late = false;
#pragma unroll
    for (u32 k = 0; k < RESOLVE_K; k++) {
        const u32 i = k * RESOLVE_THREADS + threadIdx.x;
        const bool valid = i < L;
        const u32 info = r_info[k];
        const u32 code = info & 0xFF;
        if (valid) s_code[i] = (u8)code;
        const bool ok = valid & (code == R_OK);
        panic |= code == TB_CODE_PANIC;
        const bool leg = !((wide >> k) & 1);
        if (ok && !leg) info_b[i] = info | HZ_EVAL_OK | HZ_LATE;
        last_ok = ok ? i : last_ok;
        n_app += ok;
        n_fail += valid & !ok;
        if (ok) {
            if (leg) {
                if (!TB_ABL(P, ABL_LEG_WORK)) {
                    tb_hist16_inc(s_hist, r_dr[k] >> P.leg_shift);
                    tb_hist16_inc(s_hist, r_cr[k] >> P.leg_shift);
                }
                legmask |= 1u << k;
            } else {
                late = true;
            }
        } else if (valid && (info & HZ_SPEC)) {
            tb_xindex_tombstone(T, rs_b[i]);  // a failed event's speculative record
        }
    }
    if (panic) tb_panic(T.g, PANIC_ASSERT);
    if (__ballot(late) && (threadIdx.x & 63) == 0) P.pass_words[PW_LATE] = 1;
    u64 m = last_ok == ~0u ? 0 : tb_ts_carried(P) ? tb_event_ts(P, b, boff, L, last_ok) : ts0 + last_ok;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        m = max(m, (u64)__shfl_xor((unsigned long long)m, off));
        n_app += __shfl_xor(n_app, off);
        n_fail += __shfl_xor(n_fail, off);
    }
    if ((threadIdx.x & 63) == 0) {
        s_tsmax[threadIdx.x >> 6] = m;
        if (n_app) atomicAdd(&s_applied, n_app);
        if (n_fail) atomicAdd(&s_failed, n_fail);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (blockIdx.x == 0) {  // the replay kernel's per-pass counters (k_flow.h), after every load
            for (u32 k = 0; k < FL_BAR_WORDS; k++) T.g->flow_bar[FL_BAR_STRIDE * k] = 0;
            if (P.flow_words) for (u32 k = 0; k < FLOW_WORDS; k++) P.flow_words[k] = 0;
        }
        u64 mm = 0;
        for (u32 k = 0; k < RESOLVE_THREADS / 64; k++) mm = max(mm, s_tsmax[k]);
        if (mm) atomicMax((unsigned long long*)&T.g->commit_timestamp, (unsigned long long)mm);
        if (s_applied) atomicAdd((unsigned long long*)&T.g->transfer_count, (unsigned long long)s_applied);
        P.dep_count[blockIdx.x] = 0;
    }
    tb_emit_legs(P, pbase, legmask, pendmask, r_dr, r_cr, (const u64*)nullptr, s_hist, s_win, s_wave);
    tb_write_replies(P, b, L, s_code, s_wave, s_failed);
    tb_kclock_end(P, 1);
}
