// k_aux.h — lookups (execute_lookup_accounts / _transfers, state_machine.zig:700-736), parity
// export, and the table-test `setup` action (state_machine.zig:1398-1407).
#pragma once

#include "pass.h"

// One id per lane; found records are written at out[i] and found[i] = 1.  The host keeps input
// order and skips not-found ids, exactly like the reference.
template <bool ACCOUNTS>
__global__ void tb_lookup(Tables T, const u64* ids, u32 n, u8* out, u8* found) {
    const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 lo = ids[2 * i], hi = ids[2 * i + 1];
    if (ACCOUNTS) {
        const u32 slot = tb_account_find(T, lo, hi);
        found[i] = slot != TB_NOT_FOUND;
        if (slot != TB_NOT_FOUND) *(Account*)(out + (u64)i * 128) = tb_account_load(T, slot);
    } else {
        const u32 pos = tb_transfer_find(T, lo, hi);
        found[i] = pos != TB_NOT_FOUND;
        if (pos != TB_NOT_FOUND) *(Transfer*)(out + (u64)i * 128) = T.xlog[pos];
    }
}

// Compact every live account (slots [0, cap)) into out; order unspecified (the host sorts by id).
__global__ void tb_export_accounts(Tables T, u64 first, u64 cap, u8* out, u64* count) {
    const u64 i = first + (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    const AccountHot& h = T.acct_hot[i];
    if (h.timestamp == 0 || tb_id_reserved(h.id_lo, h.id_hi)) return;
    const u64 k = atomicAdd((unsigned long long*)count, 1ULL);
    *(Account*)(out + k * 128) = tb_account_load(T, (u32)i);
}

// Compact every live transfer (index entries [first, first+n)); also the posted groove as
// {pending timestamp, fulfillment} pairs.
__global__ void tb_export_transfers(Tables T, u64 first, u64 n, u8* out, u64* count, u64* posted_out,
                                    u64* posted_count) {
    const u64 i = first + (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= first + n) return;
    const u64 e = T.xidx[i];
    if (e == 0 || (e & XI_TOMB)) return;
    const u32 pos = tb_xi_pos(e);
    const Transfer& t = T.xlog[pos];
    const u64 k = atomicAdd((unsigned long long*)count, 1ULL);
    *(Transfer*)(out + k * 128) = t;
    const u8 st = T.xposted[pos];
    if (st != POSTED_NONE) {
        const u64 q = atomicAdd((unsigned long long*)posted_count, 1ULL);
        posted_out[2 * q] = t.timestamp;
        posted_out[2 * q + 1] = st == POSTED_POSTED ? 0 : 1;
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
    AccountBal a;
    a.debits_pending = tb_u128(dp_lo, dp_hi);
    a.debits_posted = tb_u128(dpo_lo, dpo_hi);
    a.credits_pending = tb_u128(cp_lo, cp_hi);
    a.credits_posted = tb_u128(cpo_lo, cpo_hi);
    tb_bal_store(T.bal, slot, a);
    const u128 d = tb_sat_add(a.debits_pending, a.debits_posted);
    const u128 c = tb_sat_add(a.credits_pending, a.credits_posted);
    u128 bound = tb_u128(T.g->bound_lo, T.g->bound_hi);
    if (d > bound) bound = d;
    if (c > bound) bound = c;
    T.g->bound_lo = tb_lo(bound);
    T.g->bound_hi = tb_hi(bound);
    *status = 0;
}

// Bench reset between steps: zero every balance, drop the transfer count and the balance bound
// (the transfer index and posted groove are cleared with memsets).
__global__ void tb_zero_balances(Tables T, u64 cap) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        T.g->transfer_count = 0;
        T.g->bound_lo = 0;
        T.g->bound_hi = 0;
    }
    if (i >= cap) return;
    tb_bal_store(T.bal, i, AccountBal{0, 0, 0, 0});
}

// ---- groove write-back (StateMachine.checkpoint, state_machine.zig:542-582) --------------------
// The objects a durable replica must insert / upsert into its forest since the previous write-back:
// accounts created since (timestamp > ts0) or whose balances differ from the snapshot taken then,
// transfers created since, and the posted-groove entries their post / void records created.
// tb_delta_accounts is the whole-table diff, kept for the one case the host cannot name the changed
// accounts (create_accounts committed from device memory, tbgpu_commit_device_async, or more of them
// than the engine lists).  Counts past `cap` are still counted (the host retries with room).
__global__ void tb_delta_accounts(Tables T, BalView snap, u64 ts0, u64 first, u64 last, u8* out, u64 cap,
                                  u64* count, AccountBal* before, u32 world, u32 self) {
    const u64 i = first + (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= last) return;
    const AccountHot& h = T.acct_hot[i];
    if (h.timestamp == 0 || tb_id_reserved(h.id_lo, h.id_hi)) return;
    if (world > 1 && tb_home(h.id_lo, h.id_hi, world) != self) return;  // a node shard: its owned accounts
    const AccountBal b = tb_bal_load(T.bal, i), s = tb_bal_load(snap, i);
    const bool same = b.debits_pending == s.debits_pending && b.debits_posted == s.debits_posted &&
                      b.credits_pending == s.credits_pending && b.credits_posted == s.credits_posted;
    if (h.timestamp <= ts0 && same) return;
    const u64 k = atomicAdd((unsigned long long*)count, 1ULL);
    if (k < cap) {
        *(Account*)(out + k * 128) = tb_account_load(T, (u32)i);
        // The balances the forest holds for it (zero for an account created since): what a groove
        // upsert diffs the balance index trees against (src/lsm/groove.zig:925-963).
        if (before) before[k] = h.timestamp <= ts0 ? s : AccountBal{0, 0, 0, 0};
    }
}

// O(changes) write-back (tbgpu_checkpoint_delta): nothing scans a whole table.
// Transfers: the log positions written since the previous write-back, [pos0, log_end).  A record is
// new if the index holds it at that position (a withdrawn speculative record's entry is tombstoned;
// a re-inserted id points elsewhere) and it is younger than the previous write-back (records loaded
// from the forest after a restart are older).  Log order is timestamp order, and the compaction
// keeps it: a count pass (live records per workgroup), the host's exclusive prefix over the
// workgroups, then an ordered scatter.
#define DELTA_THREADS 256

__device__ static inline bool tb_delta_live(const Tables& T, u64 pos, u64 ts0) {
    const Transfer& t = T.xlog[pos];
    return t.timestamp > ts0 && tb_transfer_find(T, tb_lo(t.id), tb_hi(t.id)) == (u32)pos;
}

__global__ __launch_bounds__(DELTA_THREADS) void tb_delta_log_count(Tables T, u64 pos0, u64 n, u64 ts0, u32* block_counts) {
    __shared__ u32 s_wave[DELTA_THREADS / 64];
    const u64 i = (u64)blockIdx.x * DELTA_THREADS + threadIdx.x;
    const bool live = i < n && tb_delta_live(T, pos0 + i, ts0);
    const u64 m = __ballot(live);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 c = 0;
        for (u32 w = 0; w < DELTA_THREADS / 64; w++) c += s_wave[w];
        block_counts[blockIdx.x] = c;
    }
}

// The ordered scatter.  out (optional): the records; ids (optional): the debit and credit account
// ids of each (4 words); pv: the post / void records' {pending id lo, hi, voided}, unordered.
__global__ __launch_bounds__(DELTA_THREADS) void tb_delta_log_scatter(Tables T, u64 pos0, u64 n, u64 ts0, const u64* block_base,
                                                                      u8* out, u64* ids, u64* pv, u64* pv_count) {
    __shared__ u32 s_wave[DELTA_THREADS / 64];
    const u64 i = (u64)blockIdx.x * DELTA_THREADS + threadIdx.x;
    const bool live = i < n && tb_delta_live(T, pos0 + i, ts0);
    const u64 m = __ballot(live);
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) s_wave[wave] = __popcll(m);
    __syncthreads();
    if (!live) return;
    u64 k = block_base[blockIdx.x] + __popcll(m & ((1ULL << lane) - 1));
    for (u32 w = 0; w < wave; w++) k += s_wave[w];
    const Transfer& t = T.xlog[pos0 + i];
    if (out) *(Transfer*)(out + k * 128) = t;
    if (ids) {
        ids[4 * k] = tb_lo(t.debit_account_id);
        ids[4 * k + 1] = tb_hi(t.debit_account_id);
        ids[4 * k + 2] = tb_lo(t.credit_account_id);
        ids[4 * k + 3] = tb_hi(t.credit_account_id);
    }
    if (pv && (t.flags & (TF_POST | TF_VOID))) {
        const u64 q = atomicAdd((unsigned long long*)pv_count, 1ULL);
        pv[3 * q] = tb_lo(t.pending_id);
        pv[3 * q + 1] = tb_hi(t.pending_id);
        pv[3 * q + 2] = (t.flags & TF_POST) ? 0 : 1;
    }
}

// The ordered bases on the device (no host round trip): exclusive prefix of the per-workgroup
// counts of tb_delta_log_count, and the total.  One workgroup; each thread owns a run of counts.
__global__ __launch_bounds__(1024) void tb_delta_scan_blocks(const u32* counts, u64 nblocks, u64* base, u64* total) {
    __shared__ u32 s_wave[1024 / 64];
    const u64 per = (nblocks + 1023) / 1024;
    const u64 k0 = min(nblocks, (u64)threadIdx.x * per), k1 = min(nblocks, k0 + per);
    u32 local = 0;
    for (u64 k = k0; k < k1; k++) local += counts[k];
    u32 all;
    u64 run = tb_block_excl_sum(local, s_wave, &all);
    for (u64 k = k0; k < k1; k++) {
        base[k] = run;
        run += counts[k];
    }
    if (threadIdx.x == 0) *total = all;
}

// The posted-groove entry each new post / void record makes (state_machine.zig:987-995): {the
// pending transfer's timestamp, voided}.  A pending transfer that is missing is an invariant failure
// (status bit 0).
__global__ void tb_delta_posted(Tables T, const u64* pv, const u64* npv, u64* pairs, u64* status) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *npv) return;
    const u32 pos = tb_transfer_find(T, pv[3 * q], pv[3 * q + 1]);
    if (pos == TB_NOT_FOUND) {
        atomicOr((unsigned long long*)status, 1ULL);
        return;
    }
    pairs[2 * q] = T.xlog[pos].timestamp;
    pairs[2 * q + 1] = pv[3 * q + 2];
}

// Accounts: the ids the host names as possibly changed (the debit / credit accounts of the new
// transfers, the ids of create_accounts events and of direct balance writes since the previous
// write-back), each slot once (mark = this write-back's epoch).  Emitted when created since (timestamp
// > ts0) or when its balances differ from the snapshot; `slots` lists every slot seen, for the
// snapshot's advance.  n_dev (optional): the id count is 2 x *n_dev (the new transfers' two accounts,
// counted on the device), n is then only the grid's bound.
__global__ __launch_bounds__(256) void tb_delta_ids(Tables T, BalView snap, u64 ts0, const u64* ids, u64 n,
                                                    u32* mark, u32 epoch, u8* out, AccountBal* before, u64* count,
                                                    u32* slots, u64* slot_count, const u64* n_dev = nullptr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n && !(n_dev && i >= 2 * *n_dev);
    u32 slot = TB_NOT_FOUND;
    if (live) slot = tb_account_find(T, ids[2 * i], ids[2 * i + 1]);
    // The slot's words are read together with the epoch exchange (one round trip, not three: the
    // exchange decides only whether this copy of the id is the one that emits).
    u32 was = epoch;
    AccountHot h{};
    AccountBal b{}, sn{};
    AccountCold c{};
    if (slot != TB_NOT_FOUND) {
        was = atomicExch(&mark[slot], epoch);
        h = T.acct_hot[slot];
        b = tb_bal_load(T.bal, slot);
        sn = tb_bal_load(snap, slot);
        c = T.acct_cold[slot];
    }
    const bool first = was != epoch;  // the first copy of the id takes its slot
    const bool same = b.debits_pending == sn.debits_pending && b.debits_posted == sn.debits_posted &&
                      b.credits_pending == sn.credits_pending && b.credits_posted == sn.credits_posted;
    const bool emit = first && (h.timestamp > ts0 || !same);
    const u64 si = tb_wave_claim(first, slot_count);
    if (first) slots[si] = slot;
    const u64 k = tb_wave_claim(emit, count);
    if (emit) {
        Account a;
        a.id = tb_u128(h.id_lo, h.id_hi);
        a.debits_pending = b.debits_pending;
        a.debits_posted = b.debits_posted;
        a.credits_pending = b.credits_pending;
        a.credits_posted = b.credits_posted;
        a.user_data_128 = c.user_data_128;
        a.user_data_64 = c.user_data_64;
        a.user_data_32 = c.user_data_32;
        a.reserved = c.reserved;
        a.ledger = h.ledger;
        a.code = h.code;
        a.flags = h.flags;
        a.timestamp = h.timestamp;
        *(Account*)(out + k * 128) = a;
        before[k] = h.timestamp <= ts0 ? sn : AccountBal{0, 0, 0, 0};
    }
}

// The asynchronous write-back splits tb_delta_ids in two.  In stream order, right after the bar
// (tb_delta_capture): each id's slot, deduplicated by the epoch mark, and its balances as they are
// now — the only part of an account the next commits change.  Beside those commits, on the
// write-back stream (tb_delta_emit): the records (the hot and cold words of an existing account
// never change; a create of another account only fills an empty slot, off every existing probe
// chain), the snapshot comparison, the emission, then the snapshot's advance from the captured
// balances (tb_delta_advance_from).
__global__ __launch_bounds__(256) void tb_delta_capture(Tables T, const u64* ids, u64 n, u32* mark, u32 epoch,
                                                        u32* slots, AccountBal* cap, u64* slot_count,
                                                        const u64* n_dev = nullptr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n && !(n_dev && i >= 2 * *n_dev);
    u32 slot = TB_NOT_FOUND;
    if (live) slot = tb_account_find(T, ids[2 * i], ids[2 * i + 1]);
    u32 was = epoch;
    AccountBal b{};
    if (slot != TB_NOT_FOUND) {
        was = atomicExch(&mark[slot], epoch);
        b = tb_bal_load(T.bal, slot);
    }
    const bool first = was != epoch;
    const u64 si = tb_wave_claim(first, slot_count);
    if (first) {
        slots[si] = slot;
        cap[si] = b;
    }
}

// The same capture from the log range itself, without the gather's liveness check (so it needs
// nothing the gather computes): the debit and credit account of every record at [pos0, pos0 + n).  A
// record that did not commit (a failed or withdrawn event's position) only adds accounts whose
// balances did not change, which the emission drops (unless created since, which is listed anyway).
__global__ __launch_bounds__(256) void tb_delta_capture_log(Tables T, u64 pos0, u64 n, u32* mark, u32 epoch, u32* slots,
                                                            AccountBal* cap, u64* slot_count) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // one record: both accounts' chains together
    u32 ds = TB_NOT_FOUND, cs = TB_NOT_FOUND;
    if (i < n) {
        const u64* w = (const u64*)&T.xlog[pos0 + i];
        const u64 dlo = w[2], dhi = w[3], clo = w[4], chi = w[5];  // debit @16, credit @32
        if (!tb_id_reserved(dlo, dhi) && !tb_id_reserved(clo, chi)) {
            const u64 dpos = tb_hash_id(dlo, dhi) & T.account_mask, cpos = tb_hash_id(clo, chi) & T.account_mask;
            const AccountHot d0 = T.acct_hot[dpos], c0 = T.acct_hot[cpos];
            AccountHot dh, ch;
            tb_account_find2(T, dlo, dhi, dpos, d0, clo, chi, cpos, c0, &ds, &cs, &dh, &ch);
        } else {
            if (!tb_id_reserved(dlo, dhi)) ds = tb_account_find(T, dlo, dhi);
            if (!tb_id_reserved(clo, chi)) cs = tb_account_find(T, clo, chi);
        }
        if (cs == ds) cs = TB_NOT_FOUND;  // a garbage record naming one account twice
    }
    u32 dw = epoch, cw = epoch;
    AccountBal db{}, cb{};
    if (ds != TB_NOT_FOUND) {
        dw = atomicExch(&mark[ds], epoch);
        db = tb_bal_load(T.bal, ds);
    }
    if (cs != TB_NOT_FOUND) {
        cw = atomicExch(&mark[cs], epoch);
        cb = tb_bal_load(T.bal, cs);
    }
    const bool df = dw != epoch, cf = cw != epoch;
    const u64 dsi = tb_wave_claim(df, slot_count);
    if (df) {
        slots[dsi] = ds;
        cap[dsi] = db;
    }
    const u64 csi = tb_wave_claim(cf, slot_count);
    if (cf) {
        slots[csi] = cs;
        cap[csi] = cb;
    }
}

__global__ __launch_bounds__(256) void tb_delta_emit(Tables T, BalView snap, u64 ts0, const u32* slots,
                                                     const AccountBal* cap, const u64* slot_count, u8* out,
                                                     AccountBal* before, u64* count) {
    const u64 m = *slot_count;
    for (u64 i0 = (u64)blockIdx.x * blockDim.x; i0 < m; i0 += (u64)gridDim.x * blockDim.x) {
        const u64 i = i0 + threadIdx.x;
        const bool live = i < m;
        AccountHot h{};
        AccountCold c{};
        AccountBal b{}, sn{};
        if (live) {
            const u32 slot = slots[i];
            h = T.acct_hot[slot];
            c = T.acct_cold[slot];
            sn = tb_bal_load(snap, slot);
            b = cap[i];
        }
        const bool same = b.debits_pending == sn.debits_pending && b.debits_posted == sn.debits_posted &&
                          b.credits_pending == sn.credits_pending && b.credits_posted == sn.credits_posted;
        const bool emit = live && (h.timestamp > ts0 || !same);
        const u64 k = tb_wave_claim(emit, count);
        if (emit) {
            Account a;
            a.id = tb_u128(h.id_lo, h.id_hi);
            a.debits_pending = b.debits_pending;
            a.debits_posted = b.debits_posted;
            a.credits_pending = b.credits_pending;
            a.credits_posted = b.credits_posted;
            a.user_data_128 = c.user_data_128;
            a.user_data_64 = c.user_data_64;
            a.user_data_32 = c.user_data_32;
            a.reserved = c.reserved;
            a.ledger = h.ledger;
            a.code = h.code;
            a.flags = h.flags;
            a.timestamp = h.timestamp;
            *(Account*)(out + k * 128) = a;
            before[k] = h.timestamp <= ts0 ? sn : AccountBal{0, 0, 0, 0};
        }
    }
}

__global__ void tb_delta_advance_from(BalView snap, const u32* slots, const AccountBal* cap, const u64* n) {
    const u64 m = *n;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (u64)gridDim.x * blockDim.x) tb_bal_store(snap, slots[i], cap[i]);
}

// The snapshot follows the slots a write-back covered (*n of them), grid-stride.
__global__ void tb_delta_advance(Tables T, BalView snap, const u32* slots, const u64* n) {
    const u64 m = *n;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (u64)gridDim.x * blockDim.x) {
        tb_bal_store(snap, slots[i], tb_bal_load(T.bal, slots[i]));
    }
}

// Order of the gathered records (bit 0 of *order: a timestamp not above its predecessor's) and
// posted pairs (bit 1: a pair below its predecessor), grid-stride; the host sorts only when set,
// instead of reading every record back to find out (records appended by an upsert or a load may
// sit out of timestamp order in the log).
__device__ static inline void tb_delta_order_check(const u8* recs, u64 nt, const u64* pairs, u64 np, u64* order) {
    const u64 stride = (u64)gridDim.x * blockDim.x;
    bool unsorted_t = false, unsorted_p = false;
    for (u64 i = 1 + (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += stride) {
        const u64* t = (const u64*)(recs + i * 128 + 120);
        unsorted_t |= t[-16] >= t[0];  // the previous record's timestamp
    }
    for (u64 i = 1 + (u64)blockIdx.x * blockDim.x + threadIdx.x; pairs && i < np; i += stride) {
        const u64* q = pairs + 2 * i;
        unsorted_p |= q[-2] > q[0] || (q[-2] == q[0] && q[-1] > q[1]);
    }
    const u64 flags = (__ballot(unsorted_t) ? 1 : 0) | (__ballot(unsorted_p) ? 2 : 0);
    if ((threadIdx.x & 63) == 0 && flags) atomicOr((unsigned long long*)order, (unsigned long long)flags);
}

// The order check of a write-back's gathered records and pairs (one slice of them), on the engine
// stream after the gather.
__global__ __launch_bounds__(256) void tb_delta_order(const u8* recs, const u64* nt, const u64* pairs, const u64* np,
                                                      u64* order) {
    tb_delta_order_check(recs, *nt, pairs, *np, order);
}

// ---- pipelined host commits (tbgpu_commit_pipelined) -------------------------------------------
// After a chunk's passes: copy what the host needs straight into the slot's pinned reply arena
// (mapped host memory): the panic word and commit timestamp, every prepare's reply size and the
// non-empty replies.  Only bytes that exist cross PCIe (4 B per prepare for an all-ok chunk); the
// host reads the arena once the chunk's `done` event fired.  One workgroup per prepare.
// seq != 0 (a one-prepare call, one workgroup): after everything else, seq is written to the word
// at `done` with system scope, so the host can spin on it instead of waiting for the stream.
__global__ __launch_bounds__(64) void tb_reply_out(const u64* batch_off, u32 nb, const u32* reply_bytes,
                                                   const u32* results, const Globals* g, u8* arena,
                                                   u32* done = nullptr, u32 seq = 0) {
    u64* head = (u64*)arena;
    u32* rb = (u32*)(arena + 16);
    const u32 k = blockIdx.x;
    // Loaded before the first store: a load issued after stores into the mapped arena would wait
    // for their PCIe round trip (gfx950's vmcnt counts stores too).
    const u32 bytes = k < nb ? reply_bytes[k] : 0;
    const u64 boff = k < nb ? batch_off[k] : 0;
    if (k == 0 && threadIdx.x == 0) {
        head[0] = g->panic;
        head[1] = g->commit_timestamp;
    }
    if (k < nb) {
        if (threadIdx.x == 0) rb[k] = bytes;
        u32* out = (u32*)(arena + 16 + (u64)nb * 4 + 8 * boff);  // 4-B aligned: nb words before
        const u32* in = results + 2 * boff;
        // Eight loads in flight before their stores (each store into the arena is a PCIe write).
        const u32 nw = bytes / 4;
        for (u32 w0 = threadIdx.x; w0 < nw; w0 += 8 * 64) {
            u32 v[8];
#pragma unroll
            for (u32 q = 0; q < 8; q++) v[q] = w0 + q * 64 < nw ? in[w0 + q * 64] : 0;
#pragma unroll
            for (u32 q = 0; q < 8; q++) {
                if (w0 + q * 64 < nw) out[w0 + q * 64] = v[q];
            }
        }
    }
    if (seq) {  // one wave: its stores drain, then the flag
        __threadfence_system();
        if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

