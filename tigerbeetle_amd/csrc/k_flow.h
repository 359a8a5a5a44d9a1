// k_flow.h — kernel 3 of a create_transfers pass, parallel form: the ordered fallback as a
// dependency DAG executed by many lanes at once.
//
// The dependent events of a pass (k_resolve.h) must see each other's effects in batch order
// (execute, state_machine.zig:612-698).  They interact only through RESOURCES:
//   * the balance of a constrained account — a limit flag (tigerbeetle.zig:31-39), a balancing
//     mark of this pass (:826-846), or any account when the global overflow certificate fails
//     (:848-861);
//   * a transfer id: the event's own id (exists / insert, :824, :954) and, for a post/void, its
//     pending id (pending lookup, posted status, :927-964).
// A post/void also writes the balances of its pending transfer's accounts (:987-1010): when one of
// them is constrained it is a resource of the post/void too, found from the pending transfer
// (an earlier pass's record, or the event of this pass that creates it).  Balances of free
// accounts feed no check and take commutative atomic deltas (k_replay.h, FLOW = true).
//
// A UNIT is a linked chain (executed whole, with its undo log: chains roll back as one,
// :661-692) or a single event.  Two units that share a resource run in batch order; units that
// share none commute.  The kernel:
//   plan   every workgroup: list the pass's dependent events in order, emit (resource key, unit)
//          pairs, compact them in order, radix-sort them by key (stable, so each key's units stay
//          in batch order) and link every unit to its successor on each of its resources
//          (need[] = predecessors);
//   bounds a pass whose dependent units are plain limit checks is decided by segmented-scan
//          rounds and an in-order sweep instead of a run (fl_bounds, fl_sweep);
//   run    every lane of every workgroup: one ticket queue of ready units in global memory; a
//          lane executes its unit with the reference logic, then releases its successors,
//          queueing those with no predecessor left.  The result equals the sequential replay's:
//          every unit sees exactly the effects of the units before it on its resources, and
//          nothing else it reads can differ.
// Grid-wide phases are separated by a counter barrier among the workgroups ADMITTED at the start
// (fl_admit): the first one waits briefly for the launch's others, then closes admission; the ones
// that started by then are the grid the pass is partitioned over (FL_B of FL_G), and a workgroup
// that starts later — the device was shared and it could not be resident — exits at once.  So a
// co-tenant holding CUs makes the pass slower, never a stall.  Cases the planner does not cover (a chain longer than FLOW_CHAIN_MAX, a pending id
// whose creator in this pass is ambiguous) set a flag, and workgroup 0 runs the sequential replay
// for the pass instead.  Every wait is bounded: a stall raises PANIC_FLOW_STALL, never a hang.
#pragma once

#include "k_replay.h"

#define FLOW_THREADS 1024
#define FLOW_RMAX 6             // resources per event: id, pending id, two accounts (+2 inherited)
#define FLOW_CHAIN_MAX 64       // longer chains: sequential replay
#define FLOW_NB_MAX 4096        // prepares per pass the planner handles (LDS prefix)
#define FLOW_SENT 0xFFFFFFFFu   // empty pair slot
// This workgroup's index among the admitted ones, and their number (fl_admit); ~0: not admitted.
__shared__ u32 s_fl_b, s_fl_g;
#define FL_B ((u32)__builtin_amdgcn_readfirstlane(s_fl_b))  // uniform: a scalar register, as blockIdx.x was
#define FL_G ((u32)__builtin_amdgcn_readfirstlane(s_fl_g))
#define FL_ADM_CLOSED 0x80000000u
#define FL_ADMIT_TICKS 5000  // wall-clock ticks (50 us at 100 MHz) the first workgroup waits for the others

#ifndef FLOW_POLL_SLEEP
#define FLOW_POLL_SLEEP 16      // s_sleep units (64 cycles) between a waiting lane's polls
#endif
#ifndef FLOW_POLL_DONE
#define FLOW_POLL_DONE 32       // a waiting lane reads the done counter every this many polls
#endif

enum : u32 { FW_NUNITS = 0, FW_QTAIL = 1, FW_SEQ = 2, FW_BNO = 3, FW_BUND = 4, FW_BDEC = 5,  // 5, 6, 7
             FW_QHEAD = 8, FW_DONE = 9, FW_WMAX = 10, FW_WORDS = FLOW_WORDS };
enum : u32 {
    UF_ID_SINGLE = 1,  // the unit is the only dependent event of the pass whose id has its key
    UF_ID_UNIQUE = 2,  // ... or the others sharing the key (a 31-bit hash) name different ids
    UF_MEMBER_NEW = 4, // per flat entry f (any member of a unit): no other dependent event of the
                       // pass has f's own id key (its id is new if kernel 1's claim was: HZ_SPEC)
};

// Everything a run needs of the unit at sorted position q, packed by the planner so the run walker
// reads one level (the list entry) instead of three (list entry -> unit -> event).
struct RunEntry {
    u32 u, pe, dr, cr, rs;
    u32 flags;  // event flags | RUN_MEMBER
    u64 amt_lo, amt_hi;
};
#define RUN_MEMBER (1u << 16)

struct FlowArgs {
    u32* f_pe;      // [pass events] flat dependent f -> pass-relative event
    u32* f_batch;   // [pass events] f -> call-relative batch
    u32* f_len;     // [pass events] unit heads: members; other members: 0
    u32* need;      // [pass events] per unit head: predecessors not yet done
    u32* nsucc;     // [pass events] per unit head: successors
    u32* succ;      // [FLOW_RMAX * pass events] unit u's successors at FLOW_RMAX * u
    u32* queue;     // [pass events] ready units (head + 1; 0 = not yet published)
    u32* uflags;    // [pass events] per unit head: UF_*
    u32* nacct;     // [pass events] per unit head: account resources
    u32* rpos;      // [pass events] per unit head: sorted position of its (last) account resource
    RunEntry* run;  // [FLOW_RMAX * pass events] per sorted position (account resources)
    u32* keys[2];   // [FLOW_RMAX * pass events] radix-sort ping-pong buffers
    u32* vals[2];
    u32* hist;      // [grid * 256]
    u32* words;     // [FW_WORDS], zeroed by tb_resolve every pass
    UndoEntry* undo;  // [4 * pass events] chain of head u: [4u, 4u + 4 * len)
    u32 grid;
    u32 grid_alloc;  // workgroups the per-workgroup arrays (hist, b_blk) hold: at most this many are admitted
    u64 stall_ticks;  // wall_clock64 ticks after which a wait is taken as an engine bug (PANIC_FLOW_STALL)
    // Bounds certification of limit checks (fl_bounds): per unit head its state and the verdicts of
    // its debit-side / credit-side limit check; per account-resource position its leg.
    u32* b_st;      // [pass events] BS_*
    u8* b_vd;       // [pass events] BV_* of the debit account's check
    u8* b_vc;       // [pass events] BV_* of the credit account's check
    u64* b_amt;     // [FLOW_RMAX * pass events] leg amount (< 2^64 under the certificate)
    u32* b_meta;    // [FLOW_RMAX * pass events] unit << 3 | BT_* | BT_CR
    u64* b_blk;     // [grid * 5] per workgroup: segment-start flag, then 4 sums
    u32 bounds_rounds_max;
    // The in-order sweep that decides what the rounds leave undecided (fl_sweep).
    u32 sweep_min;  // rounds continue while one decides at least this many units
    u32* b_qd;      // [pass events] per undecided unit: sorted position of its debit leg (or FLOW_SENT)
    u32* b_qc;      // [pass events] ... of its credit leg
    u32* b_head;    // [FLOW_RMAX * pass events] per position of an undecided unit: its segment's first
    u64* b_xy;      // [2 * FLOW_RMAX * pass events] per such position: X, Y with the decided units before it
    u64* b_ex;      // [2 * FLOW_RMAX * pass events] per segment head: X, Y added by swept ok units
    struct SweepRec* b_rec;  // [pass events] per undecided unit in event order: what the sweep reads
    // Per-account walkers (fl_walk; the window sweep's replacement when every sum is below 2^62):
    // their position records live in b_ex, their segment lists and cursors in b_rec.
    u32* b_vw;      // [pass events] per undecided unit: its two checks' verdicts, vd | vc << 2 (atomicOr)
    u32 walk;       // 1: per-account walkers; 0: the one-wave window sweep (TBGPU_CONFIG_SWEEP_WINDOW)
    u32 walk_merge; // heavy segments walked merged by one wave at most (WALK_MERGE_MAX)
};

// Every wait of the kernel is bounded by wall time (s_memrealtime) since the wait began.
__device__ static inline u64 fl_now() {
    u64 t = (u64)wall_clock64();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return t;
}
// Phase timer of tb_flow (workgroup 0, thread 0; device wall clock): adds the time since the last
// mark to flow_phase_ticks[k].  Phases: FP_PLAN (flat list), FP_SORT, FP_LINK (links + packing),
// FP_BSETUP, FP_BROUNDS, FP_SWEEP, FP_RUN (ordered run, or applying the bounds' decisions),
// FP_REPLIES.
enum : u32 { FP_PLAN = 0, FP_SORT, FP_LINK, FP_BSETUP, FP_BROUNDS, FP_SWEEP, FP_RUN, FP_REPLIES };
__device__ static inline void fl_mark(Globals* g, u64& t, u32 k) {
    if (FL_B != 0 || threadIdx.x != 0) return;
    const u64 now = (u64)wall_clock64();
    atomicAdd((unsigned long long*)&g->flow_phase_ticks[k], (unsigned long long)(now - t));
    t = now;
}
__device__ static inline bool fl_expired(const FlowArgs& F, u64 w0) {
    const u64 now = fl_now();
    return now > w0 && now - w0 > F.stall_ticks;
}

// Resource keys: an account slot (< 2^31) or 2^31 | a 31-bit hash of a transfer id.  Two ids that
// share a hash only add an ordering edge, never lose one.
__device__ static inline u32 fl_key_id(u64 lo, u64 hi) {
    return 0x80000000u | (u32)(tb_mix64(lo ^ tb_mix64(hi ^ 0x9e3779b97f4a7c15ULL)) % 0x7FFFFFFFu);
}

// Admission (tb_flow's first step): every workgroup takes a ticket on the entry counter; the first
// waits until the whole launch (at most grid_alloc workgroups) has entered or FL_ADMIT_TICKS passed,
// closes the counter and publishes how many entered.  Those are the grid: indices FL_B = their
// tickets, FL_G = the number published.  A workgroup whose ticket comes after the close returns false (the host launches at
// most its share of the device, engine.hip flow_grid, so on a device this process owns every
// workgroup enters within microseconds; one a co-tenant kept off the device enters late).  The
// counters are zeroed with the barrier's by tb_resolve every pass.
__device__ static inline bool fl_admit(Globals* g, const FlowArgs& F) {
    if (threadIdx.x == 0) {
        u32* entry = &g->flow_bar[FL_BAR_STRIDE * (FL_BAR_GROUPS + 2)];
        u32* grid = &g->flow_bar[FL_BAR_STRIDE * (FL_BAR_GROUPS + 3)];
        const u32 cap = min(gridDim.x, F.grid_alloc);
        const u32 t = __hip_atomic_fetch_add(entry, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_fl_b = (t & FL_ADM_CLOSED) || t >= cap ? ~0u : t;
        if (t == 0) {
            const u64 w0 = fl_now();
            while ((__hip_atomic_load(entry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~FL_ADM_CLOSED) < cap) {
                __builtin_amdgcn_s_sleep(2);
                const u64 now = fl_now();
                if (now > w0 && now - w0 > FL_ADMIT_TICKS) break;
            }
            const u32 n = __hip_atomic_fetch_or(entry, FL_ADM_CLOSED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(grid, min(n & ~FL_ADM_CLOSED, cap), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (s_fl_b != ~0u) {
            const u64 w0 = fl_now();
            u32 n;
            while ((n = __hip_atomic_load(grid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
                __builtin_amdgcn_s_sleep(2);
                if (fl_expired(F, w0)) {
                    tb_panic(g, PANIC_FLOW_STALL);
                    break;
                }
            }
            s_fl_g = n;
            if (n == 0 || s_fl_b >= n) s_fl_b = ~0u;  // (a stall: leave)
        }
    }
    __syncthreads();
    return s_fl_b != ~0u;
}

// Grid barrier of the co-resident grid (engine.hip flow_grid).  Two levels, so arrivals do not all
// serialise on one word: the workgroups of each of FL_BAR_GROUPS groups (FL_B mod groups)
// count on their group's word, the last of a group counts on the root word, and the last group
// publishes the generation, which every workgroup polls.  Every counter only grows (generation gen
// waits for gen * members); tb_resolve zeroes them each pass.  Each workgroup writes its L2 back
// (release) before it arrives and invalidates (acquire) after it leaves.
__device__ static inline void fl_grid_sync(Globals* g, u32 nblocks, u32& gen, const FlowArgs& F) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the barrier
    __syncthreads();
    gen++;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const u32 groups = min(nblocks, (u32)FL_BAR_GROUPS), grp = FL_B % groups;
        const u32 members = (nblocks - grp + groups - 1) / groups;
        u32* bar = g->flow_bar;
        const u32 a = __hip_atomic_fetch_add(&bar[FL_BAR_STRIDE * grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a + 1 == gen * members) {
            const u32 r = __hip_atomic_fetch_add(&bar[FL_BAR_STRIDE * FL_BAR_GROUPS], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            if (r + 1 == gen * groups) {
                __hip_atomic_store(&bar[FL_BAR_STRIDE * (FL_BAR_GROUPS + 1)], gen, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const u64 w0 = fl_now();
        while (__hip_atomic_load(&bar[FL_BAR_STRIDE * (FL_BAR_GROUPS + 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               gen) {
            __builtin_amdgcn_s_sleep(2);
            if (fl_expired(F, w0)) {
                tb_panic(g, PANIC_FLOW_STALL);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

__device__ static inline bool fl_stalled(Globals* g) {
    return (__hip_atomic_load(&g->panic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & PANIC_FLOW_STALL) != 0;
}

// Resources a post/void inherits from its pending transfer: the constrained accounts of an
// earlier pass's pending record, and those of the event of this pass that claimed the pending id
// (its creator; the ordering on the pending id puts the post/void after it).  Returns false when
// the creator is ambiguous (its id collided in this pass).
__device__ static inline bool fl_pending_accounts(const PassArgs& P, u64 lo, u64 hi, bool cert_global, u32* keys,
                                                  u32& nk) {
    const Tables& T = P.T;
    if (tb_id_reserved(lo, hi)) return true;
    const u64 fp = tb_fp32(lo, hi);
    u64 pos = tb_hash_id(lo, hi) & T.xidx_mask;
    for (u64 n = 0; n <= T.xidx_mask; n++) {
        const u64 e = T.xidx[pos];
        if (e == 0) return true;
        if ((e >> 32) == fp) {
            const u32 lp = tb_xi_pos(e);
            u32 drs = TB_NOT_FOUND, crs = TB_NOT_FOUND;
            if ((u64)lp < P.log_base) {
                if (!(e & XI_TOMB)) {
                    const Transfer& p = T.xlog[lp];
                    if (p.id == tb_u128(lo, hi)) {
                        drs = tb_account_find(T, tb_lo(p.debit_account_id), tb_hi(p.debit_account_id));
                        crs = tb_account_find(T, tb_lo(p.credit_account_id), tb_hi(p.credit_account_id));
                    }
                }
            } else {
                const u32 c = (u32)(lp - P.log_base);
                const Transfer& ce = *(const Transfer*)(P.events + (P.e0 + c) * 128);
                if (ce.id == tb_u128(lo, hi)) {
                    if (T.xdup[pos]) return false;  // its id collided in this pass: creator ambiguous
                    if (!(P.eflags[c] & (TF_POST | TF_VOID)) && (P.info[c] & HZ_ACCTS)) {
                        drs = P.dr[c];
                        crs = P.cr[c];
                    }
                }
            }
            if (drs != TB_NOT_FOUND && fl_account_is_resource(T, drs, P.epoch, cert_global)) keys[nk++] = drs;
            if (crs != TB_NOT_FOUND && fl_account_is_resource(T, crs, P.epoch, cert_global)) keys[nk++] = crs;
            if (nk > FLOW_RMAX - 2) return false;  // several matching records: keep it simple
        }
        pos = (pos + 1) & T.xidx_mask;
    }
    return true;
}

// Execute one unit (a chain or a single event) with the reference logic; returns the max
// timestamp of its events that returned ok.
__device__ static inline u64 fl_run_unit(const PassArgs& P, const FlowArgs& F, Replay& R, u32 u) {
    const u32 m = F.f_len[u];
    R.undo = F.undo + 4ULL * u;
    R.undo_cap = 4 * m;
    R.undo_len = 0;
    R.scope = false;
    u64 tsmax = 0;
    bool in_chain = false, broken = false;
    // A member's words are loaded together, one level after its flat-list entry, and the next
    // member's entry is loaded with them (a chain's members then cost one round trip less each).
    u32 pe_next = F.f_pe[u], b_next = F.f_batch[u];
    for (u32 j = 0; j < m && !R.failed; j++) {
        const u32 f = u + j;
        const u32 pe = pe_next;
        const u32 b = b_next;
        if (j + 1 < m) {
            pe_next = F.f_pe[f + 1];
            b_next = F.f_batch[f + 1];
        }
        const u8* ev = P.events + (P.e0 + pe) * 128;
        const u64 boff = P.batch_off[b];
        const u64 bend = P.batch_off[b + 1];
        const u16 flags = P.eflags[pe];
        const u32 info = P.info[pe];
        const u32 w_dr = P.dr[pe], w_cr = P.cr[pe], w_rs = P.rs[pe];
        const u32 uf = F.uflags[f];
        Transfer t = *(const Transfer*)ev;
        const u32 L = (u32)(bend - boff);
        const u32 i = (u32)(P.e0 + pe - boff);
        // In place, kernel 1 stamped an HZ_INPLACE event's record (= the event): its field was 0.
        const u64 evts = (P.routed || (info & HZ_INPLACE)) ? 0 : t.timestamp;
        const bool linked = flags & TF_LINKED;
        u32 result;
        if (linked && !in_chain) {
            in_chain = true;
            R.scope = true;
            R.undo_len = 0;
        }
        if (linked && i == L - 1) {
            result = R_LINKED_EVENT_CHAIN_OPEN;
        } else if (broken) {
            result = R_LINKED_EVENT_FAILED;
        } else if (evts != 0) {
            result = R_TIMESTAMP_MUST_BE_ZERO;
        } else {
            const u64 ts = tb_event_ts(P, b, boff, L, i);
            t.timestamp = ts;
            FastHint hint;
            // Kernel 1's account slots: a create's two accounts, or a post/void's pending transfer's
            // (it reached HZ_ACCTS only with that pending from an earlier pass).
            const bool slots = (info & HZ_ACCTS) != 0;
            const bool fast = slots && (info & HZ_SPEC) && !(flags & (TF_POST | TF_VOID)) &&
                              ((m == 1 && (uf & UF_ID_SINGLE)) || (uf & UF_MEMBER_NEW));
            if (slots) {
                hint.drs = w_dr;
                hint.crs = w_cr;
                hint.entry = (info & HZ_SPEC) ? w_rs : TB_NOT_FOUND;
                hint.known_new = fast;
                hint.rec = (info & HZ_REC) && !(flags & (TF_POST | TF_VOID | TF_BAL_DEBIT | TF_BAL_CREDIT));
            }
            result = rp_create_transfer<true>(R, t, (u32)(R.log_base + pe), slots ? &hint : nullptr);
            if (result == R_OK && !R.failed) tsmax = ts;
        }
        if (R.failed) break;
        if (result != R_OK && in_chain && !broken) {
            broken = true;
            rp_scope_close<true>(R, false);  // commit_timestamp keeps their timestamps (:763, :882)
            for (u32 jj = 0; jj < j; jj++) {
                u32* w = &P.info[F.f_pe[u + jj]];
                *w = (*w & 0xFFFFFF00u) | R_LINKED_EVENT_FAILED;
            }
        }
        P.info[pe] = (info & 0xFFFFFF00u) | result;  // only this lane writes it from here
        if (in_chain && (!linked || result == R_LINKED_EVENT_CHAIN_OPEN)) {
            if (!broken) rp_scope_close<true>(R, true);
            in_chain = false;
            broken = false;
        }
    }
    return tsmax;
}

// A RUN: consecutive units on one account resource r that each are a single plain create_transfer
// whose only other state is free — kernel 1 validated it fully (code ok through the timeout check,
// :779-862), its id is new and named by no other dependent event, r is its only constrained
// account, and it is not balancing.  The only open check is r's limit (tigerbeetle.zig:31-39)
// against r's running balance: a lane keeps r's balances in registers and walks the run down r's
// sorted resource list, eight units per step with their loads issued together.  Kernel 1 already
// wrote each record; an ok unit revives its index entry, adds its amount to r (registers) and to
// its free account (atomic delta); a failed one gets exceeds_credits / exceeds_debits.
#define FLOW_RUN_STEP 8

// Runs the run headed by unit u (a run member); returns the last unit it ran (its successors are
// released by the caller), *count = units run, *tsmax = max ok timestamp.
// (q, r): the head's sorted position and its account resource, already read by the caller.
__device__ static inline u32 fl_run_run(const PassArgs& P, const FlowArgs& F, Replay& R, u32 u, u32 N,
                                        u32 q, u32 r, u32* count, u64* tsmax) {
    const Tables& T = P.T;
    const u32* K = F.keys[0];
    AccountBal B = rp_bal_load<true>(T.bal, r);
    const u16 rflags = T.acct_hot[r].flags;
    u32 n = 0, n_ok = 0, last = u, last_ok_pe = TB_NOT_FOUND;
    bool more = true;
    while (more) {
        // One load level for eight candidates at once: the planner's packed entries (RunEntry).
        u32 cu[FLOW_RUN_STEP], cpe[FLOW_RUN_STEP], cdr[FLOW_RUN_STEP], ccr[FLOW_RUN_STEP], crs_[FLOW_RUN_STEP];
        u64 camt[FLOW_RUN_STEP], camt_hi[FLOW_RUN_STEP];
        u16 cfl[FLOW_RUN_STEP];
        bool ok[FLOW_RUN_STEP];
#pragma unroll
        for (u32 j = 0; j < FLOW_RUN_STEP; j++) {
            ok[j] = q + j < N && K[q + j] == r;
            RunEntry x = {};
            if (ok[j]) x = F.run[q + j];
            cu[j] = x.u;
            cpe[j] = x.pe;
            cdr[j] = x.dr;
            ccr[j] = x.cr;
            crs_[j] = x.rs;
            cfl[j] = (u16)x.flags;
            camt[j] = x.amt_lo;
            camt_hi[j] = x.amt_hi;
            ok[j] = ok[j] && (x.flags & RUN_MEMBER);
        }
        u32 j = 0;
        for (; j < FLOW_RUN_STEP && ok[j]; j++) {
            const u32 pe = cpe[j];
            const u32 drs = cdr[j], crs = ccr[j];
            const bool debit = drs == r;  // else r is the credit side
            const bool pend = cfl[j] & TF_PENDING;
            const u128 amount = tb_u128(camt[j], camt_hi[j]);
            u32 code = R_OK;
            if (debit && (rflags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
                B.debits_pending + B.debits_posted + amount > B.credits_posted) {
                code = CT_EXCEEDS_CREDITS;
            } else if (!debit && (rflags & AF_CREDITS_MUST_NOT_EXCEED_DEBITS) &&
                       B.credits_pending + B.credits_posted + amount > B.debits_posted) {
                code = CT_EXCEEDS_DEBITS;
            }
            if (code == R_OK) {
                u128* rf = debit ? (pend ? &B.debits_pending : &B.debits_posted)
                                 : (pend ? &B.credits_pending : &B.credits_posted);
                *rf += amount;
                // The free side: one field, +amount (exact in any order).
                const u32 fs = debit ? crs : drs;
                const u32 ff = debit ? (pend ? BAL_CP : BAL_CPOST) : (pend ? BAL_DP : BAL_DPOST);
                if (R.cert64) tb_bal_add_lo(T.bal, fs, ff, tb_lo(amount));
                else tb_bal_add(T.bal, fs, ff, amount);
                __hip_atomic_fetch_and(&T.xidx[crs_[j]], ~(u64)XI_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                n_ok++;
                last_ok_pe = pe;
            } else {
                P.info[pe] = (P.info[pe] & 0xFFFFFF00u) | code;
            }
            last = cu[j];
            n++;
        }
        more = j == FLOW_RUN_STEP;
        q += FLOW_RUN_STEP;
    }
    rp_bal_store<true>(T.bal, r, B);
    R.xcount += n_ok;
    if (last_ok_pe != TB_NOT_FOUND) {  // commit_timestamp: the run's last ok event is its latest
        u32 lo = P.b0, hi = P.b1;
        const u64 e = P.e0 + last_ok_pe;
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (P.batch_off[mid] <= e) lo = mid; else hi = mid;
        }
        const u64 boff = P.batch_off[lo];
        *tsmax = tb_event_ts(P, lo, boff, (u32)(P.batch_off[lo + 1] - boff), (u32)(e - boff));
    }
    *count = n;
    return last;
}

// Replies of every prepare with dependent events (their final codes are in P.info), then close
// the pass: bound += S, reset the dependent counter.  Workgroup 0, every thread.
// Replies of the prepares with dependent events, those with k % parts == part (every workgroup of a
// grid takes its share); the pass bookkeeping by the closing workgroup (`close`).
__device__ static inline void fl_finish(const PassArgs& P, u8* s_code, u32* s_wave, u32* s_list, u64 tsmax_block,
                                         bool any, u32 part = 0, u32 parts = 1, bool close = true) {
    Globals* g = P.T.g;
    const u32 nb = P.b1 - P.b0;
    for (u32 c = 0; any && c < nb; c += blockDim.x) {
        const u32 k = c + threadIdx.x;
        const bool has = k < nb && k % parts == part && P.dep_count[k] > 0;
        u32 total;
        const u32 r = tb_block_rank(has, s_wave, total);
        if (has) s_list[r] = k;
        __syncthreads();
        for (u32 q = 0; q < total; q++) {
            const u32 b = P.b0 + s_list[q];
            const u64 boff = P.batch_off[b];
            const u32 L = (u32)(P.batch_off[b + 1] - boff);
            const u32 pbase = (u32)(boff - P.e0);
            for (u32 i = threadIdx.x; i < L; i += blockDim.x) s_code[i] = (u8)(P.info[pbase + i] & 0xFF);
            __syncthreads();
            tb_write_replies(P, b, L, s_code, s_wave);
            __syncthreads();
        }
    }
    if (close && threadIdx.x < 64) {
        const u128 S = tb_sum_total_wave(P.sum_shards);  // wave 0, every lane
        if (threadIdx.x == 0) {
            // Every load before the first store (a load after a store waits for it).
            const u64 blo = g->bound_lo, bhi = g->bound_hi, da = g->dependent_all, dt = g->dependent_total;
            // Other workgroups' atomicMax of their own maxima may still be in flight: max, not a store.
            if (tsmax_block) atomicMax((unsigned long long*)&g->commit_timestamp, (unsigned long long)tsmax_block);
            const u128 nb2 = tb_sat_add(tb_u128(blo, bhi), S);
            g->bound_lo = tb_lo(nb2);
            g->bound_hi = tb_hi(nb2);
            g->dependent_all = da + dt;
            g->dependent_total = 0;
        }
    }
}

// ---- bounds certification of the limit checks (north star (c)) ---------------------------------
// A pass whose dependent events are all single plain create_transfers that kernel 1 validated
// (their only open checks are the limits of their flagged accounts, tigerbeetle.zig:31-39,
// state_machine.zig:863-864; the certificate rules out every overflow check and 64-bit sums
// suffice) is decided without the ordered run.  Per limit account, its events in batch order form
// a segment (the planner's sorted resource list).  For a debits_must_not_exceed_credits account
// the check of a debit is  dp + dpost + (earlier ok debits) + amount <= cpost + (earlier ok posted
// credits);  credits_must_not_exceed_debits is the mirror image.  Each ROUND takes a segmented
// prefix scan (LDS + wave shuffles, grid-wide carries) of four sums per position: the earlier debits
// counting only decided-ok units (min) or every unit not decided failing (max), and the same for the
// credits.  A check certainly passes if it passes with max debits and min credits, certainly fails if
// it fails with min debits and max credits.  A unit is decided once its checks decide its result in
// the reference's order (exceeds_credits before exceeds_debits).  The first undecided event of every
// segment sees only decided events before it, so each round decides at least one event per segment
// and the rounds terminate; the bounds usually decide far more.  Decisions are
// facts, not effects: nothing is applied until every unit is decided, then the ok units' balance
// legs and index entries are applied in parallel (the sums commute).  A pass with any other kind of
// dependent unit, or one that does not converge within bounds_rounds_max, takes the ordered run
// with nothing changed.
#define FLOW_BOUNDS_ROUNDS_MAX 4096
// A scan round costs about as much as sweeping this many units in order (fl_sweep).
#ifndef FLOW_SWEEP_MIN
#define FLOW_SWEEP_MIN 512
#endif
enum : u8 { BS_UNK = 0, BS_OK = 1, BS_FAIL_CREDITS = 2, BS_FAIL_DEBITS = 3, BS_FAIL_STATIC = 4 };
enum : u8 { BV_UNK = 0, BV_PASS = 1, BV_FAIL = 2 };
enum : u32 { BT_NONE = 0, BT_X = 1, BT_Y = 2, BT_CR = 4 };  // X: checked side (any field); Y: other side, posted

// Inclusive segmented scan of four u64 sums over the workgroup (one position per thread), on top of
// `carry` (the running sums of the segment open at the chunk start).  f = 1 starts a segment.
// Returns the inclusive sums in v; carry becomes the chunk's last inclusive sums.
__device__ static inline void fl_seg_scan4(u64 (&v)[4], u32 f, u64 (&carry)[4], u64 (*s_wv)[4], u32* s_wf) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (u32 off = 1; off < 64; off <<= 1) {
        u64 o[4];
#pragma unroll
        for (u32 k = 0; k < 4; k++) o[k] = __shfl_up((unsigned long long)v[k], off);
        const u32 of = __shfl_up(f, off);
        if (lane >= off) {
            if (!f) {
#pragma unroll
                for (u32 k = 0; k < 4; k++) v[k] += o[k];
            }
            f |= of;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (u32 k = 0; k < 4; k++) s_wv[wave][k] = v[k];
        s_wf[wave] = f;
    }
    __syncthreads();
    u64 pv[4] = {carry[0], carry[1], carry[2], carry[3]};
    for (u32 w = 0; w < wave; w++) {
        if (s_wf[w]) {
#pragma unroll
            for (u32 k = 0; k < 4; k++) pv[k] = s_wv[w][k];
        } else {
#pragma unroll
            for (u32 k = 0; k < 4; k++) pv[k] += s_wv[w][k];
        }
    }
    if (!f) {
#pragma unroll
        for (u32 k = 0; k < 4; k++) v[k] += pv[k];
    }
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) {
#pragma unroll
        for (u32 k = 0; k < 4; k++) s_wv[0][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (u32 k = 0; k < 4; k++) carry[k] = s_wv[0][k];
    __syncthreads();
}

// Contribution of position q this round: {debits min, max, credits min, max} of the checked
// account's sides (X = the checked side, Y = the other side's posted field).
__device__ static inline void fl_bound_contrib(const FlowArgs& F, u32 q, u64 (&v)[4]) {
    const u32 meta = F.b_meta[q];
    const u64 a = F.b_amt[q];
    const u32 st = F.b_st[meta >> 3];
    const u64 mn = st == BS_OK ? a : 0, mx = (st == BS_OK || st == BS_UNK) ? a : 0;
    const bool x = meta & BT_X, y = meta & BT_Y;
    v[0] = x ? mn : 0;
    v[1] = x ? mx : 0;
    v[2] = y ? mn : 0;
    v[3] = y ? mx : 0;
}

// ---- the in-order sweep of what the rounds leave undecided --------------------------------------
// When a round decides few units (a limit account whose balance hovers at its limit: every check
// depends on the one before), the rest is decided exactly, in event order, by one wave:
//  1. every workgroup: a last segmented scan over the positions with the decided units only records,
//     per position of an undecided unit, X and Y of its account with every decided ok unit before it
//     (the pre-pass balance plus the min sums) and its segment's first position (a segmented sum of
//     q at the segment starts); then the undecided units are listed in event order;
//  2. wave 0 of workgroup 0 walks the list 64 units at a time: a lane holds one unit's legs, adds
//     what the swept ok units before its window added to its segments (b_ex, by segment head), and
//     the window is resolved lane by lane in order, each verdict broadcast to the later lanes that
//     share an account; the ok units' legs go to b_ex for the later windows.
// X, Y are exact at every step: a position's earlier units are decided (in the min sums), or swept
// (b_ex, and the window's broadcasts), or later in event order than the unit being swept.
__device__ static inline void fl_record_contrib(const FlowArgs& F, const u32* K, u32 q, u64 (&v)[4], u32& f) {
    const u32 meta = F.b_meta[q];
    const u64 a = F.b_amt[q];
    const bool ok = F.b_st[meta >> 3] == BS_OK;
    f = q == 0 || K[q] != K[q - 1];
    v[0] = ok && (meta & BT_X) ? a : 0;
    v[1] = f ? q : 0;  // summed over a segment: its first position
    v[2] = ok && (meta & BT_Y) ? a : 0;
    v[3] = 0;
}

// Wave-uniform u64 read of lane j / write of lane j (j uniform).
__device__ static inline u64 fl_rl64(u64 v, u32 j) {
    return ((u64)(u32)__builtin_amdgcn_readlane((u32)(v >> 32), j) << 32) | (u32)__builtin_amdgcn_readlane((u32)v, j);
}

struct SweepRec {  // one undecided unit, in event order (fl_sweep)
    u32 f, hd, hc;     // unit; segment heads of its debit / credit leg (FLOW_SENT: no leg)
    u32 t;             // BT_* of the debit leg | ... of the credit leg << 4 | vd << 8 | vc << 12
    u64 a;             // amount
    u64 xd, yd, xc, yc;  // X, Y at each leg with the decided units before it
    u64 pad;
};

// The sweep's LDS home for the swept sums of segment heads (b_ex in global memory otherwise): an
// open-addressing table of SW_CAP heads in LDS the planner and the sort no longer use.  A head
// claims a slot on first sight and keeps it; a head that finds its SW_PROBES slots taken stays in
// global memory for the whole sweep (slots are never freed, so it never finds one later).
#define SW_CAP 1024
#define SW_PROBES 16
#define SW_NONE 0xFFFFFFFFu
__device__ static inline u32 fl_sw_slot(u32* s_hk, u32 head) {
    if (head == FLOW_SENT) return SW_NONE;
    u32 h = (head * 2654435761u) >> 22;  // 10 bits: SW_CAP
    for (u32 n = 0; n < SW_PROBES; n++) {
        const u32 k = s_hk[h];
        if (k == head) return h;
        if (k == FLOW_SENT) {
            const u32 old = atomicCAS(&s_hk[h], FLOW_SENT, head);
            if (old == FLOW_SENT || old == head) return h;
        }
        h = (h + 1) & (SW_CAP - 1);
    }
    return SW_NONE;
}

// ---- the sweep as per-account walkers (fl_walk) --------------------------------------------------
// What the rounds leave undecided is a set of SEGMENTS: per limit account, its undecided positions in
// event order.  A check at position q passes iff the account's slack there — Y − X with every
// decided ok unit before q (b_xy) plus the swept ok units before q on the same account — is at
// least the amount.  So one walker per segment decides its checks in order with a running sum d of
// its own swept deltas (an ok X leg: −a, an ok Y leg: +a), and walkers meet only at units with legs
// on two segments:
//   * a Y leg (the other side's posted field) needs the unit's final status, which the walker of
//     the unit's check publishes (b_st, agent scope);
//   * a unit with two open checks (a debits-limited debit account and a credits-limited credit
//     account) combines them in the reference's order (:863-864): each side ORs its verdict into
//     b_vw, and whichever side completes the pair publishes the status.  A side that fails needs
//     nothing more (its account takes no delta whatever the other side says).
// Walkers wait only on units earlier in event order on their partner's account, so the walker at
// the globally earliest waiting point is never blocked: no deadlock while every walker keeps
// being visited.  A segment with at least WALK_HEAVY positions (a Zipf-hot limit account's) gets a
// wave of its own; the others share the remaining waves, each wave cycling through its segments
// and moving on from a blocked one.  A wave walks its segment 64 positions a window: the
// records and the statuses its Y legs and paired checks need are loaded by the 64 lanes at once,
// then the window is resolved in order — in parallel by runs of ok / failed positions (a prefix
// sum and a ballot per run, fl_runs32) — stopping at a position whose partner has not decided yet.
// A heavy walker takes an open Y leg as a pending credit and goes on, and carries the credits
// still pending at a window's end into the next window (WalkCarry) rather than waiting for them.
struct WalkRec {
    i64 base;  // Y − X of the account with every decided ok unit before this position (balances included)
    i64 a;     // the leg's amount
    u32 u;     // unit
    u32 kind;  // BT_X | BT_Y | BT_CR of the leg; the unit's verdicts when listed: vd << 8 | vc << 12
    u32 head;  // the segment's (account's) first sorted position
    u32 pad;
};
#ifndef WALK_HEAVY
#define WALK_HEAVY 256
#endif
#define WALK_RING 8  // windows a feeder wave keeps ahead of its walker in LDS

#ifndef WALK_CARRY
#define WALK_CARRY 1  // windows a heavy walker carries its pending credits (0: each window waits for its own);
                      // C3h 0: 99.5, 1: 120.1, 2: 116.9, 3: 113.2 M/s
#endif
#define WALK_NC (WALK_CARRY > 0 ? WALK_CARRY : 1)
#ifndef WALK_PAR
#define WALK_PAR 1  // 0: the 32-bit chain as a scalar step per lane (C3h 73.2 M/s against 99.2)
#endif
#ifndef WALK_CNT
#define WALK_CNT 0  // A/B builds only: count the critical walker's positions by path (walk_dbg)
#endif
#ifndef WALK_PROF
#define WALK_PROF 0  // A/B builds only: time the critical heavy walker's phases (walk_dbg)
#endif
#ifndef WALK_DEEP
#define WALK_DEEP 0  // 1: a heavy walker loads statuses two windows ahead, records three (C3h 121.7 M/s against 124.1)
#endif
#ifndef WALK_PEND_NOW
#define WALK_PEND_NOW 1  // 0: a heavy walker polls an open Y leg's status before taking it as pending (C3h 94.2 against 99.1)
#endif

#define WALK_BIG (1LL << 62)  // a position whose outcome is known: "always" (+) / "never" (−)

__device__ static inline u32 fl_combine(u32 vd, u32 vc) {  // the unit's status from its two checks
    if (vd == BV_FAIL) return BS_FAIL_CREDITS;
    if (vd == BV_PASS && vc == BV_FAIL) return BS_FAIL_DEBITS;
    if (vd == BV_PASS && vc == BV_PASS) return BS_OK;
    return BS_UNK;
}
__device__ static inline u32 fl_ld32(const u32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ static inline void fl_st32(u32* p, u32 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Ordered compaction of [0, n) over the grid: emit(i, k) for the k-th i (in order) with pred(i).
// Every workgroup gets the total.  Two grid barriers; false if the kernel stalled.
template <class Pred, class Emit>
__device__ static inline bool fl_compact(const FlowArgs& F, Globals* g, u32 n, u32& gen, u32* s_wf, u32& total,
                                         Pred pred, Emit emit) {
    const u32 NT = FLOW_THREADS, tid = threadIdx.x, G = FL_G, lane = tid & 63, wave = tid >> 6;
    const u32 ut = ((n + G - 1) / G + NT - 1) / NT * NT;
    const u32 u0 = min(n, FL_B * ut), u1 = min(n, u0 + ut);
    u32 cnt = 0;
    for (u32 c0 = u0; c0 < u1; c0 += NT) {
        const u32 i = c0 + tid;
        cnt += __syncthreads_count(i < u1 && pred(i));
    }
    if (tid == 0) F.b_blk[5 * FL_B] = cnt;
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;
    u32 off = 0;
    total = 0;
    for (u32 b = 0; b < G; b++) {
        const u32 c = (u32)F.b_blk[5 * b];
        off += b < FL_B ? c : 0;
        total += c;
    }
    for (u32 c0 = u0; c0 < u1; c0 += NT) {
        const u32 i = c0 + tid;
        const bool p = i < u1 && pred(i);
        const u64 m = __ballot(p);
        if (lane == 0) s_wf[wave] = __popcll(m);
        __syncthreads();
        u32 before = 0, tot = 0;
        for (u32 w = 0; w < NT / 64; w++) {
            before += w < wave ? s_wf[w] : 0;
            tot += s_wf[w];
        }
        if (p) emit(i, off + before + __popcll(m & ((1ULL << lane) - 1)));
        off += tot;
        __syncthreads();
    }
    fl_grid_sync(g, G, gen, F);
    return !fl_stalled(g);
}

// A window's inputs beyond its records: for a Y leg and for a check paired with another open one,
// the unit's status; for the paired check, the other side's verdict so far (b_vw).
__device__ static inline void fl_walk_status(const FlowArgs& F, const WalkRec& r, bool valid, u32& st, u32& vw) {
    const bool isx = r.kind & BT_X, cr = r.kind & BT_CR;
    const bool pair = valid && isx && (cr ? (r.kind >> 8) & 15 : (r.kind >> 12) & 15) == BV_UNK;
    st = BS_UNK;
    vw = 0;
    if ((valid && !isx) || pair) st = fl_ld32(&F.b_st[r.u]);
    if (pair) vw = fl_ld32(&F.b_vw[r.u]);
}

// The heavy walker's loads, issued unconditionally (a clamped index: lanes past the segment read its
// last record, a valid address) and raw, their lanes selected only where a window consumes them: a
// load under a branch leaves the compiler unsure how many loads are in flight, so it waits for all
// of them (vmcnt(0)) at the next use of any, and a select right after a load waits for that load —
// either put a full memory round trip on every window of the critical walker.
__device__ static inline WalkRec fl_walk_rec(const WalkRec* R, u32 s0, u32 n_seg, u32 i) {
    return R[s0 + min(i, n_seg - 1)];
}
__device__ static inline WalkRec fl_walk_rec_valid(WalkRec x, bool ok) {  // lanes past the segment: zero
    x.base = ok ? x.base : 0;
    x.a = ok ? x.a : 0;
    x.u = ok ? x.u : 0;
    x.kind = ok ? x.kind : 0;
    x.head = ok ? x.head : 0;
    return x;
}
__device__ static inline void fl_walk_status_raw(const FlowArgs& F, const WalkRec& r, u32& st, u32& vw) {
    st = fl_ld32(&F.b_st[r.u]);
    vw = fl_ld32(&F.b_vw[r.u]);
}
__device__ static inline void fl_walk_status_sel(const WalkRec& r, bool valid, u32& st, u32& vw) {  // as fl_walk_status
    const bool isx = r.kind & BT_X, cr = r.kind & BT_CR;
    const bool pair = valid && isx && (cr ? (r.kind >> 8) & 15 : (r.kind >> 12) & 15) == BV_UNK;
    st = (valid && !isx) || pair ? st : (u32)BS_UNK;
    vw = pair ? vw : 0;
}

struct WalkStats {
    u64 windows = 0, stops = 0, blocks = 0, loop_ticks = 0, block_ticks = 0;
#if WALK_CNT
    u64 cnt[4] = {};  // A/B builds: the critical walker's positions by path (walk_dbg)
#endif
#if WALK_PROF
    u64 pt[4] = {};   // A/B builds: ticks in the window's fetch, setup, loop and end (walk_dbg)
    u64 pt_last = 0;
#endif
};

// One step of the 32-bit chain on the scalar unit: t = v + dc; if t >= 0 { dc += e; okm |= bit }.
// Written out so the compare's SCC feeds both selects (the compiler materialises the bool instead).
__device__ static inline void fl_step32(int v, int e, u64 bit, int& dc, u64& okm) {
    int t;
    u64 y;
    asm("s_add_i32 %2, %4, %0\n\t"
        "s_cmp_ge_i32 %2, 0\n\t"
        "s_cselect_b32 %2, %5, 0\n\t"
        "s_cselect_b64 %3, %6, 0\n\t"
        "s_add_i32 %0, %0, %2\n\t"
        "s_or_b64 %1, %1, %3"
        : "+s"(dc), "+s"(okm), "=&s"(t), "=&s"(y)
        : "s"(v), "s"(e), "s"(bit)
        : "scc");
}

// The 32-bit chain over lanes [j, e) of one account: lane i is ok iff v32 + dc >= 0, and an ok lane
// adds d32 to dc; okm collects the outcomes.  Four lanes a step: their inputs read ahead of the
// chain (a readlane's result reaches the scalar unit late), then the chain itself.
// Inclusive prefix sum over the wave's 64 lanes: within each row of 16 lanes by DPP row shifts
// (a lane whose source is outside its row adds 0), then the rows' totals carried on.
__device__ static inline int fl_scan32(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    const int r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31);
    const int r2 = __builtin_amdgcn_readlane(x, 47);
    const u32 row = (threadIdx.x & 63) >> 4;
    return x + (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
}

// The in-order walk of lanes [j, e) (lane i ok iff v32 + dc >= 0; an ok lane adds d32 to dc) in
// parallel, by RUNS.  With P the prefix sum of the lanes' deltas (one scan) and w = v32 + P, a run of
// ok lanes from s on base dc fails first at the first lane k >= s with w < P(s) - dc; a run of failed
// lanes from k (their deltas left out, so dc stays) ends at the first lane with v32 + dc >= 0.  So
// the walk costs a scan and a ballot per run, not a scalar step per lane (a lone wave issues one
// instruction per four cycles: the scalar chain cost the critical walker ~50 ns a position).
// p32 > 0 (pending credits): a lane that fails without them but passes with them stops the walk;
// returns where (e: none).  Every sum stays below 2^31 in magnitude: |v32| <= 2^30, and dc plus
// any partial sum of one window's deltas (each below 2^24) is below 2^30.
__device__ static inline u64 fl_from(u32 s) { return s >= 64 ? 0 : ~0ULL << s; }
__device__ static inline u32 fl_runs32(int v32, int d32, u32 j, u32 e, int& dc, u64& okm, int p32,
                                       u64* trips = nullptr) {
    const u32 lane = threadIdx.x & 63;
    const bool in = lane >= j && lane < e;
    const int x = in ? d32 : 0;
    const int S = fl_scan32(x);
    const int P = S - x;  // the deltas of [j, lane)
    const int w = v32 + P;
    const u64 inm = __ballot(in);
    int B = __builtin_amdgcn_readfirstlane(dc);
    u32 s = j;
    int Ps = 0;
    for (;;) {
        if (trips) (*trips)++;
        const int c = Ps - B;  // lane k >= s of the ok run fails iff v32 + B + P(k) - P(s) < 0
        const u64 bad = __ballot(w < c) & inm & fl_from(s);
        if (!bad) {
            okm |= inm & fl_from(s);
            dc = B + (e > j ? __builtin_amdgcn_readlane(S, e - 1) : 0) - Ps;
            return e;
        }
        const u32 k = (u32)__builtin_ctzll(bad);
        okm |= inm & fl_from(s) & ~fl_from(k);
        B += __builtin_amdgcn_readlane(P, k) - Ps;
        if (p32 && __builtin_amdgcn_readlane(w, k) + p32 >= c) {  // the pending credits could flip it
            dc = B;
            return k;
        }
        const u64 nxt = __ballot(v32 + B + p32 >= 0) & inm & fl_from(k + 1);  // the failed run's end
        if (!nxt) {
            dc = B;
            return e;
        }
        const u32 q = (u32)__builtin_ctzll(nxt);
        if (p32 && __builtin_amdgcn_readlane(v32, q) + B < 0) {  // passes only with the pending credits
            dc = B;
            return q;
        }
        s = q;
        Ps = __builtin_amdgcn_readlane(P, q);
    }
}

__device__ static inline void fl_chain32(int v32, int d32, u32 j, u32 e, int& dc, u64& okm, u64* trips = nullptr) {
    // Wave-uniform by construction; said so, or the compiler may keep them in vector registers.
    j = __builtin_amdgcn_readfirstlane(j);
    e = __builtin_amdgcn_readfirstlane(e);
    dc = __builtin_amdgcn_readfirstlane(dc);
    okm = fl_rl64(okm, 0);
#if WALK_PAR
    (void)fl_runs32(v32, d32, j, e, dc, okm, 0, trips);
    return;
#endif
    for (; j + 4 <= e; j += 4) {
        const int v0 = __builtin_amdgcn_readlane(v32, j), v1 = __builtin_amdgcn_readlane(v32, j + 1);
        const int v2 = __builtin_amdgcn_readlane(v32, j + 2), v3 = __builtin_amdgcn_readlane(v32, j + 3);
        const int e0 = __builtin_amdgcn_readlane(d32, j), e1 = __builtin_amdgcn_readlane(d32, j + 1);
        const int e2 = __builtin_amdgcn_readlane(d32, j + 2), e3 = __builtin_amdgcn_readlane(d32, j + 3);
        const u64 bit = 1ULL << j;
        __builtin_amdgcn_sched_barrier(0);  // every read issued before the chain starts
        fl_step32(v0, e0, bit, dc, okm);
        fl_step32(v1, e1, bit << 1, dc, okm);
        fl_step32(v2, e2, bit << 2, dc, okm);
        fl_step32(v3, e3, bit << 3, dc, okm);
    }
    for (; j < e; j++) {
        fl_step32(__builtin_amdgcn_readlane(v32, j), __builtin_amdgcn_readlane(d32, j), 1ULL << j, dc, okm);
    }
}

// The in-order walk of lanes [j, e) of one account from its running sum d: lane i is ok iff
// v + d >= 0, and an ok lane adds dl to d; okm collects the outcomes.  When every |dl| of the run is
// below 2^24 the run is walked in 32 bits, relative to d at its start (|sum of dl| < 2^30): each v + d0
// is clamped to +-2^30, which keeps its sign against any partial sum, so every outcome is the same.
__device__ static inline bool fl_walk_run(i64 v, i64 dl, u32 j, u32 e, i64& d, u64& okm, u64* trips = nullptr) {
    const u32 lane = threadIdx.x & 63;
    const bool in = lane >= j && lane < e;
    if (!__ballot(in && (dl >= (1LL << 24) || dl <= -(1LL << 24)))) {
        const i64 vv = (i64)((u64)v + (u64)d);  // the true value fits
        const int v32 = (int)(vv > (1LL << 30) ? (1LL << 30) : vv < -(1LL << 30) ? -(1LL << 30) : vv);
        const int d32 = (int)dl;
        int dd = 0;
        fl_chain32(v32, d32, j, e, dd, okm, trips);
        d += dd;
        return true;
    }
    for (; j < e; j++) {
        const u64 vj = fl_rl64((u64)v, j), dj = fl_rl64((u64)dl, j);
        // ok iff v + d >= 0: the sign of the sum (its true value fits in 64 bits)
        const bool ok = (int)(u32)((vj + (u64)d) >> 32) >= 0;
        d = (i64)((u64)d + (ok ? dj : 0));
        okm |= ok ? 1ULL << j : 0;
    }
    return false;
}

struct WalkCarry {  // a heavy walker's pending credits, carried from one window to the next
    u32 u = 0;        // lane i: the unit of carried leg i
    u32 st = BS_UNK;  // lane i: its status as loaded at the window's start
    i64 a = 0;        // lane i: its amount
    u64 mask = 0;     // the carried legs
    i64 dp = 0;       // their amounts' sum
};

// Resolves one window of n <= 64 positions (lane j: position j) in order from the running sum d
// (wave-uniform), publishing the statuses its checks decide.  Returns the positions decided: n, or
// the position of a partner that has not decided yet (the walk resumes there).
// wait (a heavy walker: its wave walks this one segment) keeps a stopped window in place, polling the
// partner's status, instead of returning; a light wave returns and visits its other segments.
__device__ static inline u32 fl_walk_window(const FlowArgs& F, const WalkRec& r, u32 st, u32 vw, u32 s, u32 n,
                                            i64& d, WalkStats& ws, Globals* g = nullptr, bool wait = false,
                                            WalkCarry* cw = nullptr) {
    const u32 lane = threadIdx.x & 63;
    const bool valid = lane >= s && lane < n;  // positions [s, n): the window from where it stopped
    const bool isx = r.kind & BT_X, isy = valid && !isx, cr = r.kind & BT_CR;
    const u32 vd = (r.kind >> 8) & 15, vc = (r.kind >> 12) & 15;
    u32 oth = cr ? vd : vc;
    // A position is SIMPLE when its outcome follows from d alone: a check whose partner side is
    // known (v = slack − amount: ok iff v + d >= 0; its outcome is this side's verdict), or a leg
    // whose unit is decided (v = ±BIG).  The others stop the scalar walk: a Y leg of an open unit, a
    // check paired with an open one.
    bool simple = true, check = false;
    i64 v = 0, dl = 0;
    auto classify = [&]() {
        if (valid && isx && oth == BV_UNK && st == BS_UNK) oth = cr ? (vw & 3) : ((vw >> 2) & 3);
        simple = true;
        check = false;
        v = 0;
        dl = 0;
        if (!valid) {
            simple = false;
        } else if (st != BS_UNK) {
            v = st == BS_OK ? WALK_BIG : -WALK_BIG;
            dl = isx ? -r.a : r.a;
        } else if (isy || oth == BV_UNK) {
            simple = false;
        } else {
            check = true;
            v = r.base - r.a;
            dl = oth == BV_FAIL ? 0 : -r.a;  // the other side failed: no delta here either way
        }
    };
#if WALK_PROF
    if (wait) {
        const u64 t = fl_now();
        ws.pt[0] += t - ws.pt_last;
        ws.pt_last = t;
    }
#endif
    classify();
    u64 smask = __ballot(simple);
    const u64 vmask = n == 64 ? ~0ULL : ((1ULL << n) - 1);
    u64 okm = 0;  // lane j's outcome in the walk (a check's own verdict)
    u32 j = s, m = n, pub = s;  // [s, pub): published while waiting in place
    // A waiting walker goes past a Y leg whose unit is still open: the leg is PENDING (pmask), its
    // amount in dp, and d stays the sum without it.  A later check is decided if it decides the same
    // way with and without every pending credit (d and d + dp); only a check that it would flip
    // waits — for the pending units, not for the first of them.
    // With cw (a heavy walker), the window leaves its pending credits to the next ones instead of
    // waiting for them (cmask[k]: the ones carried in, set 0 the oldest; dp counts them all).
    u64 pmask = 0, cmask[WALK_NC];
#pragma unroll
    for (int k = 0; k < WALK_NC; k++) cmask[k] = cw ? cw[k].mask : 0;
    i64 dp = cw ? cw[0].dp : 0;
    auto publish_to = [&](u32 upto) {  // this window's checks in [pub, upto)
        if (check && valid && lane >= pub && lane < upto) {
            const u32 mine = (okm >> lane) & 1 ? BV_PASS : BV_FAIL;
            fl_st32(&F.b_st[r.u], cr ? fl_combine(oth, mine) : fl_combine(mine, oth));
        }
        pub = max(pub, upto);
    };
    // The pending units decided by now (sx: this window's, sc: the carried ones' statuses): their
    // amounts leave dp, and the ok ones' enter d.
    // A few lanes: summed on the scalar unit (a shuffle reduction is 12 dependent LDS permutes).
    auto settle_set = [&](u64& mask, u32 sx, i64 a_lane) {
        const bool known = ((mask >> lane) & 1) && sx != BS_UNK;
        const u64 km = __ballot(known);
        if (!km) return;
        const u64 okk = __ballot(known && sx == BS_OK);
        for (u64 m = km; m; m &= m - 1) {
            const u32 k = (u32)__builtin_ctzll(m);
            const i64 a = (i64)fl_rl64((u64)a_lane, k);
            if ((okk >> k) & 1) d += a;
            dp -= a;
        }
        mask &= ~km;
    };
    auto pend = [&]() {
        u64 m = pmask;
#pragma unroll
        for (int k = 0; k < WALK_NC; k++) m |= cmask[k];
        return m;
    };
    auto settle = [&]() {  // polls every pending unit once
        u32 sx = BS_UNK;
        if ((pmask >> lane) & 1) sx = fl_ld32(&F.b_st[r.u]);
        u32 sc[WALK_NC];
#pragma unroll
        for (int k = 0; k < WALK_NC; k++) {
            sc[k] = BS_UNK;
            if (cw && ((cmask[k] >> lane) & 1)) sc[k] = fl_ld32(&F.b_st[cw[k].u]);
        }
        settle_set(pmask, sx, r.a);
        if (cw) {
#pragma unroll
            for (int k = 0; k < WALK_NC; k++) settle_set(cmask[k], sc[k], cw[k].a);
        }
    };
    auto wait_until = [&](auto decided) {  // publish, then poll the pending units until decided()
        publish_to(j);
        ws.blocks++;
        const u64 w0 = fl_now();
        settle();
        while (!decided()) {
            __builtin_amdgcn_s_sleep(1);
            settle();
            if (__builtin_amdgcn_readfirstlane(!decided() && (fl_expired(F, w0) || fl_stalled(g)))) {
                if (lane == 0) tb_panic(g, PANIC_FLOW_STALL);
                pmask = 0;  // give up (the pass is lost to the panic)
#pragma unroll
                for (int k = 0; k < WALK_NC; k++) cmask[k] = 0;
                dp = 0;
                break;
            }
        }
        ws.block_ticks += fl_now() - w0;
    };
#if WALK_PROF
    if (wait) {
        const u64 t = fl_now();
        ws.pt[1] += t - ws.pt_last;
        ws.pt_last = t;
    }
#endif
    while (j < n) {
        const u64 bar = ~smask & vmask & (~0ULL << j);
        const u32 b = bar ? (u32)__builtin_ctzll(bar) : n;
        // Bounded walk while credits are pending: d without them, d + dp with them.  In 32 bits when
        // the stretch's moves and the pending credits stay below 2^29 (amounts below 2^22): v + d
        // clamped to +-2^29 keeps both signs.
        if (pend() && j < b && dp < (1LL << 28) &&
            !__ballot(lane >= j && lane < b && (dl >= (1LL << 22) || dl <= -(1LL << 22)))) {
            const i64 vv = (i64)((u64)v + (u64)d);
            const int v32 = (int)(vv > (1LL << 29) ? (1LL << 29) : vv < -(1LL << 29) ? -(1LL << 29) : vv);
            const int d32 = (int)dl, p32 = (int)dp;
            int dd = 0;
            u32 i = j;
#if WALK_PAR
#if WALK_CNT
            i = fl_runs32(v32, d32, j, b, dd, okm, p32 > 0 ? p32 : 0, wait ? &ws.cnt[2] : nullptr);
#else
            i = fl_runs32(v32, d32, j, b, dd, okm, p32 > 0 ? p32 : 0);
#endif
#else
            for (; i < b; i++) {
                const int vi = __builtin_amdgcn_readlane(v32, i), di = __builtin_amdgcn_readlane(d32, i);
                if (vi + dd >= 0) {
                    dd += di;
                    okm |= 1ULL << i;
                } else if (vi + dd + p32 >= 0) {
                    break;  // the pending credits could flip it
                }
            }
#endif
            d += dd;

            j = i;
        }
        while (pend() && j < b) {  // bounded walk: d without the pending credits, d + dp with them
            const i64 vj = (i64)fl_rl64((u64)v, j), dj = (i64)fl_rl64((u64)dl, j);
            const bool lo = (i64)((u64)vj + (u64)d) >= 0, hi = (i64)((u64)vj + (u64)d + (u64)dp) >= 0;
            if (lo != hi) {
                wait_until([&]() {
                    return !pend() ||
                           ((i64)((u64)vj + (u64)d) >= 0) == ((i64)((u64)vj + (u64)d + (u64)dp) >= 0);
                });
                continue;
            }
            if (lo) {
                d += dj;
                okm |= 1ULL << j;
            }

            j++;
        }
#if WALK_CNT
        // A/B builds: runs walked (fl_runs32 trips), loop iterations, bounded-walk trips, windows
        const bool r32 = fl_walk_run(v, dl, j, b, d, okm, wait ? &ws.cnt[0] : nullptr);
        (void)r32;
        if (wait) ws.cnt[1]++;
#else
        fl_walk_run(v, dl, j, b, d, okm);
#endif
        j = b;
        if (b == n) break;
        // Position b: its partner was open when the window loaded.  The window's other open
        // positions after b re-read their statuses in the same round trip as b's poll (they were
        // loaded a window ahead; a partner walker has usually decided them since): each one decided
        // by now walks as a simple position instead of stopping the walk again.
        ws.stops++;
        const u32 bu = __builtin_amdgcn_readlane(r.u, b), bk = __builtin_amdgcn_readlane(r.kind, b);
        const i64 ba = (i64)fl_rl64((u64)r.a, b);
#if WALK_PEND_NOW
        if (wait && !(bk & BT_X)) {
            // A waiting walker takes an open Y leg as pending at once, without polling its status: the
            // pending statuses are read together, in one round trip, when a check needs them and at
            // the window's end (a poll per stop was the heavy walker's main cost).
            pmask |= 1ULL << b;
            dp += ba;
            j = b + 1;
            continue;
        }
#endif
        const bool refresh = valid && lane > b && !simple;
        if (refresh) {
            st = fl_ld32(&F.b_st[r.u]);
            if (isx) vw = fl_ld32(&F.b_vw[r.u]);
        }
        if ((bk & BT_X) && pend()) wait_until([&]() { return !pend(); });  // a paired check needs the exact d
        const i64 bb = (i64)fl_rl64((u64)r.base, b);
        // The unit's status now: a paired check ORs this side's verdict in first (whoever completes
        // the pair publishes; a partner that walked its side as a plain check publishes the status,
        // not its bit).  BS_UNK: still open.
        const bool side_ok = (bk & BT_X) && (i64)((u64)bb + (u64)d) >= ba;
        auto poll = [&]() -> u32 {
            u32 old = 0, s2 = 0;
            const u32 mine = (bk & BT_X) ? (side_ok ? BV_PASS : BV_FAIL) << ((bk & BT_CR) ? 2 : 0) : 0;
            if (lane == 0) {
                if (bk & BT_X) old = __hip_atomic_fetch_or(&F.b_vw[bu], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s2 = fl_ld32(&F.b_st[bu]);
            }
            const u32 both = __builtin_amdgcn_readfirstlane(old) | mine;
            const u32 fin = (bk & BT_X) ? fl_combine(both & 3, (both >> 2) & 3) : BS_UNK;
            if (fin != BS_UNK) {
                if (lane == 0) fl_st32(&F.b_st[bu], fin);
                return fin;
            }
            return __builtin_amdgcn_readfirstlane(s2);
        };
        u32 fin = poll();
        if (__ballot(refresh)) {  // the refreshed positions after b, classified again
            if (refresh) classify();
            smask = __ballot(simple);
        }
        // A paired check whose own side failed moves nothing here, whatever the other side says.
        const bool moot = (bk & BT_X) && !side_ok;
        if (fin == BS_UNK && !(bk & BT_X) && wait) {  // an open Y leg: pending (above)
            pmask |= 1ULL << b;
            dp += ba;
            j = b + 1;
            continue;
        }
        if (fin == BS_UNK && !moot && wait) {
            // Publish what this window decided so far (the partner may be waiting on it), then wait.
            if (check && valid && lane >= pub && lane < b) {
                const u32 mine = (okm >> lane) & 1 ? BV_PASS : BV_FAIL;
                fl_st32(&F.b_st[r.u], cr ? fl_combine(oth, mine) : fl_combine(mine, oth));
            }
            pub = b;
            ws.blocks++;
            const u64 w0 = fl_now();
            while (fin == BS_UNK) {
                __builtin_amdgcn_s_sleep(1);
                fin = poll();
                // (readfirstlane: an atomic load counts as divergent, which would make the walk's
                // sums vector values)
                if (__builtin_amdgcn_readfirstlane(fin == BS_UNK && (fl_expired(F, w0) || fl_stalled(g)))) {
                    if (lane == 0) tb_panic(g, PANIC_FLOW_STALL);
                    break;
                }
            }
            ws.block_ticks += fl_now() - w0;
        }
        if (fin == BS_UNK && !moot) {
            m = b;  // blocked: the partner has not decided yet
            break;
        }
        if (fin == BS_OK) d += (bk & BT_X) ? -ba : ba;
        j = b + 1;
    }
#if WALK_PROF
    if (wait) {
        const u64 t = fl_now();
        ws.pt[2] += t - ws.pt_last;
        ws.pt_last = t;
    }
#endif
    if (cw) {
        // The oldest carried legs, with their statuses as loaded at the start of the window after
        // theirs (fl_walk_heavy; WALK_NC windows ago): the ones still open are polled until
        // decided.  The others move down, and this window's pending legs carry on (no round trip
        // when the partners kept up).
        settle_set(cmask[0], cw[0].st, cw[0].a);
        if (cmask[0]) wait_until([&]() { return !cmask[0]; });
#pragma unroll
        for (int k = 0; k + 1 < WALK_NC; k++) {
            cw[k].u = cw[k + 1].u;
            cw[k].a = cw[k + 1].a;
            cw[k].st = cw[k + 1].st;
            cw[k].mask = cmask[k + 1];
        }
        cw[WALK_NC - 1].u = r.u;
        cw[WALK_NC - 1].a = r.a;
        cw[WALK_NC - 1].st = BS_UNK;  // (loaded at the next window's start)
        cw[WALK_NC - 1].mask = pmask;
        cw[0].dp = dp;
    } else if (pmask) {
        wait_until([&]() { return !pmask; });  // the window leaves with an exact d
    }
    ws.windows++;
#if WALK_CNT
    if (wait) ws.cnt[3]++;
#endif
    // Publish the checks walked in the scalar loop, once per window: a status poll issued after a
    // store waits for it (vmcnt counts both), so publishing in smaller pieces ahead of the stops
    // cost more than it saved partners (C3h 66.5 -> 54 M/s with 16-position pieces).
    if (check && valid && lane >= pub && lane < m) {
        const u32 mine = (okm >> lane) & 1 ? BV_PASS : BV_FAIL;
        fl_st32(&F.b_st[r.u], cr ? fl_combine(oth, mine) : fl_combine(mine, oth));
    }
#if WALK_PROF
    if (wait) {
        const u64 t = fl_now();
        ws.pt[3] += t - ws.pt_last;
        ws.pt_last = t;
    }
#endif
    return m;
}

// A light segment [s0, s0 + n_seg) from cursor c with running sum d (wave-uniform) until it is done
// or blocked.  Returns the positions decided.
__device__ static inline u32 fl_walk_segment(const FlowArgs& F, const WalkRec* R, u32 s0, u32 n_seg, u32& c, i64& d,
                                             WalkStats& ws) {
    const u32 lane = threadIdx.x & 63;
    // Wave-uniform by construction; told to the compiler, so the walk runs on the scalar unit.
    s0 = __builtin_amdgcn_readfirstlane(s0);
    n_seg = __builtin_amdgcn_readfirstlane(n_seg);
    c = __builtin_amdgcn_readfirstlane(c);
    d = (i64)fl_rl64((u64)d, 0);
    u32 done = 0;
    while (c < n_seg) {
        const u32 n = min(64u, n_seg - c);
        WalkRec r = {};
        if (lane < n) r = R[s0 + c + lane];
        u32 st, vw;
        fl_walk_status(F, r, lane < n, st, vw);
        const u32 m = fl_walk_window(F, r, st, vw, 0, n, d, ws);
        c += m;
        done += m;
        if (m < n) break;
    }
    return done;
}

// A heavy segment, walked to its end by one wave with the next windows in flight: the records two
// windows ahead and the statuses one window ahead (a status read early may be stale — still open —
// which only stops the walk there; the stopped window is retried in place, the stopping position
// re-reading its status).
__device__ static inline bool fl_walk_heavy(const FlowArgs& F, Globals* g, const WalkRec* R, u32 s0, u32 n_seg,
                                            WalkStats& ws) {
    const u32 lane = threadIdx.x & 63;
    s0 = __builtin_amdgcn_readfirstlane(s0);
    n_seg = __builtin_amdgcn_readfirstlane(n_seg);
    i64 d = 0;
    u64 wb = 0, tblock = 0;
#if WALK_CARRY
    WalkCarry cw[WALK_NC];
#endif
#if WALK_PROF
    ws.pt_last = fl_now();
#endif
    WalkRec r0 = fl_walk_rec(R, s0, n_seg, lane), r1 = fl_walk_rec(R, s0, n_seg, 64 + lane);
    u32 st0, vw0;
    fl_walk_status_raw(F, r0, st0, vw0);
#if WALK_DEEP
    // Statuses two windows ahead, records three.
    WalkRec r2 = fl_walk_rec(R, s0, n_seg, 128 + lane);
    u32 st1, vw1;
    fl_walk_status_raw(F, r1, st1, vw1);
#endif
    for (u32 c = 0; c < n_seg; c += 64) {
        const u32 n = min(64u, n_seg - c);
#if WALK_DEEP
        const WalkRec r3 = fl_walk_rec(R, s0, n_seg, c + 192 + lane);
        u32 st2, vw2;
        fl_walk_status_raw(F, r2, st2, vw2);
#else
        const WalkRec r2 = fl_walk_rec(R, s0, n_seg, c + 128 + lane);
        u32 st1, vw1;
        fl_walk_status_raw(F, r1, st1, vw1);
#endif
#if WALK_CARRY
        // The newest carried legs' statuses, loaded now and read WALK_NC window ends later.
        cw[WALK_NC - 1].st = fl_ld32(&F.b_st[cw[WALK_NC - 1].u]);  // (masked where it is read)
        WalkCarry* cwp = cw;
#else
        WalkCarry* cwp = nullptr;
#endif
        // This window's records and statuses (loaded one and two windows ago), lanes selected now.
        const WalkRec rw = fl_walk_rec_valid(r0, c + lane < n_seg);
        u32 stw = st0, vww = vw0;
        fl_walk_status_sel(rw, c + lane < n_seg, stw, vww);
        for (u32 s = 0;;) {
            const u32 m = fl_walk_window(F, rw, stw, vww, s, n, d, ws, g, true, cwp);
            if (m > s && tblock) {
                ws.block_ticks += wall_clock64() - tblock;
                tblock = 0;
                wb = 0;
            }
            s = m;
            if (s >= n) break;
            ws.blocks++;
            const u64 now = fl_now();
            if (!tblock) tblock = now;
            if (!wb) wb = now;
            if (now - wb > F.stall_ticks) {
                const u32 bu = __builtin_amdgcn_readlane(rw.u, s), bk = __builtin_amdgcn_readlane(rw.kind, s);
                if (lane == 0) {
                    g->walk_dbg[0] = 1 | ((u64)bk << 8) | ((u64)c << 32);
                    g->walk_dbg[1] = bu;
                    g->walk_dbg[2] = fl_ld32(&F.b_st[bu]);
                    g->walk_dbg[3] = fl_ld32(&F.b_vw[bu]);
                    tb_panic(g, PANIC_FLOW_STALL);
                }
                return false;
            }
            if (fl_stalled(g)) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        r0 = r1;
        r1 = r2;
        st0 = st1;
        vw0 = vw1;
#if WALK_DEEP
        r2 = r3;
        st1 = st2;
        vw1 = vw2;
#endif
    }
    return true;
}

// ---- the merged heavy walk --------------------------------------------------------------------------
// Heavy segments couple densely (the hottest limit accounts pay each other: thousands of units per
// pass carry a leg on two of them), and a walker waiting on another through global memory loses
// microseconds each time.  So up to WALK_MERGE_MAX heavy segments are walked TOGETHER by one wave,
// in event order over the units that have a leg on any of them: lane i holds heavy segment i's
// running sum, a run of consecutive units on one heavy account is walked with that sum on the scalar
// unit, and a unit on two heavy accounts updates both.  Only units whose other check is on a light
// segment still wait for that segment's walker.
#define WALK_MERGE_MAX 63
// Measured on the adversarial C3 (bench --workload c3h): a wave per heavy segment, 67.5 M
// transfers/s, against 36 M/s merged — the single merged wave walks every heavy unit itself, while
// separate walkers overlap and only stop at the units they share.  Merging stays for A/B runs.
#ifndef WALK_MERGE_DEFAULT
#define WALK_MERGE_DEFAULT 0
#endif
struct HotRec {  // an undecided unit with a leg on a heavy segment, in event order
    i64 bd, bc;  // the debit / credit leg's base: Y − X with the decided units before it
    i64 a;       // amount
    u32 u;       // unit
    u32 info;    // HI_*
};
enum : u32 {
    HI_HD = 0x3Fu,        // bits 0-5: heavy index + 1 of the debit leg (0: light, or no leg)
    HI_HC_SHIFT = 6,      // bits 6-11: the same for the credit leg
    HI_DP = 1u << 12,     // the debit leg is a listed position (a limit account's)
    HI_DX = 1u << 13,     // ... and carries the unit's debit-side check
    HI_CP = 1u << 14,     // the credit leg is a listed position
    HI_CX = 1u << 15,     // ... and carries the credit-side check (credits_must_not_exceed_debits)
    HI_VD_SHIFT = 16,     // the unit's verdicts when listed (BV_*)
    HI_VC_SHIFT = 20,
};

// The generic resolution of stream unit j (a unit on two heavy segments, or one whose other check is
// on a light segment): its checks from the absolute running sums, the light side's verdict read
// (or waited for), the status published when complete.  d(h) = dreg + rel of lane h - 1; an ok unit
// moves rel.  Returns false when the unit waits on a light walker.
template <typename T>  // int: rel in a 32-bit window; i64: a window with large amounts
__device__ static inline bool fl_walk_hot_unit(const FlowArgs& F, const HotRec& r, u32 j, i64 dreg, T& rel,
                                               WalkStats& ws) {
    const u32 lane = threadIdx.x & 63;
    ws.stops++;
    const u32 u = __builtin_amdgcn_readlane(r.u, j), inf = __builtin_amdgcn_readlane(r.info, j);
    const u32 jhd = inf & HI_HD, jhc = (inf >> HI_HC_SHIFT) & HI_HD;
    const i64 a = (i64)fl_rl64((u64)r.a, j);
    const i64 dd = jhd ? (i64)(fl_rl64((u64)dreg, jhd - 1) + fl_rl64((u64)(i64)rel, jhd - 1)) : 0;
    const i64 dc = jhc ? (i64)(fl_rl64((u64)dreg, jhc - 1) + fl_rl64((u64)(i64)rel, jhc - 1)) : 0;
    u32 vd = (inf >> HI_VD_SHIFT) & 15, vc = (inf >> HI_VC_SHIFT) & 15, mine = 0;
    if ((inf & HI_DX) && jhd) {
        vd = (i64)((u64)fl_rl64((u64)r.bd, j) + (u64)dd) >= a ? BV_PASS : BV_FAIL;
        mine |= vd;
    }
    if ((inf & HI_CX) && jhc) {
        vc = (i64)((u64)fl_rl64((u64)r.bc, j) + (u64)dc) >= a ? BV_PASS : BV_FAIL;
        mine |= vc << 2;
    }
    u32 fin = fl_combine(vd, vc);
    if (fin == BS_UNK) {
        // A light side is open: ours go in (b_vw); whoever completes the pair publishes.
        u32 old = 0, s2 = 0;
        if (lane == 0) {
            old = __hip_atomic_fetch_or(&F.b_vw[u], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s2 = fl_ld32(&F.b_st[u]);
        }
        const u32 both = __builtin_amdgcn_readfirstlane(old) | mine;
        fin = fl_combine(both & 3, (both >> 2) & 3);
        if (fin == BS_UNK) fin = __builtin_amdgcn_readfirstlane(s2);
        if (fin == BS_UNK) {
            // Heavy legs move only if the unit is ok: a failed side settles it for them.
            return (both & 3) == BV_FAIL || ((both >> 2) & 3) == BV_FAIL;
        }
    }
    if (lane == 0) fl_st32(&F.b_st[u], fin);
    if (fin == BS_OK) {
        if (jhd && lane == jhd - 1) rel += (inf & HI_DX) ? -(T)a : (T)a;
        if (jhc && lane == jhc - 1) rel += (inf & HI_CX) ? -(T)a : (T)a;
    }
    return true;
}

// Resolves stream units [s, n) of a window (lane j: unit j) in event order.  dreg (lane i) is heavy
// segment i's running sum.  Every amount of the window is below 2^24 (the caller checks), so the
// window's moves stay below 2^30 per segment and the walk runs in 32 bits relative to dreg: rel
// (lane i) is segment i's move so far in the window, dc the current segment's.  A unit with one heavy
// leg whose outcome follows from its sum alone is SIMPLE (see fl_walk_window): one add, compare and
// select on the scalar unit, switching segments where consecutive units change segment.  The others
// go through fl_walk_hot_unit.  Returns the units decided (n, or the unit waiting on a light walker).
__device__ static inline u32 fl_walk_hot_window(const FlowArgs& F, const HotRec& r, u32 s, u32 n, i64& dreg,
                                                WalkStats& ws) {
    const u32 lane = threadIdx.x & 63;
    const bool valid = lane >= s && lane < n;
    const u32 info = r.info;
    const u32 hd = info & HI_HD, hc = (info >> HI_HC_SHIFT) & HI_HD;
    const u32 vd0 = (info >> HI_VD_SHIFT) & 15, vc0 = (info >> HI_VC_SHIFT) & 15;
    const bool one = (hd != 0) != (hc != 0);
    const u32 h = hd ? hd : hc;
    const bool hx = hd ? (info & HI_DX) : (info & HI_CX);  // the heavy leg is a check
    const u32 oth = hd ? vc0 : vd0;                          // the other side's verdict as listed
    // Simple: the heavy leg is a check whose other side is known (a light check that was still
    // open when the unit was listed goes through fl_walk_hot_unit).
    const bool check = valid && one && hx && oth != BV_UNK;
    const i64 v = (hd ? r.bd : r.bc) - r.a, dl = oth == BV_FAIL ? 0 : -r.a;
    const u32 hs = check ? h : 0;
    // 32-bit walk: v + d at the window start, clamped to +-2^30 (keeps its sign against any move).
    const i64 d0 = (i64)__shfl((unsigned long long)dreg, (int)(hs ? hs - 1 : 0));
    const i64 vv = (i64)((u64)v + (u64)d0);
    const int v32 = (int)(vv > (1LL << 30) ? (1LL << 30) : vv < -(1LL << 30) ? -(1LL << 30) : vv);
    const int d32 = (int)dl;
    // Where the segment changes (a simple unit after another segment's, or a unit on its own).
    const u32 hprev = __shfl_up(hs, 1);
    const u64 sw = __ballot(valid && (lane == s || hs != hprev || !hs));
    int rel = 0;
    u64 okm = 0;  // the simple units' outcomes
    u32 m = n;
    for (u32 j = s; j < n;) {
        // j starts a stretch: units j .. e - 1 on one segment, or a unit on its own.
        const u32 cur = __builtin_amdgcn_readlane(hs, j);
        if (!cur) {
            const bool ok = fl_walk_hot_unit(F, r, j, dreg, rel, ws);
            if (!ok) {
                m = j;  // waits on a light walker
                break;
            }
            j++;
            continue;
        }
        const u64 next = sw & ~((2ULL << j) - 1);
        const u32 e = next ? (u32)__builtin_ctzll(next) : n;
        int dc = __builtin_amdgcn_readlane(rel, cur - 1);
        fl_chain32(v32, d32, j, e, dc, okm);
        j = e;
        if (lane == cur - 1) rel = dc;
    }
    dreg += rel;
    ws.windows++;
    // Publish the checks walked in the scalar loop.
    if (check && lane < m) {
        const u32 mine = (okm >> lane) & 1 ? BV_PASS : BV_FAIL;
        fl_st32(&F.b_st[r.u], hd ? fl_combine(mine, oth) : fl_combine(oth, mine));
    }
    return m;
}

// The same for a window with an amount of 2^24 or more: 64-bit sums, every unit on its own.
__device__ static inline u32 fl_walk_hot_window64(const FlowArgs& F, const HotRec& r, u32 s, u32 n, i64& dreg,
                                                  WalkStats& ws) {
    u32 m = n;
    for (u32 j = s; j < n; j++) {
        i64 rel = 0;
        const bool ok = fl_walk_hot_unit(F, r, j, dreg, rel, ws);
        dreg += rel;
        if (!ok) {
            m = j;
            break;
        }
    }
    return m;
}

// The merged walk over N stream units by wave 0 of workgroup 0, fed through an LDS ring by wave 1
// (WALK_RING windows ahead), so the walker itself issues no global load: its only memory operations
// are LDS reads of its windows and the fire-and-forget status stores (a load behind those would
// wait for them).  ctl[0]: windows filled, ctl[1]: windows consumed (N windows: the walker quit).
__device__ static inline void fl_walk_merged(const FlowArgs& F, Globals* g, const HotRec* H, u32 N, WalkStats& ws,
                                             u32* ctl, HotRec* ring) {
    const u32 lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    N = __builtin_amdgcn_readfirstlane(N);
    const u32 nw = (N + 63) / 64;
    if (wave == 1) {
        // The prefetcher: windows w .. w + 3 loaded together, then written to their ring slots.
        for (u32 w = 0; w < nw; w += 4) {
            const u64 w0 = fl_now();
            while (__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) + WALK_RING < min(nw, w + 4)) {
                __builtin_amdgcn_s_sleep(1);
                if (fl_expired(F, w0) || fl_stalled(g)) return;
            }
            if (__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= nw) return;  // quit
            HotRec x[4];
#pragma unroll
            for (u32 k = 0; k < 4; k++) {
                const u32 i = (w + k) * 64 + lane;
                x[k] = i < N ? H[i] : HotRec{};
            }
#pragma unroll
            for (u32 k = 0; k < 4; k++) {
                // (a slot past the last window may still hold an unconsumed one: left alone)
                if (w + k < nw) ring[((w + k) % WALK_RING) * 64 + lane] = x[k];
            }
            if (lane == 0) __hip_atomic_store(&ctl[0], min(nw, w + 4), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    }
    if (wave != 0) return;
    i64 dreg = 0;
    u64 wb = 0, tblock = 0;
    const u64 ta = wall_clock64();
    for (u32 w = 0; w < nw; w++) {
        const u64 w0 = fl_now();
        while (__hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= w) {
            __builtin_amdgcn_s_sleep(1);
            if (fl_expired(F, w0)) {
                if (lane == 0) tb_panic(g, PANIC_FLOW_STALL);
                w = nw;
                break;
            }
        }
        if (w >= nw) break;
        const HotRec r = ring[(w % WALK_RING) * 64 + lane];
        const u32 n = min(64u, N - w * 64);
        const bool big = __ballot(lane < n && r.a >= (1LL << 24));
        u32 s = 0;
        for (;;) {
            const u32 m = big ? fl_walk_hot_window64(F, r, s, n, dreg, ws) : fl_walk_hot_window(F, r, s, n, dreg, ws);
            if (m > s && tblock) {
                ws.block_ticks += wall_clock64() - tblock;
                tblock = 0;
                wb = 0;
            }
            s = m;
            if (s >= n) break;
            // Waiting on a light walker.
            ws.blocks++;
            const u64 now = fl_now();
            if (!tblock) tblock = now;
            if (!wb) wb = now;
            if (now - wb > F.stall_ticks) {
                if (lane == 0) tb_panic(g, PANIC_FLOW_STALL);
                break;
            }
            if (fl_stalled(g)) break;
            __builtin_amdgcn_s_sleep(1);
        }
        if (s < n) break;
        if (lane == 0) __hip_atomic_store(&ctl[1], w + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (lane == 0) __hip_atomic_store(&ctl[1], nw, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);  // done or quit
    if (tblock) ws.block_ticks += wall_clock64() - tblock;
    ws.loop_ticks += wall_clock64() - ta;
}

__device__ static inline bool fl_walk(const PassArgs& P, const FlowArgs& F, u32 ndep, u32 NA, u32& gen, u32* s_wf,
                                       u32* s_ctl, HotRec* s_ring) {
    Globals* g = P.T.g;
    const u32 NT = FLOW_THREADS, tid = threadIdx.x, G = FL_G;
    const u32 lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    WalkRec* R = (WalkRec*)F.b_ex;                 // [2 * ndep] position records (sorted order)
    const u32 segcap = 2 * ndep + 2;
    u32* seg = (u32*)F.b_rec;                      // [NS + 1] segment first records
    u32* hv = seg + segcap;                        // [NH] heavy segments
    u32* cur = hv + segcap;                        // [NS] cursors (light segments)
    i64* dsv = (i64*)(cur + segcap + (segcap & 1));  // [NS] running sums (light segments)

    // W1. Units: the verdict words; the undecided count (stats).
    u32 nu = 0;
    for (u32 f = FL_B * NT + tid; f < ndep; f += G * NT) {
        if (F.f_len[f] && F.b_st[f] == BS_UNK) {
            F.b_vw[f] = (u32)F.b_vd[f] | ((u32)F.b_vc[f] << 2);
            nu++;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nu += __shfl_xor(nu, off);
    if (lane == 0 && nu) atomicAdd((unsigned long long*)&g->bounds_swept, (unsigned long long)nu);
    // W2. The undecided positions in sorted order (segments stay contiguous, in event order).
    u32 M = 0;
    if (!fl_compact(F, g, NA, gen, s_wf, M,
                    [&](u32 q) {
                        const u32 meta = F.b_meta[q];
                        return (meta & (BT_X | BT_Y)) && F.b_st[meta >> 3] == BS_UNK;
                    },
                    [&](u32 q, u32 p) {
                        const u32 meta = F.b_meta[q], u = meta >> 3;
                        WalkRec r;
                        r.base = (i64)(F.b_xy[2 * q + 1] - F.b_xy[2 * q]);
                        r.a = (i64)F.b_amt[q];
                        r.u = u;
                        r.kind = (meta & (BT_X | BT_Y | BT_CR)) | ((u32)F.b_vd[u] << 8) | ((u32)F.b_vc[u] << 12);
                        r.head = F.b_head[q];
                        r.pad = 0;
                        R[p] = r;
                        F.b_head[q] = p;  // from here on: position -> its record
                    }))
        return false;
    // W3. Segment starts.
    u32 NS = 0;
    if (!fl_compact(F, g, M, gen, s_wf, NS, [&](u32 p) { return p == 0 || R[p].head != R[p - 1].head; },
                    [&](u32 p, u32 k) {
                        seg[k] = p;
                        if (k + 1 == NS) seg[NS] = M;  // NS is the total by now
                        cur[k] = 0;
                        dsv[k] = 0;
                    }))
        return false;
    // W4. Heavy segments (a workgroup's first wave each).
    u32 NH = 0;
    if (!fl_compact(F, g, NS, gen, s_wf, NH,
                    [&](u32 k) {
                        const u32 len = seg[k + 1] - seg[k];
                        if (len >= WALK_HEAVY) {
                            atomicMax((unsigned long long*)&g->walk[7], (unsigned long long)len);
                            atomicMax(&F.words[FW_WMAX], len);
                        }
                        return len >= WALK_HEAVY;
                    },
                    [&](u32 k, u32 i) { hv[i] = k; }))
        return false;
    if (FL_B == 0 && tid == 0) {
        atomicAdd((unsigned long long*)&g->walk[0], (unsigned long long)NS);
        atomicAdd((unsigned long long*)&g->walk[1], (unsigned long long)NH);
    }

    // W5. The walk.  Up to WALK_MERGE_MAX heavy segments: merged, on the first wave of workgroup 0
    // (a CU whose other waves stay idle, so its scalar unit serves the walk alone).  More: heavy
    // segment i on the first wave of workgroup i when at most half the workgroups are taken by them.
    // The light segments spread over the waves of the other workgroups.
    const bool merged = NH > 0 && NH <= F.walk_merge;
    const bool split = !merged && NH > 0 && NH <= G / 2;
    HotRec* H = (HotRec*)F.b_xy;  // [ndep] the merged stream (b_xy is read by W2 only)
    u32 NHU = 0;
    if (merged) {
        // Tag the heavy positions with their heavy index, then list the units with a heavy leg.
        for (u32 i = 0; i < NH; i++) {
            const u32 k = hv[i], s0 = seg[k], len = seg[k + 1] - s0;
            for (u32 p = FL_B * NT + tid; p < len; p += G * NT) R[s0 + p].pad = i + 1;
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return false;
        auto heavy_leg = [&](u32 q) { return q != FLOW_SENT && R[F.b_head[q]].pad != 0; };
        if (!fl_compact(F, g, ndep, gen, s_wf, NHU,
                        [&](u32 f) {
                            return F.f_len[f] && F.b_st[f] == BS_UNK && (heavy_leg(F.b_qd[f]) || heavy_leg(F.b_qc[f]));
                        },
                        [&](u32 f, u32 i) {
                            HotRec h = {};
                            h.u = f;
                            u32 info = ((u32)F.b_vd[f] << HI_VD_SHIFT) | ((u32)F.b_vc[f] << HI_VC_SHIFT);
                            const u32 qd = F.b_qd[f], qc = F.b_qc[f];
                            if (qd != FLOW_SENT) {
                                const WalkRec& x = R[F.b_head[qd]];
                                h.bd = x.base;
                                h.a = x.a;
                                info |= HI_DP | ((x.kind & BT_X) ? HI_DX : 0) | x.pad;
                            }
                            if (qc != FLOW_SENT) {
                                const WalkRec& x = R[F.b_head[qc]];
                                h.bc = x.base;
                                h.a = x.a;
                                info |= HI_CP | ((x.kind & BT_X) ? HI_CX : 0) | (x.pad << HI_HC_SHIFT);
                            }
                            h.info = info;
                            H[i] = h;
                        }))
            return false;
    }
    WalkStats ws;
    const u64 w0 = fl_now();
    bool heavy_walker = false, light_wave = true;
    u32 lw = FL_B * (NT / 64) + wave, LW = G * (NT / 64);
    if (merged) {
        if (FL_B == 0) {
            // The walker (wave 0) and its feeder (wave 1); the ring lives in the planner's LDS.
            if (tid == 0) {
                s_ctl[0] = 0;
                s_ctl[1] = 0;
            }
            __syncthreads();
            heavy_walker = wave == 0;
            fl_walk_merged(F, g, H, NHU, ws, s_ctl, s_ring);
            if (heavy_walker && lane == 0) atomicAdd((unsigned long long*)&g->walk[2], (unsigned long long)NHU);
        }
        light_wave = G >= 2 ? FL_B >= 1 : wave >= 2;  // (waves 0, 1 of workgroup 0: the walker, its feeder)
        lw = G >= 2 ? (FL_B - 1) * (NT / 64) + wave : wave - 2;
        LW = G >= 2 ? (G - 1) * (NT / 64) : NT / 64 - 2;
    } else if (split) {
        u32 len = 0;
        if (FL_B < NH && wave == 0) {
            heavy_walker = true;
            const u32 k = hv[FL_B];
            const u32 s0 = seg[k];
            len = seg[k + 1] - s0;
            fl_walk_heavy(F, g, R, s0, len, ws);
        }
        if (heavy_walker) {
            if (lane == 0) {
                atomicAdd((unsigned long long*)&g->walk[2], (unsigned long long)len);
                if (len == *(volatile u32*)&F.words[FW_WMAX]) {  // the critical walker: the longest segment
                    atomicAdd((unsigned long long*)&g->walk[8], (unsigned long long)ws.windows);
                    atomicAdd((unsigned long long*)&g->walk[9], (unsigned long long)ws.blocks);
                    atomicAdd((unsigned long long*)&g->walk[10], (unsigned long long)ws.block_ticks);
#if WALK_PROF
                    for (int k = 0; k < 4; k++) atomicAdd((unsigned long long*)&g->walk_dbg[k], (unsigned long long)ws.pt[k]);
#endif
                    atomicAdd((unsigned long long*)&g->walk[11], (unsigned long long)(fl_now() - w0));
#if WALK_CNT
                    for (int k = 0; k < 4; k++) atomicAdd((unsigned long long*)&g->walk_dbg[k], (unsigned long long)ws.cnt[k]);
#endif
                }
            }
        }
        light_wave = FL_B >= NH;
        lw = (FL_B - NH) * (NT / 64) + wave;
        LW = (G - NH) * (NT / 64);
    }
    if (light_wave) {
        const bool skip_heavy = merged || split;
        u64 wb = 0;
        for (;;) {
            bool left = false, moved = false;
            for (u32 k = lw; k < NS; k += LW) {
                const u32 s0 = seg[k], n_seg = seg[k + 1] - s0;
                if (skip_heavy && n_seg >= WALK_HEAVY) continue;
                u32 c = fl_ld32(&cur[k]);
                if (c == n_seg) continue;
                i64 d = (i64)fl_ld64(&dsv[k]);
                if (fl_walk_segment(F, R, s0, n_seg, c, d, ws)) {
                    moved = true;
                    if (lane == 0) {
                        cur[k] = c;
                        dsv[k] = d;
                    }
                }
                left |= c < n_seg;
            }
            if (!left) break;
            const u64 now = fl_now();
            if (moved) {
                wb = 0;
                continue;
            }
            if (!wb) wb = now;
            if (now - wb > F.stall_ticks) {
                if (lane == 0) {
                    g->walk_dbg[0] = 2 | ((u64)lw << 8) | ((u64)NS << 32);
                    tb_panic(g, PANIC_FLOW_STALL);
                }
                break;
            }
            if (fl_stalled(g)) break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (heavy_walker && lane == 0) {
        const u64 t = fl_now() - w0;
        atomicAdd((unsigned long long*)&g->walk[3], (unsigned long long)ws.windows);
        atomicAdd((unsigned long long*)&g->walk[4], (unsigned long long)ws.stops);
        atomicAdd((unsigned long long*)&g->walk[5], (unsigned long long)ws.blocks);
        atomicAdd((unsigned long long*)&g->walk[6], (unsigned long long)ws.block_ticks);

        if (FL_B == 0) {
            atomicAdd((unsigned long long*)&g->sweep_ticks[1], (unsigned long long)ws.loop_ticks);
            atomicAdd((unsigned long long*)&g->sweep_ticks[2], (unsigned long long)(t - ws.loop_ticks));
        }
    }
    fl_grid_sync(g, G, gen, F);
    return !fl_stalled(g);
}

__device__ static inline bool fl_sweep(const PassArgs& P, const FlowArgs& F, u32 ndep, u32 NA, u32& gen,
                                       u64 (*s_wv)[4], u32* s_wf, u32* s_cnt, u32* s_hk, u64* s_hx) {
    Globals* g = P.T.g;
    const Tables& T = P.T;
    const u32 NT = FLOW_THREADS, tid = threadIdx.x, G = FL_G;
    const u32 lane = tid & 63, wave = tid >> 6;
    const u32* K = F.keys[0];
    const u64 t_all = (FL_B == 0 && tid == 0) ? fl_now() : 0;

    // Every balance, amount and sum below 2^63 (bound + S, the certificate's own numbers): the
    // signed slack form; below 2^62: the per-account walkers (fl_walk), whose "always" / "never"
    // sentinels (+-2^62) then cannot overflow.
    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);
    u128 bs;
    const bool slack = !P.cert_ext && cert_global && !tb_add_overflows(tb_u128(g->bound_lo, g->bound_hi), S, &bs) &&
                       tb_hi(bs) == 0 && (tb_lo(bs) >> 63) == 0;
    const bool walk = F.walk && slack && (tb_lo(bs) >> 62) == 0;

    // 1a. Units: no legs yet.
    for (u32 f = FL_B * NT + tid; f < ndep; f += G * NT) {
        F.b_qd[f] = FLOW_SENT;
        F.b_qc[f] = FLOW_SENT;
    }
    // 1b. The record scan (statuses are fixed from here to the sweep).
    const u32 tile = ((NA + G - 1) / G + NT - 1) / NT * NT;
    const u32 t0 = min(NA, FL_B * tile), t1 = min(NA, t0 + tile);
    u64 carry[4] = {0, 0, 0, 0};
    u32 any_start = 0;
    for (u32 c0 = t0; c0 < t1; c0 += NT) {
        const u32 q = c0 + tid;
        u64 v[4] = {0, 0, 0, 0};
        u32 f = 0;
        if (q < t1) fl_record_contrib(F, K, q, v, f);
        any_start |= __syncthreads_or(f);
        fl_seg_scan4(v, f, carry, s_wv, s_wf);
    }
    if (tid == 0) {
        F.b_blk[5 * FL_B] = any_start;
#pragma unroll
        for (u32 k = 0; k < 4; k++) F.b_blk[5 * FL_B + 1 + k] = carry[k];
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;
    u64 cin[4] = {0, 0, 0, 0};
    for (int b = (int)FL_B - 1; b >= 0; b--) {
#pragma unroll
        for (u32 k = 0; k < 4; k++) cin[k] += F.b_blk[5 * b + 1 + k];
        if (F.b_blk[5 * b]) break;
    }
    for (u32 c0 = t0; c0 < t1; c0 += NT) {
        const u32 q = c0 + tid;
        u64 v[4] = {0, 0, 0, 0}, own[4] = {0, 0, 0, 0};
        u32 f = 0;
        if (q < t1) {
            fl_record_contrib(F, K, q, v, f);
#pragma unroll
            for (u32 k = 0; k < 4; k++) own[k] = v[k];
        }
        fl_seg_scan4(v, f, cin, s_wv, s_wf);
        if (q >= t1) continue;
        const u32 meta = F.b_meta[q];
        const u32 u = meta >> 3;
        if (!(meta & (BT_X | BT_Y)) || F.b_st[u] != BS_UNK) continue;
        const u32 r = K[q];
        const u64* L = T.bal.lo + 4 * (u64)r;  // low words (the bounds run in u64)
        const bool dlim = T.acct_hot[r].flags & AF_DEBITS_MUST_NOT_EXCEED_CREDITS;
        const u64 xb = dlim ? L[BAL_DP] + L[BAL_DPOST] : L[BAL_CP] + L[BAL_CPOST];
        const u64 yb = dlim ? L[BAL_CPOST] : L[BAL_DPOST];
        const u32 head = (u32)v[1];
        F.b_xy[2 * q] = xb + v[0] - own[0];
        F.b_xy[2 * q + 1] = yb + v[2] - own[2];
        F.b_head[q] = head;
        if (!walk) {
            F.b_ex[2 * head] = 0;
            F.b_ex[2 * head + 1] = 0;
        }
        if (F.run[q].dr == r) F.b_qd[u] = q;
        else F.b_qc[u] = q;
    }
    if (walk) {
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return false;
        const bool done = fl_walk(P, F, ndep, NA, gen, s_wf, s_hk, (HotRec*)s_hx);
        if (FL_B == 0 && tid == 0)
            atomicAdd((unsigned long long*)&g->sweep_ticks[0], (unsigned long long)(fl_now() - t_all));
        return done;
    }
    // 1c. The undecided units in event order: per workgroup tile of units its count, then its offset.
    const u32 ut = ((ndep + G - 1) / G + NT - 1) / NT * NT;
    const u32 u0 = min(ndep, FL_B * ut), u1 = min(ndep, u0 + ut);
    u32 cnt = 0;
    for (u32 c0 = u0; c0 < u1; c0 += NT) {
        const u32 f = c0 + tid;
        cnt += __syncthreads_count(f < u1 && F.f_len[f] && F.b_st[f] == BS_UNK);
    }
    if (tid == 0) F.b_blk[5 * FL_B] = cnt;
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;
    u32 off = 0, nu = 0;
    for (u32 b = 0; b < G; b++) {
        const u32 c = (u32)F.b_blk[5 * b];
        off += b < FL_B ? c : 0;
        nu += c;
    }
    for (u32 c0 = u0; c0 < u1; c0 += NT) {
        const u32 f = c0 + tid;
        const bool pred = f < u1 && F.f_len[f] && F.b_st[f] == BS_UNK;
        const u64 m = __ballot(pred);
        if (lane == 0) s_wf[wave] = __popcll(m);
        __syncthreads();
        u32 before = 0, total = 0;
        for (u32 w = 0; w < NT / 64; w++) {
            before += w < wave ? s_wf[w] : 0;
            total += s_wf[w];
        }
        if (pred) {  // the unit's sweep record (its legs with the decided units before them)
            SweepRec x = {};
            x.f = f;
            x.hd = x.hc = FLOW_SENT;
            const u32 qd = F.b_qd[f], qc = F.b_qc[f];
            u32 td = BT_NONE, tc = BT_NONE;
            if (qd != FLOW_SENT) {
                x.hd = F.b_head[qd];
                td = F.b_meta[qd] & (BT_X | BT_Y);
                x.xd = F.b_xy[2 * qd];
                x.yd = F.b_xy[2 * qd + 1];
                x.a = F.b_amt[qd];
            }
            if (qc != FLOW_SENT) {
                x.hc = F.b_head[qc];
                tc = F.b_meta[qc] & (BT_X | BT_Y);
                x.xc = F.b_xy[2 * qc];
                x.yc = F.b_xy[2 * qc + 1];
                x.a = F.b_amt[qc];
            }
            x.t = td | (tc << 4) | ((u32)F.b_vd[f] << 8) | ((u32)F.b_vc[f] << 12);
            F.b_rec[off + before + __popcll(m & ((1ULL << lane) - 1))] = x;
        }
        off += total;
        __syncthreads();
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;

    // 2. The sweep: wave 0 of workgroup 0, 64 units a window; the next window's records load while
    // this one is resolved.  A lane holds one unit: its legs' X, Y with the decided units and the
    // swept ok units of earlier windows (b_ex); the window is resolved in lane order, each ok unit
    // adding its legs to the later lanes that share an account (branch-free: one wave, so every
    // instruction's latency is on the critical path).
    if (FL_B == 0 && wave == 0) {
        SweepRec nx = {};
        if (lane < nu) nx = F.b_rec[lane];
        for (u32 k = lane; k < SW_CAP; k += 64) {
            s_hk[k] = FLOW_SENT;
            s_hx[2 * k] = 0;
            s_hx[2 * k + 1] = 0;
        }
        u64 t_wait = 0, t_loop = 0;
        const u64 t_walk = fl_now();
        for (u32 w0 = 0; w0 < nu; w0 += 64) {
            const SweepRec x = nx;
            const u64 ta = fl_now();
            const u32 nv = min(64u, nu - w0);
            const bool valid = lane < nv;
            u64 xd = x.xd, yd = x.yd, xc = x.xc, yc = x.yc;
            // The swept sums of the lane's segments: LDS (one wave: its LDS operations complete in
            // order), global memory for a head without a slot.
            const u32 sld = valid ? fl_sw_slot(s_hk, x.hd) : SW_NONE;
            const u32 slc = valid ? fl_sw_slot(s_hk, x.hc) : SW_NONE;
            bool glob = false;
            if (valid && x.hd != FLOW_SENT) {
                if (sld != SW_NONE) {
                    xd += s_hx[2 * sld];
                    yd += s_hx[2 * sld + 1];
                } else {
                    xd += fl_ld64(&F.b_ex[2 * x.hd]);
                    yd += fl_ld64(&F.b_ex[2 * x.hd + 1]);
                    glob = true;
                }
            }
            if (valid && x.hc != FLOW_SENT) {
                if (slc != SW_NONE) {
                    xc += s_hx[2 * slc];
                    yc += s_hx[2 * slc + 1];
                } else {
                    xc += fl_ld64(&F.b_ex[2 * x.hc]);
                    yc += fl_ld64(&F.b_ex[2 * x.hc + 1]);
                    glob = true;
                }
            }
            if (__ballot(glob)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const u64 tb = fl_now();
            if (w0 + 64 + lane < nu) nx = F.b_rec[w0 + 64 + lane];
            const u32 vd = (x.t >> 8) & 15, vc = (x.t >> 12) & 15;
            const u64 a = x.a;
            // A known verdict never changes; only the sums move.
            const bool dknown = vd != BV_UNK, cknown = vc != BV_UNK;
            const bool dfix = vd == BV_FAIL, cfix = vc == BV_FAIL;
            bool dfl, cfl;  // this lane's verdicts, final once every earlier lane has been told
            if (slack) {
                // Every balance, amount and sum below 2^63 (cert63): one signed slack Y - X per
                // leg, "fails if slack < amount"; an ok unit moves each of its accounts' slack by
                // one signed delta (an X leg: -a, a Y leg: +a) — half the work of X and Y apart.
                i64 sd = (i64)(yd - xd), sc = (i64)(yc - xc);
                const u32 td = x.t & 15, tc2 = (x.t >> 4) & 15;
                const i64 dd_ = (td & BT_X) ? -(i64)a : (td & BT_Y) ? (i64)a : 0;
                const i64 dc_ = (tc2 & BT_X) ? -(i64)a : (tc2 & BT_Y) ? (i64)a : 0;
                // Verdicts as wave masks (scalar registers): step j compares every lane's slack
                // (one vector compare per side), keeps lane j's bit, and only an ok lane j
                // broadcasts its legs.  Lane j's verdict is final at step j (every earlier lane has
                // been applied), so later steps may add to it freely: no lane > j guard.
                const u64 nkd = ~__ballot(dknown), nkc = ~__ballot(cknown);
                const u64 fxd = __ballot(dknown && dfix), fxc = __ballot(cknown && cfix);
                u64 dflm = 0, cflm = 0;
                for (u32 j = 0; j < nv; j++) {
                    const u64 dfm = (__ballot(sd < (i64)a) & nkd) | fxd;
                    const u64 cfm = (__ballot(sc < (i64)a) & nkc) | fxc;
                    const u64 bit = 1ULL << j;
                    dflm |= dfm & bit;
                    cflm |= cfm & ~dfm & bit;
                    if ((dfm | cfm) & bit) continue;  // lane j fails: nothing to broadcast
                    const u32 jhd = __builtin_amdgcn_readlane(x.hd, j), jhc = __builtin_amdgcn_readlane(x.hc, j);
                    const i64 jdd = (i64)fl_rl64((u64)dd_, j), jdc = (i64)fl_rl64((u64)dc_, j);
                    sd += (x.hd == jhd ? jdd : 0) + (x.hd == jhc ? jdc : 0);
                    sc += (x.hc == jhd ? jdd : 0) + (x.hc == jhc ? jdc : 0);
                }
                dfl = (dflm >> lane) & 1;
                cfl = (cflm >> lane) & 1;
            } else {
                for (u32 j = 0; j < nv; j++) {
                    const u32 jhd = __builtin_amdgcn_readlane(x.hd, j), jhc = __builtin_amdgcn_readlane(x.hc, j);
                    const u32 jt = __builtin_amdgcn_readlane(x.t, j);
                    const u64 ja = fl_rl64(a, j);
                    const bool dfail = dknown ? dfix : xd + a > yd;
                    const bool cfail = cknown ? cfix : xc + a > yc;
                    const u64 okj = __builtin_amdgcn_readlane((u32)(!dfail & !cfail), j);
                    const u64 m = lane > j && okj ? ja : 0;  // lane j's legs, if it is ok, for the later lanes
                    const u64 dxd = jt & BT_X ? m : 0, dyd = jt & BT_Y ? m : 0;
                    const u64 dxc = (jt >> 4) & BT_X ? m : 0, dyc = (jt >> 4) & BT_Y ? m : 0;
                    const bool dd = x.hd == jhd, dc = x.hd == jhc, cd = x.hc == jhd, cc = x.hc == jhc;
                    xd += (dd ? dxd : 0) + (dc ? dxc : 0);
                    yd += (dd ? dyd : 0) + (dc ? dyc : 0);
                    xc += (cd ? dxd : 0) + (cc ? dxc : 0);
                    yc += (cd ? dyd : 0) + (cc ? dyc : 0);
                }
                dfl = dknown ? dfix : xd + a > yd;
                cfl = !dfl && (cknown ? cfix : xc + a > yc);
            }
            const u64 tc = fl_now();
            t_loop += tc - tb;
            bool gadd = false;
            if (valid) {
                F.b_st[x.f] = dfl ? BS_FAIL_CREDITS : cfl ? BS_FAIL_DEBITS : BS_OK;
                if (!dfl && !cfl) {
                    const u32 td = x.t & 15, tc2 = (x.t >> 4) & 15;
                    if (x.hd != FLOW_SENT) {
                        if (sld != SW_NONE) {
                            if (td & BT_X) atomicAdd((unsigned long long*)&s_hx[2 * sld], (unsigned long long)a);
                            if (td & BT_Y) atomicAdd((unsigned long long*)&s_hx[2 * sld + 1], (unsigned long long)a);
                        } else {
                            if (td & BT_X) tb_atomic_add_lo_noret(&F.b_ex[2 * x.hd], a);
                            if (td & BT_Y) tb_atomic_add_lo_noret(&F.b_ex[2 * x.hd + 1], a);
                            gadd = true;
                        }
                    }
                    if (x.hc != FLOW_SENT) {
                        if (slc != SW_NONE) {
                            if (tc2 & BT_X) atomicAdd((unsigned long long*)&s_hx[2 * slc], (unsigned long long)a);
                            if (tc2 & BT_Y) atomicAdd((unsigned long long*)&s_hx[2 * slc + 1], (unsigned long long)a);
                        } else {
                            if (tc2 & BT_X) tb_atomic_add_lo_noret(&F.b_ex[2 * x.hc], a);
                            if (tc2 & BT_Y) tb_atomic_add_lo_noret(&F.b_ex[2 * x.hc + 1], a);
                            gadd = true;
                        }
                    }
                }
            }
            if (__ballot(gadd)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next window reads b_ex
            t_wait += (tb - ta) + (fl_now() - tc);
        }
        if (lane == 0) {
            F.words[FW_BUND] = 0;
            atomicAdd((unsigned long long*)&g->bounds_swept, (unsigned long long)nu);
            if (!slack) atomicAdd((unsigned long long*)&g->sweep_u64_passes, 1ULL);
            atomicAdd((unsigned long long*)&g->sweep_ticks[0], (unsigned long long)(fl_now() - t_walk));
            atomicAdd((unsigned long long*)&g->sweep_ticks[1], (unsigned long long)t_loop);
            atomicAdd((unsigned long long*)&g->sweep_ticks[2], (unsigned long long)t_wait);
        }
    }
    fl_grid_sync(g, G, gen, F);
    return !fl_stalled(g);
}

// No-return add of v to the low word at p (p == nullptr: nothing) for every lane of the wave; lanes
// naming the same word add their sum with a single atomic.
#ifndef FL_ADD_ROUNDS
#define FL_ADD_ROUNDS 16
#endif
__device__ static inline void fl_add_lo(u64* p, u64 v) {
    const u32 lane = threadIdx.x & 63;
    bool left = p != nullptr;
    // Leader by leader (the lowest lane still left), up to FL_ADD_ROUNDS of them: a lone lane adds
    // its own value, a group its wave sum.  Stopping at the first lone leader (a cold account in
    // lane 0 is the common case under Zipf) left the hot words' lanes to add one by one, and
    // thousands of same-address atomics per pass serialise (C3's bounds apply: 0.15 ms per chunk).
#pragma unroll 1
    for (int r = 0; r < FL_ADD_ROUNDS; r++) {
        const u64 live = __ballot(left);
        if (!live) return;
        const u32 l = (u32)__builtin_ctzll(live);
        const u64 lead = ((u64)(u32)__builtin_amdgcn_readlane((u32)((uintptr_t)p >> 32), l) << 32) |
                         (u32)__builtin_amdgcn_readlane((u32)(uintptr_t)p, l);
        const bool mine = left && (u64)(uintptr_t)p == lead;
        const u64 group = __ballot(mine);
        u64 part = mine ? v : 0;
        if (__popcll(group) > 1) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) part += __shfl_xor((unsigned long long)part, off);
        }
        if (lane == l) tb_atomic_add_lo_noret(p, part);
        left = left && !mine;
    }
    if (left) tb_atomic_add_lo_noret(p, v);
}

// Returns true when every unit was decided and applied (the ordered run is skipped).
__device__ static inline bool fl_bounds(const PassArgs& P, const FlowArgs& F, u32 ndep, u32 N, bool cert64, u32& gen,
                                        u64& tsmax, u64 (*s_wv)[4], u32* s_wf, u32* s_cnt, u64& tp, u32* s_hk,
                                        u64* s_hx) {
    Globals* g = P.T.g;
    const Tables& T = P.T;
    const u32 NT = FLOW_THREADS, tid = threadIdx.x, G = FL_G;
    const u32* K = F.keys[0];
    if (!cert64 || F.bounds_rounds_max == 0) return false;
    // Account positions are the prefix of the sorted list (keys < 2^31).
    u32 lo = 0, hi = N;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (K[mid] < 0x80000000u) lo = mid + 1; else hi = mid;
    }
    const u32 NA = lo;

    // S1: units — eligibility, static failures, no check yet.
    for (u32 f = FL_B * NT + tid; f < ndep; f += G * NT) {
        if (!F.f_len[f]) continue;
        const u32 pe = F.f_pe[f];
        const u32 info = P.info[pe];
        const u16 fl = P.eflags[pe];
        const bool elig = F.f_len[f] == 1 && (F.uflags[f] & (UF_ID_SINGLE | UF_ID_UNIQUE)) && (info & HZ_SPEC) &&
                          (info & HZ_ACCTS) &&
                          !(fl & (TF_LINKED | TF_POST | TF_VOID | TF_BAL_DEBIT | TF_BAL_CREDIT)) &&
                          !(info & HZ_AMT_HI);
        if (!elig) {
            atomicOr(&F.words[FW_BNO], 1u);
            continue;
        }
        const bool ok = (info & 0xFF) == R_OK;
        F.b_st[f] = ok ? BS_UNK : BS_FAIL_STATIC;
        F.b_vd[f] = BV_PASS;
        F.b_vc[f] = BV_PASS;
        if (ok) atomicAdd(&F.words[FW_BUND], 1u);
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;
    if (*(volatile u32*)&F.words[FW_BNO]) {
        if (FL_B == 0 && tid == 0) atomicAdd((unsigned long long*)&g->bounds_skipped, 1ULL);
        return false;
    }

    // S2: positions — the leg each holds, and which checks are open.
    for (u32 q = FL_B * NT + tid; q < NA; q += G * NT) {
        const RunEntry x = F.run[q];
        const u32 r = K[q];
        const u16 rf = T.acct_hot[r].flags;
        const bool debit = x.dr == r, pend = x.flags & TF_PENDING;
        u32 type = BT_NONE;
        if (rf & AF_DEBITS_MUST_NOT_EXCEED_CREDITS) type = debit ? BT_X : (pend ? BT_NONE : BT_Y);
        else if (rf & AF_CREDITS_MUST_NOT_EXCEED_DEBITS) type = debit ? (pend ? BT_NONE : BT_Y) : (BT_X | BT_CR);
        F.b_meta[q] = (x.u << 3) | type;
        F.b_amt[q] = x.amt_lo;
        if ((type & BT_X) && F.b_st[x.u] == BS_UNK) {
            if (type & BT_CR) F.b_vc[x.u] = BV_UNK;
            else F.b_vd[x.u] = BV_UNK;
        }
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;
    // S3: units with no open check (a credit to a debits-limited account, ...) are ok.
    for (u32 f = FL_B * NT + tid; f < ndep; f += G * NT) {
        if (F.f_len[f] && F.b_st[f] == BS_UNK && F.b_vd[f] == BV_PASS && F.b_vc[f] == BV_PASS) {
            F.b_st[f] = BS_OK;
            atomicSub(&F.words[FW_BUND], 1u);
        }
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return false;

    fl_mark(g, tp, FP_BSETUP);
    const u32 tile = ((NA + G - 1) / G + NT - 1) / NT * NT;
    const u32 t0 = min(NA, FL_B * tile), t1 = min(NA, t0 + tile);
    bool converged = *(volatile u32*)&F.words[FW_BUND] == 0;
    u32 rounds = 0;
    for (; !converged && rounds < F.bounds_rounds_max; rounds++) {
        u32* dec = &F.words[FW_BDEC + rounds % 3];
        if (FL_B == 0 && tid == 0) F.words[FW_BDEC + (rounds + 1) % 3] = 0;
        // Phase A: this tile's aggregate (sums since its last segment start; start flag).
        u64 carry[4] = {0, 0, 0, 0};
        u32 any_start = 0;
        for (u32 c0 = t0; c0 < t1; c0 += NT) {
            const u32 q = c0 + tid;
            u64 v[4] = {0, 0, 0, 0};
            u32 f = 0;
            if (q < t1) {
                fl_bound_contrib(F, q, v);
                f = q == 0 || K[q] != K[q - 1];
            }
            any_start |= __syncthreads_or(f);
            fl_seg_scan4(v, f, carry, s_wv, s_wf);
        }
        if (tid == 0) {
            F.b_blk[5 * FL_B] = any_start;
#pragma unroll
            for (u32 k = 0; k < 4; k++) F.b_blk[5 * FL_B + 1 + k] = carry[k];
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return false;
        // Phase B: carry-in from the preceding tiles, then the scan again with the decisions.
        u64 cin[4] = {0, 0, 0, 0};
        for (int b = (int)FL_B - 1; b >= 0; b--) {
#pragma unroll
            for (u32 k = 0; k < 4; k++) cin[k] += F.b_blk[5 * b + 1 + k];
            if (F.b_blk[5 * b]) break;
        }
        if (tid == 0) *s_cnt = 0;
        __syncthreads();
        u32 mine = 0;
        for (u32 c0 = t0; c0 < t1; c0 += NT) {
            const u32 q = c0 + tid;
            u64 v[4] = {0, 0, 0, 0}, own[4] = {0, 0, 0, 0};
            u32 f = 0;
            if (q < t1) {
                fl_bound_contrib(F, q, v);
                f = q == 0 || K[q] != K[q - 1];
#pragma unroll
                for (u32 k = 0; k < 4; k++) own[k] = v[k];
            }
            fl_seg_scan4(v, f, cin, s_wv, s_wf);
            if (q >= t1) continue;
            const u32 meta = F.b_meta[q];
            const u32 u = meta >> 3;
            if (!(meta & BT_X) || F.b_st[u] != BS_UNK) continue;
            const bool cr_side = meta & BT_CR;
            if ((cr_side ? F.b_vc[u] : F.b_vd[u]) == BV_UNK) {
                // Exclusive sums: the decided / possible effects of the earlier events of the
                // segment.  Statuses read in the middle of a round are facts, old or new, so any mix
                // of them still bounds the truth.
                const u64 xmin = v[0] - own[0], xmax = v[1] - own[1], ymin = v[2] - own[2], ymax = v[3] - own[3];
                const u64* L = T.bal.lo + 4 * (u64)K[q];  // low words
                const u64 xb = cr_side ? L[BAL_CP] + L[BAL_CPOST] : L[BAL_DP] + L[BAL_DPOST];
                const u64 yb = cr_side ? L[BAL_DPOST] : L[BAL_CPOST];
                const u64 a = F.b_amt[q];
                u8 verdict = BV_UNK;
                if (xb + xmax + a <= yb + ymin) verdict = BV_PASS;
                else if (xb + xmin + a > yb + ymax) verdict = BV_FAIL;
                if (verdict == BV_UNK) continue;
                if (cr_side) F.b_vc[u] = verdict;
                else F.b_vd[u] = verdict;
                __threadfence();
            }
            // Combine in the reference's order (:863-864: exceeds_credits first).  A unit whose two
            // verdicts land in one round from two lanes is combined by either lane in a later round.
            const u8 vd = *(volatile u8*)&F.b_vd[u], vc = *(volatile u8*)&F.b_vc[u];
            u32 st = BS_UNK;
            if (vd == BV_FAIL) st = BS_FAIL_CREDITS;
            else if (vd == BV_PASS && vc == BV_FAIL) st = BS_FAIL_DEBITS;
            else if (vd == BV_PASS && vc == BV_PASS) st = BS_OK;
            if (st != BS_UNK && atomicCAS(&F.b_st[u], (u32)BS_UNK, st) == BS_UNK) mine++;
        }
        if (mine) atomicAdd(s_cnt, mine);
        __syncthreads();
        if (tid == 0 && *s_cnt) {
            atomicAdd(dec, *s_cnt);
            atomicSub(&F.words[FW_BUND], *s_cnt);
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return false;
        converged = *(volatile u32*)&F.words[FW_BUND] == 0;
        // A round that decides few units costs more than sweeping them in order.
        if (!converged && *(volatile u32*)dec < max(1u, F.sweep_min)) {
            rounds++;
            break;
        }
    }
    fl_mark(g, tp, FP_BROUNDS);
    if (!converged && F.sweep_min) {
        converged = fl_sweep(P, F, ndep, NA, gen, s_wv, s_wf, s_cnt, s_hk, s_hx);
        if (fl_stalled(g)) return false;
        fl_mark(g, tp, FP_SWEEP);
    }
    if (!converged) {
        if (FL_B == 0 && tid == 0) {
            atomicAdd((unsigned long long*)&g->bounds_abandoned, 1ULL);
            atomicAdd((unsigned long long*)&g->bounds_rounds, (unsigned long long)rounds);
        }
        return false;
    }

    // Apply: the ok units' legs (both accounts; sums commute), their index entries and counts; the
    // failed ones' codes.  Kernel 1 already wrote every record at its log position (in place: the
    // event is there, stamped).
    // Zipf-hot accounts put one balance word in many lanes of a wave: atomics on one address
    // serialise in L2, so the lanes sharing the first lane's word add their sum once (fl_add_lo).
    u32 n_ok = 0;
    u64 tsm = 0;
    for (u32 f0 = FL_B * NT; f0 < ndep; f0 += G * NT) {  // whole waves iterate together
        const u32 f = f0 + tid;
        bool ok = false;
        u32 pe = 0;
        if (f < ndep && F.f_len[f]) {
            pe = F.f_pe[f];
            const u8 st = F.b_st[f];
            ok = st == BS_OK;
            if (st == BS_FAIL_CREDITS || st == BS_FAIL_DEBITS) {
                P.info[pe] = (P.info[pe] & 0xFFFFFF00u) | (st == BS_FAIL_CREDITS ? CT_EXCEEDS_CREDITS : CT_EXCEEDS_DEBITS);
            }
        }
        u64* dw = nullptr;
        u64* cw = nullptr;
        u64 a = 0;
        if (ok) {
            a = P.amt[pe];
            const bool pend = P.eflags[pe] & TF_PENDING;
            dw = T.bal.lo + 4 * (u64)P.dr[pe] + (pend ? BAL_DP : BAL_DPOST);
            cw = T.bal.lo + 4 * (u64)P.cr[pe] + (pend ? BAL_CP : BAL_CPOST);
            __hip_atomic_fetch_and(&T.xidx[P.rs[pe]], ~(u64)XI_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            n_ok++;
            const u32 b = F.f_batch[f];
            const u64 boff = P.batch_off[b];
            const u64 ts = tb_event_ts(P, b, boff, (u32)(P.batch_off[b + 1] - boff), (u32)(P.e0 + pe - boff));
            tsm = max(tsm, ts);
        }
        fl_add_lo(dw, a);
        fl_add_lo(cw, a);
    }
    u64 nw = n_ok;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nw += __shfl_xor((unsigned long long)nw, off);
    if ((tid & 63) == 0 && nw) atomicAdd((unsigned long long*)&g->transfer_count, (unsigned long long)nw);
    tsmax = max(tsmax, tsm);
    if (FL_B == 0 && tid == 0) {
        atomicAdd((unsigned long long*)&g->bounds_passes, 1ULL);
        atomicAdd((unsigned long long*)&g->bounds_units, (unsigned long long)ndep);
        atomicAdd((unsigned long long*)&g->bounds_rounds, (unsigned long long)rounds);
    }
    return true;
}

// Exclusive prefix of v over the workgroup, in thread order; `total` = the workgroup's sum.
__device__ static inline u32 fl_block_excl(u32 v, u32* s_wave, u32& total) {
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (u32 off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    u32 before = 0;
    total = 0;
    for (u32 w = 0; w < blockDim.x / 64; w++) {
        const u32 c = s_wave[w];
        before += w < wave ? c : 0;
        total += c;
    }
    __syncthreads();
    return before + x - v;
}

__global__ __launch_bounds__(FLOW_THREADS) void tb_flow(PassArgs P, FlowArgs F, UndoEntry* seq_undo, u32 seq_undo_cap) {
    __shared__ u32 s_dpre[FLOW_NB_MAX + 1];
    __shared__ u32 s_wave[FLOW_THREADS / 64];
    __shared__ u32 s_hist[256];
    __shared__ u32 s_base[256];
    __shared__ __attribute__((aligned(16))) u32 s_wcnt[FLOW_THREADS / 64][256];
    static_assert(SW_CAP <= FLOW_NB_MAX + 1 && 2 * SW_CAP * 8 <= sizeof(u32) * (FLOW_THREADS / 64) * 256,
                  "the sweep's head table fits in s_dpre / s_wcnt");
    __shared__ u8 s_code[BATCH_LDS];
    __shared__ u32 s_list[FLOW_THREADS];
    __shared__ u64 s_tsmax[FLOW_THREADS / 64];

    Globals* g = P.T.g;
    const u32 NT = FLOW_THREADS, tid = threadIdx.x;
    const u32 nb = P.b1 - P.b0;
    // tb_apply_events' work first, when this launch replaces it (one launch a pass fewer): the
    // independent ok transfers that are not legs touch no constrained account, id or pending transfer
    // a dependent unit reads, so their balance adds commute with everything below.
    if (P.late_in_flow) tb_apply_late(P);
    if (__hip_atomic_load(&g->dependent_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (blockIdx.x == 0) fl_finish(P, s_code, s_wave, s_list, 0, false);  // (before any admission)
        return;
    }
    if (!fl_admit(g, F)) return;  // started after admission closed: the admitted workgroups cover the pass
    const u32 G = FL_G;
    u128 S;
    bool cert_global, cert64;
    tb_pass_cert(P, S, cert_global, cert64);
    u32 gen = 0;
    const u64 ft0 = (FL_B == 0 && tid == 0) ? fl_now() : 0;
    u64 tp = ft0;

    // ---- plan 1: flat list of dependent events, units, resource pairs ------------------------
    for (u32 k = tid; k < nb; k += NT) s_dpre[k] = P.dep_count[k];
    __syncthreads();
    tb_block_scan_lds(s_dpre, nb, s_wave);
    const u32 ndep = s_dpre[nb];
    // Each workgroup plans a contiguous tile of the flat list; its resource pairs go to FLOW_RMAX
    // slots per event in keys[1] / vals[1] first, and are compacted (in order) into keys[0] /
    // vals[0] below, so the sort sees only real pairs (C4: ~1.3 of the 6 slots per event).
    const u32 ftile = ((ndep + G - 1) / G + NT - 1) / NT * NT;
    const u32 fa = min(ndep, FL_B * ftile), fb = min(ndep, fa + ftile);
    u32 my_pairs = 0;
    for (u32 c0 = fa; c0 < fb; c0 += NT) {
        const u32 f = c0 + tid;
        if (f >= fb) break;
        u32 lo = 0, hi = nb;  // the batch k with s_dpre[k] <= f < s_dpre[k + 1]
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (s_dpre[mid] <= f) lo = mid; else hi = mid;
        }
        const u32 b = P.b0 + lo;
        const u64 boff = P.batch_off[b];
        const u32 L = (u32)(P.batch_off[b + 1] - boff);
        const u32 pbase = (u32)(boff - P.e0);
        const u32 i = P.dep_list[pbase + (f - s_dpre[lo])];
        const u32 pe = pbase + i;
        F.f_pe[f] = pe;
        F.f_batch[f] = b;
        F.need[f] = 0;
        F.nsucc[f] = 0;
        F.queue[f] = 0;
        F.uflags[f] = 0;
        F.nacct[f] = 0;
        // Unit: the chain (execute :628-692) this event belongs to, headed by its first member.
        u32 i0 = i;
        while (i0 > 0 && (P.eflags[pbase + i0 - 1] & TF_LINKED)) {
            i0--;
            if (i - i0 > FLOW_CHAIN_MAX) break;
        }
        const bool seq = i - i0 > FLOW_CHAIN_MAX;
        const u32 unit = f - (i - i0);
        u32 m = 0;
        if (unit == f) {
            m = 1;
            for (u32 j = i; (P.eflags[pbase + j] & TF_LINKED) && j + 1 < L && m <= FLOW_CHAIN_MAX; j++) m++;
            atomicAdd(&F.words[FW_NUNITS], 1u);
        }
        F.f_len[f] = m;
        // Resources.
        u32 keys[FLOW_RMAX];
        u32 nk = 0;
        bool ok = !seq && m <= FLOW_CHAIN_MAX;
        const Transfer* ev = (const Transfer*)(P.events + (P.e0 + pe) * 128);
        const u16 fl = P.eflags[pe];
        const u32 info = P.info[pe];
        keys[nk++] = fl_key_id(tb_lo(ev->id), tb_hi(ev->id));
        F.b_qd[f] = keys[0];  // own id key, for the link phase's UF_MEMBER_NEW (the sweep reuses b_qd)
        if (fl & (TF_POST | TF_VOID)) {
            keys[nk++] = fl_key_id(tb_lo(ev->pending_id), tb_hi(ev->pending_id));
            ok = ok && fl_pending_accounts(P, tb_lo(ev->pending_id), tb_hi(ev->pending_id), cert_global, keys, nk);
        } else if (info & HZ_ACCTS) {
            if (fl_account_is_resource(P.T, P.dr[pe], P.epoch, cert_global)) keys[nk++] = P.dr[pe];
            if (fl_account_is_resource(P.T, P.cr[pe], P.epoch, cert_global)) keys[nk++] = P.cr[pe];
        }
        if (!ok) atomicOr(&F.words[FW_SEQ], 1u);
#pragma unroll
        for (u32 k = 0; k < FLOW_RMAX; k++) F.keys[1][FLOW_RMAX * f + k] = k < nk ? keys[k] : FLOW_SENT;
        F.vals[1][FLOW_RMAX * f] = unit;
        my_pairs += nk;
    }
    {
        u32 total;
        (void)fl_block_excl(my_pairs, s_wave, total);
        if (tid == 0) F.b_blk[FL_B] = total;
    }
    fl_grid_sync(g, G, gen, F);
    if (fl_stalled(g)) return;
    const bool sequential = *(volatile u32*)&F.words[FW_SEQ] != 0;
    // Compaction: this workgroup's pairs start after those of the workgroups before it.
    u32 N = 0, base = 0;
    for (u32 w = 0; w < G; w++) {
        const u32 c = (u32)F.b_blk[w];
        base += w < FL_B ? c : 0;
        N += c;
    }
    if (!sequential) {
        for (u32 c0 = fa; c0 < fb; c0 += NT) {
            const u32 f = c0 + tid;
            u32 kk[FLOW_RMAX], nk = 0;
            if (f < fb) {
#pragma unroll
                for (u32 k = 0; k < FLOW_RMAX; k++) {
                    kk[k] = F.keys[1][FLOW_RMAX * f + k];
                    nk += kk[k] != FLOW_SENT ? 1u : 0u;
                }
            }
            u32 total;
            const u32 at = base + fl_block_excl(nk, s_wave, total);
            if (nk) {
                const u32 unit = F.vals[1][FLOW_RMAX * f];
#pragma unroll
                for (u32 k = 0; k < FLOW_RMAX; k++) {
                    if (k < nk) {  // a slot's keys are packed at its front
                        F.keys[0][at + k] = kk[k];
                        F.vals[0][at + k] = unit;
                    }
                }
            }
            base += total;
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return;
    }
    fl_mark(g, tp, FP_PLAN);

    if (!sequential) {
        // ---- plan 2: stable LSD radix sort of the pairs by key (4 x 8 bits) ---------------------
        const u32 tile = ((N + G - 1) / G + NT - 1) / NT * NT;
        const u32 t0 = min(N, FL_B * tile), t1 = min(N, t0 + tile);
        const u32 lane = tid & 63, wave = tid >> 6;
        for (u32 pass = 0; pass < 4; pass++) {
            const u32 shift = 8 * pass;
            const u32* sk = F.keys[pass & 1];
            const u32* sv = F.vals[pass & 1];
            u32* dk = F.keys[(pass + 1) & 1];
            u32* dv = F.vals[(pass + 1) & 1];
            if (tid < 256) s_hist[tid] = 0;
            __syncthreads();
            for (u32 q = t0 + tid; q < t1; q += NT) atomicAdd(&s_hist[(sk[q] >> shift) & 255], 1u);
            __syncthreads();
            if (tid < 256) F.hist[FL_B * 256 + tid] = s_hist[tid];
            fl_grid_sync(g, G, gen, F);
            if (fl_stalled(g)) return;
            // Digit totals over the grid and the counts of the workgroups before this one: every
            // thread sums one digit over a quarter of the workgroups (G / 4 loads, eight in flight),
            // then the quarters are combined.
            {
                const u32 d = tid & 255, qt = tid >> 8;  // FLOW_THREADS = 4 x 256
                const u32 w0 = qt * G / 4, w1 = (qt + 1) * G / 4;
                u32 tot = 0, before = 0;
                for (u32 w = w0; w < w1; w += 8) {
                    u32 c[8];
#pragma unroll
                    for (u32 k = 0; k < 8; k++) c[k] = w + k < w1 ? F.hist[(w + k) * 256 + d] : 0;
#pragma unroll
                    for (u32 k = 0; k < 8; k++) {
                        tot += c[k];
                        before += w + k < FL_B ? c[k] : 0;
                    }
                }
                s_wcnt[qt][d] = tot;
                s_wcnt[4 + qt][d] = before;
            }
            __syncthreads();
            u32 before = 0;
            if (tid < 256) {
                u32 tot = 0;
#pragma unroll
                for (u32 qt = 0; qt < 4; qt++) {
                    tot += s_wcnt[qt][tid];
                    before += s_wcnt[4 + qt][tid];
                }
                s_hist[tid] = tot;
            }
            __syncthreads();
            if (tid < 256) {  // exclusive scan of the digit totals (256 entries, one wave per 64)
                u32 start = 0;
                for (u32 d = 0; d < tid; d++) start += s_hist[d];
                s_base[tid] = start + before;
            }
            __syncthreads();
            for (u32 c0 = t0; c0 < t1; c0 += NT) {
                const u32 q = c0 + tid;
                const bool valid = q < t1;
                const u32 key = valid ? sk[q] : 0, val = valid ? sv[q] : 0;
                const u32 d = (key >> shift) & 255;
                for (u32 k = tid; k < (NT / 64) * 256; k += NT) (&s_wcnt[0][0])[k] = 0;
                u64 peers = __ballot(valid);
#pragma unroll
                for (u32 bit = 0; bit < 8; bit++) {
                    const u64 m = __ballot((d >> bit) & 1);
                    peers &= ((d >> bit) & 1) ? m : ~m;
                }
                const u32 rank = __popcll(peers & ((1ULL << lane) - 1));
                __syncthreads();
                if (valid && rank == 0) s_wcnt[wave][d] = __popcll(peers);
                __syncthreads();
                if (tid < 256) {
                    u32 run = s_base[tid];
                    for (u32 w = 0; w < NT / 64; w++) {
                        const u32 c = s_wcnt[w][tid];
                        s_wcnt[w][tid] = run;
                        run += c;
                    }
                    s_base[tid] = run;
                }
                __syncthreads();
                if (valid) {
                    const u32 pos = s_wcnt[wave][d] + rank;
                    dk[pos] = key;
                    dv[pos] = val;
                }
                __syncthreads();
            }
            fl_grid_sync(g, G, gen, F);
            if (fl_stalled(g)) return;
        }

        fl_mark(g, tp, FP_SORT);
        // ---- plan 3: link each unit to its successor on every resource --------------------------
        const u32* K = F.keys[0];
        const u32* V = F.vals[0];
        for (u32 q = FL_B * NT + tid; q < N; q += G * NT) {
            const u32 key = K[q];
            if (key == FLOW_SENT) continue;
            const bool first = q == 0 || K[q - 1] != key;
            const u32 u = V[q];
            if (first && (key & 0x80000000u) && (q + 1 == N || K[q + 1] != key)) {
                atomicOr(&F.uflags[u], UF_ID_SINGLE);
                // Which member's own id is it (not a post/void's pending id)?  b_qd holds each
                // entry's own id key until the sweep (plan 1).
                const u32 m = F.f_len[u];
                for (u32 j = 0; j < m; j++) {
                    if (F.b_qd[u + j] == key) atomicOr(&F.uflags[u + j], UF_MEMBER_NEW);
                }
            }
            if ((key & 0x80000000u) && !(first && (q + 1 == N || K[q + 1] != key))) {
                // A key shared by several units: a hash collision of different ids only orders them;
                // the id is unique if no other unit of the run names the same one.
                const Transfer* me = (const Transfer*)(P.events + (P.e0 + F.f_pe[u]) * 128);
                bool unique = true;
                u32 a = q;
                while (a > 0 && K[a - 1] == key) a--;
                for (u32 z = a; z < N && K[z] == key && unique; z++) {
                    if (z == q || V[z] == u) continue;
                    const Transfer* o = (const Transfer*)(P.events + (P.e0 + F.f_pe[V[z]]) * 128);
                    unique = o->id != me->id && !((P.eflags[F.f_pe[V[z]]] & (TF_POST | TF_VOID)) && o->pending_id == me->id);
                }
                if (unique && (P.eflags[F.f_pe[u]] & (TF_POST | TF_VOID)) == 0) atomicOr(&F.uflags[u], UF_ID_UNIQUE);
            }
            if (!first && V[q - 1] == u) continue;  // the same unit holds this resource twice
            if (!(key & 0x80000000u)) {
                atomicAdd(&F.nacct[u], 1u);
                F.rpos[u] = q;
            }
            if (first) continue;
            const u32 v = V[q - 1];
            atomicAdd(&F.need[u], 1u);
            const u32 slot = atomicAdd(&F.nsucc[v], 1u);
            F.succ[FLOW_RMAX * v + slot] = u;
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return;
        for (u32 f = FL_B * NT + tid; f < ndep; f += G * NT) {
            if (F.f_len[f] && F.need[f] == 0) {
                const u32 pos = atomicAdd(&F.words[FW_QTAIL], 1u);
                F.queue[pos] = f + 1;
            }
        }
        // Pack the run walker's view of every account-resource position (unit flags are final now).
        for (u32 q = FL_B * NT + tid; q < N; q += G * NT) {
            const u32 key = K[q];
            if (key == FLOW_SENT || (key & 0x80000000u)) continue;
            const u32 u = V[q];
            const u32 pe = F.f_pe[u];
            RunEntry x;
            x.u = u;
            x.pe = pe;
            const bool unit_ok = F.f_len[u] == 1 && F.nacct[u] == 1 && (F.uflags[u] & UF_ID_SINGLE);
            const u32 info = P.info[pe];
            const u16 fl = P.eflags[pe];
            x.dr = P.dr[pe];
            x.cr = P.cr[pe];
            x.rs = P.rs[pe];
            x.amt_lo = P.amt[pe];
            x.amt_hi = (info & HZ_AMT_HI) ? P.amt_hi[pe] : 0ULL;
            const bool member = unit_ok && (info & HZ_SPEC) && (info & HZ_ACCTS) && (info & 0xFF) == R_OK &&
                                !(fl & (TF_LINKED | TF_POST | TF_VOID | TF_BAL_DEBIT | TF_BAL_CREDIT));
            x.flags = fl | (member ? RUN_MEMBER : 0u);
            F.run[q] = x;
        }
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return;
    }
    const u64 ft1 = (FL_B == 0 && tid == 0) ? fl_now() : 0;
    fl_mark(g, tp, FP_LINK);
    if (!sequential) {
        __shared__ u64 s_bwv[FLOW_THREADS / 64][4];
        __shared__ u32 s_bwf[FLOW_THREADS / 64];
        __shared__ u32 s_bcnt;
        u64 tsb = 0;
        // The sweep's head table lives in s_dpre / s_wcnt: plan 1 and the sort are done with them.
        if (fl_bounds(P, F, ndep, N, cert64, gen, tsb, s_bwv, s_bwf, &s_bcnt, tp, s_dpre, (u64*)&s_wcnt[0][0])) {
            // Every unit decided and applied: replies and the pass close (workgroup 0) after all
            // workgroups' writes.
            if (tsb) atomicMax((unsigned long long*)&g->commit_timestamp, (unsigned long long)tsb);
            fl_grid_sync(g, G, gen, F);
            if (FL_B == 0 && tid == 0) {
                const u64 ft2 = fl_now();
                atomicAdd((unsigned long long*)&g->flow_plan_ticks, (unsigned long long)(ft1 - ft0));
                atomicAdd((unsigned long long*)&g->flow_run_ticks, (unsigned long long)(ft2 - ft1));
                atomicAdd(&g->flow_passes, 1u);
            }
            fl_mark(g, tp, FP_RUN);
            fl_finish(P, s_code, s_wave, s_list, 0, true, FL_B, G, FL_B == 0);
            fl_mark(g, tp, FP_REPLIES);  // workgroup 0's share
            return;
        }
        // Not certifiable: nothing was applied; the ordered run decides every unit.
        fl_grid_sync(g, G, gen, F);
        if (fl_stalled(g)) return;
    }
    // ---- run --------------------------------------------------------------------------------------
    u64 tsmax = 0;
    if (sequential) {
        if (FL_B != 0) return;
        Replay R;
        R.T = P.T;
        R.undo = seq_undo;
        R.undo_len = 0;
        R.undo_cap = seq_undo_cap;
        R.scope = false;
        R.failed = false;
        R.log_base = P.log_base;
        R.epoch = P.epoch;
        R.cert_global = cert_global;
        if (tid == 0) {
            for (u32 k = 0; k < nb && !R.failed; k++) {
                if (P.dep_count[k] == 0) continue;
                tsmax = max(tsmax, rp_batch<OP_CREATE_TRANSFERS>(P, R, P.b0 + k));
            }
        }
    } else {
        // Every lane of every workgroup (all co-resident, engine.hip flow_grid) takes tickets from one
        // queue in global memory; the state units share is read with agent-scope loads and each
        // unit's writes drain before its successors are released, so lanes on different CUs see
        // exactly what lanes of one workgroup would.
        const u32 nunits = *(volatile u32*)&F.words[FW_NUNITS];
        u32* qhead = &F.words[FW_QHEAD];
        u32* qtail = &F.words[FW_QTAIL];
        u32* done = &F.words[FW_DONE];
        Replay R;
        R.T = P.T;
        R.failed = false;
        R.log_base = P.log_base;
        R.epoch = P.epoch;
        R.cert_global = cert_global;
        R.cert64 = cert64;
        // Each lane: take a ticket (a queue position), wait for its unit, run it, release its
        // successors; the lane continues with the first successor that became ready (a chain of
        // units on one hot resource then never goes through the queue) and queues the others.
        // Not every ticket is filled (continued units skip the queue): a lane stops when all
        // units are done.
        u32 ticket = FLOW_SENT, spins = 0, next = FLOW_SENT;
        u64 w0 = 0;
        u32 runs = 0, run_units = 0;
        u64 exec_ticks = 0;  // this lane's time executing units (stats: flow_exec_ms)
        while (true) {
            u32 u;
            if (next != FLOW_SENT) {
                u = next;
                next = FLOW_SENT;
            } else {
                if (ticket == FLOW_SENT) ticket = atomicAdd(qhead, 1u);
                // At most nunits units are ever queued (each once), so a ticket past them is never
                // filled: the lane leaves instead of polling `done` with the others.
                if (ticket >= nunits) break;
                const u32 item = ticket < nunits
                                     ? __hip_atomic_load(&F.queue[ticket], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : 0;
                if (item == 0) {
                    // A waiting lane polls its queue slot, and the done counter only every
                    // FLOW_POLL_DONE-th time, sleeping between polls: the polls of idle waves
                    // otherwise crowd the lines the running units' atomics need.
                    if (spins % FLOW_POLL_DONE == 0 &&
                        __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nunits) {
                        break;
                    }
                    if (spins++ == 0) w0 = fl_now();
                    if (spins % 256 == 0 && (fl_expired(F, w0) || fl_stalled(g))) {
                        tb_panic(g, PANIC_FLOW_STALL);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(FLOW_POLL_SLEEP);
                    continue;
                }
                spins = 0;
                ticket = FLOW_SENT;
                u = item - 1;
            }
            u32 ran = 1;
            const u64 te = (u64)wall_clock64();
            // Run head?  Two load levels through the packed entry (position, then entry + resource)
            // instead of the unit's and the event's words.
            const u32 rq = F.rpos[u];
            const bool one_acct = F.nacct[u] == 1;
            bool head = false;
            u32 rr = 0;
            if (one_acct && rq < N) {
                const RunEntry& x = F.run[rq];
                rr = F.keys[0][rq];
                head = x.u == u && (x.flags & RUN_MEMBER) && rr != FLOW_SENT && !(rr & 0x80000000u);
            }
            if (head) {
                u64 ts = 0;
                u = fl_run_run(P, F, R, u, N, rq, rr, &ran, &ts);
                tsmax = max(tsmax, ts);
                runs++;
                run_units += ran;
            } else {
                tsmax = max(tsmax, fl_run_unit(P, F, R, u));
            }
            R.failed = false;  // a panic is recorded in g->panic; keep releasing successors
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this unit's writes land first
            exec_ticks += (u64)wall_clock64() - te;
            const u32 ns = F.nsucc[u];
            for (u32 k = 0; k < ns; k++) {
                const u32 s = F.succ[FLOW_RMAX * u + k];
                if (atomicSub(&F.need[s], 1u) == 1u) {
                    if (next == FLOW_SENT) {
                        next = s;
                    } else {
                        const u32 pos = atomicAdd(qtail, 1u);
                        __hip_atomic_store(&F.queue[pos], s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            atomicAdd(done, ran);
        }
        u64 et = exec_ticks;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) et += __shfl_xor((unsigned long long)et, off);
        if ((tid & 63) == 0 && et) atomicAdd((unsigned long long*)&g->flow_exec_ticks, (unsigned long long)et);
        u64 xc = R.xcount;  // the wave's transfers, one atomic
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) xc += __shfl_xor((unsigned long long)xc, off);
        if ((tid & 63) == 0 && xc) atomicAdd((unsigned long long*)&g->transfer_count, (unsigned long long)xc);
        if (runs) {
            atomicAdd((unsigned long long*)&g->flow_runs, (unsigned long long)runs);
            atomicAdd((unsigned long long*)&g->flow_run_units, (unsigned long long)run_units);
        }
        if (FL_B == 0 && tid == 0) {
            atomicAdd(&g->flow_passes, 1u);
            atomicAdd((unsigned long long*)&g->flow_units, (unsigned long long)nunits);
        }
        // Every workgroup's commit timestamp, then workgroup 0 closes the pass after all writes.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u64 m = tsmax;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m = max(m, (u64)__shfl_xor((unsigned long long)m, off));
        if ((tid & 63) == 0 && m) atomicMax((unsigned long long*)&g->commit_timestamp, (unsigned long long)m);
        tsmax = 0;
        fl_grid_sync(g, G, gen, F);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u64 m = tsmax;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (u64)__shfl_xor((unsigned long long)m, off));
    if ((tid & 63) == 0) s_tsmax[tid >> 6] = m;
    __syncthreads();
    u64 mm = 0;
    for (u32 k = 0; k < NT / 64; k++) mm = max(mm, s_tsmax[k]);
    if (FL_B == 0 && tid == 0) {
        const u64 ft2 = fl_now();
        atomicAdd((unsigned long long*)&g->flow_plan_ticks, (unsigned long long)(ft1 - ft0));
        atomicAdd((unsigned long long*)&g->flow_run_ticks, (unsigned long long)(ft2 - ft1));
    }
    // The replies: every workgroup its share after the parallel run (all are still here), workgroup
    // 0 alone after the sequential one (the others have left).
    const u32 parts = sequential ? 1u : G;
    fl_mark(g, tp, FP_RUN);
    fl_finish(P, s_code, s_wave, s_list, mm, true, FL_B, parts, FL_B == 0);
    fl_mark(g, tp, FP_REPLIES);  // workgroup 0's share
}
