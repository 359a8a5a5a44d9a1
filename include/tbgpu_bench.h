/*
 * tbgpu_bench.h — synthetic workload generation for bench.py and the parity tests (same library
 * as tbgpu.h).  Not part of the StateMachine boundary.
 */
#ifndef TBGPU_BENCH_H
#define TBGPU_BENCH_H

#include <stdint.h>

#include "tbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbgpu_workload {
    uint64_t seed;
    uint64_t account_count;    /* accounts 0..account_count-1 exist (ids by IdPermutation.inversion) */
    uint32_t kind;             /* 0: uniform dr != cr, no flags (BASELINE config C2)
                                  1: Zipf(zipf_s) dr/cr over a rank permutation; the first transfers
                                     fund every limit account from account 0 (C3)
                                  2: uniform, 20% linked chains (5% chain-breaking), pending with
                                     timeouts, post/void of earlier transfers, balancing (C4) */
    uint32_t limit_permille;   /* accounts with debits_must_not_exceed_credits, per mille */
    double zipf_s;             /* kind 1: Zipf exponent (BASELINE C3: 1.2) */
    uint32_t hot_limited;      /* kind 1: the hottest Zipf ranks [0, hot_limited) also get
                                  debits_must_not_exceed_credits (the adversarial C3: a limit
                                  account on the hot path); account generation needs account_count */
    uint32_t reserved;
} tbgpu_workload;

/* Write `count` Account events for account indices [first, first+count) into device memory. */
int tbgpu_bench_generate_accounts(tbgpu_t* engine, void* out_dev, uint64_t first, uint64_t count,
                                  const tbgpu_workload* w);
/* Write `count` Transfer events for transfer indices [first, first+count) into device memory. */
int tbgpu_bench_generate_transfers(tbgpu_t* engine, void* out_dev, uint64_t first, uint64_t count,
                                   const tbgpu_workload* w);

/* Restore the post-account-creation state between bench steps: empty the transfer store and the
 * posted groove, zero every account balance.  Accounts and commit_timestamp are kept. */
int tbgpu_bench_reset_transfers(tbgpu_t* engine);
/* Device duration (ms) of every pass since the last tbgpu_reset_stats (TBGPU_CONFIG_PROFILE):
 * a prepare's reply is available when its pass completes, so this is the batch latency. */
int tbgpu_bench_pass_latencies(tbgpu_t* engine, double* out_ms, uint64_t cap, uint64_t* count);

/* Which kernels TBGPU_CONFIG_PROFILE times with HIP events (every event pair on the stream costs
 * a little): bit 1 << kind, kinds 0 validate, 1 resolve, 2 replay/flow, 3 clears, 4 whole pass,
 * 5 apply_legs.  Default: all.  Any of validate, resolve, apply or TBGPU_PROF_SPANS also stamps the
 * launch spans of validate, resolve and apply on the device clock (tbgpu_stats.span_ms); SPANS alone
 * records no event pair (each pair on the stream separates two launches by a few microseconds). */
enum { TBGPU_PROF_VALIDATE = 1, TBGPU_PROF_RESOLVE = 2, TBGPU_PROF_REPLAY = 4, TBGPU_PROF_CLEAR = 8,
       TBGPU_PROF_PASS = 16, TBGPU_PROF_APPLY = 32, TBGPU_PROF_ALL = 63, TBGPU_PROF_SPANS = 64 };
int tbgpu_bench_profile_mask(tbgpu_t* engine, uint32_t mask);
/* Passes of at least this many create_transfers events apply balances through sorted legs
 * (k_apply.h), smaller ones with atomics (default 262144; tests set 0 to cover legs on small
 * passes).  Exact either way. */
int tbgpu_bench_legs_min_events(tbgpu_t* engine, uint32_t events);
/* The limit-check sweep's walkers (k_flow.h fl_walk): up to this many heavy segments are walked
 * merged by one wave (default 63); 0: every heavy segment on a wave of its own. */
int tbgpu_bench_walk_merge_max(tbgpu_t* engine, uint32_t segments);
/* Liveness tests: launch the ordered fallback (tb_flow) with this many workgroups (0: its own
 * grid), more than the device can hold at once — the ones that are not resident when its admission
 * closes exit (k_flow.h fl_admit), as under a co-tenant. */
int tbgpu_bench_flow_launch(tbgpu_t* engine, uint32_t workgroups);

/* The memory-access mix of tb_transfers_validate without its logic, on scratch buffers sized like
 * this engine's account table and transfer index, for `transfers` events (one pass): mean ms of
 * {stream, probe, cas, stream+probe, stream+cas, probe+cas, all three} (k_workload.h).  The
 * kernel's practical bound for its access pattern; allocates and frees its own buffers. */
int tbgpu_bench_access_mix(tbgpu_t* engine, uint64_t transfers, double out_ms[7]);

/* Size-independent properties of a full-size run without exporting the tables: the sums of the
 * four balance fields over every account (u128, as {lo, hi} pairs: dp, dpost, cp, cpost), the live
 * accounts, and — on a node engine — the accounts whose balances sit on a shard that is not their
 * owner (must be 0).  On a node the sums are over every shard. */
typedef struct tbgpu_ledger_summary {
    uint64_t sums[8];
    uint64_t accounts;
    uint64_t stray;
} tbgpu_ledger_summary;
int tbgpu_bench_ledger_summary(tbgpu_t* engine, tbgpu_ledger_summary* out);

/* Take the current state as written back (tbgpu_checkpoint_delta's snapshot and positions), so the
 * next write-back covers only what is committed after this call: the bench times a bar's write-back
 * at any number of stored objects without first writing them all back. */
int tbgpu_bench_checkpoint_mark(tbgpu_t* engine);

/* A node engine's shard d (tbgpu_config.devices[d]) as an engine handle of its own, for the bench's
 * per-GPU buffers: tbgpu_device_alloc / _free, tbgpu_copy_* and the generators on that handle work on
 * shard d's device (the prepares of a device-resident node commit are generated in their source
 * GPU's HBM).  Owned by the node: never tbgpu_deinit it, and commit only through the node. */
int tbgpu_bench_node_shard(tbgpu_t* engine, uint32_t shard, tbgpu_t** out);

/* Device memory helpers for callers without a device allocator (ctypes users). */
int tbgpu_device_alloc(tbgpu_t* engine, uint64_t bytes, void** out);
int tbgpu_device_free(tbgpu_t* engine, void* ptr);
int tbgpu_copy_to_host(tbgpu_t* engine, void* dst, const void* src_dev, uint64_t bytes);
int tbgpu_copy_to_device(tbgpu_t* engine, void* dst_dev, const void* src, uint64_t bytes);

/* Device-side timing of the last tbgpu_sync'ed work: elapsed ms between two markers recorded on
 * the engine stream. */
int tbgpu_marker(tbgpu_t* engine, uint32_t slot);          /* slot < 16 */
double tbgpu_marker_elapsed_ms(tbgpu_t* engine, uint32_t a, uint32_t b);

/* Device allocations, pinned host allocations and HIP events the library has made so far (every
 * engine of the process): a test reads it around commits to hold tbgpu.h's "no allocation after
 * tbgpu_init". */
uint64_t tbgpu_debug_allocations(void);

#ifdef __cplusplus
}
#endif
#endif
