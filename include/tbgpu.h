/*
 * tbgpu.h — C ABI of the MI355X batch-commit engine for TigerBeetle's create_accounts /
 * create_transfers state-machine path.
 *
 * Drop-in boundary: these entry points are what a Zig `StateMachineType` wrapper binds through
 * `@cImport` to replace the reference's synchronous commit:
 *
 *   reference interface                                   replaced by
 *   ----------------------------------------------------  ----------------------------------------
 *   StateMachine.init(allocator, grid, options)            tbgpu_init
 *     (src/state_machine.zig:264-278)
 *   StateMachine.deinit / reset (:280-299)                 tbgpu_deinit / tbgpu_reset
 *   StateMachine.prefetch (:345-506)                       tbgpu_prefetch (stages a pageable body)
 *   StateMachine.commit(client, op, timestamp, operation,  tbgpu_commit (one prepare) and
 *     input, output) -> usize (:508-540)                     tbgpu_commit_many (N prepares, one
 *                                                             device pass; same bytes as N commits)
 *   execute_lookup_accounts / _transfers (:700-736)        tbgpu_commit with operation 130 / 131
 *   `setup` action of the table tests (:1398-1407)         tbgpu_test_set_balances (test only)
 *   StateMachine.commit_timestamp field (:251)             tbgpu_commit_timestamp
 *
 * Layouts are the reference's extern structs (src/tigerbeetle.zig:7-249), identical to the C
 * client header (src/clients/c/tb_client.h:25-64,150-158): Account and Transfer are 128-byte
 * little-endian records, results are {uint32 index, uint32 result} pairs, only non-ok events,
 * ascending index.  Operation numbers: 128 create_accounts, 129 create_transfers,
 * 130 lookup_accounts, 131 lookup_transfers (src/state_machine.zig:208-214).
 *
 * Conventions (src/state_machine.zig:508-540):
 *   - Every call is synchronous unless its name ends in _async; calls never overlap.
 *   - Invalid input is reported through result codes, never through the status.
 *   - A non-zero status is TBGPU_STATUS_INVALID (bad arguments: the reference could not have
 *     been called that way), TBGPU_STATUS_PANIC (the reference would have trapped: an overflow
 *     assert, a failed invariant, `timestamp <= commit_timestamp`), or TBGPU_STATUS_DEVICE
 *     (a HIP error).  The Zig wrapper turns PANIC/DEVICE into @panic.
 *   - No allocation after tbgpu_init: every device buffer, pinned host buffer and HIP event is
 *     made there (tbgpu_debug_allocations, tbgpu_bench.h, counts them; tests/test_gpu_alloc.py
 *     holds the commit, prefetch and write-back entry points to zero).
 *   - A device panic (the reference would have trapped mid-commit) leaves state the reference
 *     never reaches, so the engine stops: every later call that changes state returns
 *     TBGPU_STATUS_PANIC until tbgpu_reset (or tbgpu_deinit).  Reads (exports, stats) still work.
 *   - Device exclusivity: the ordered fallback kernel (tb_flow) synchronises its workgroups with a
 *     software grid barrier among the workgroups it ADMITS at its start — those resident within
 *     ~50 us of the first one (at most a quarter of the CUs, shared among this process's engines on
 *     the device); a workgroup that starts later exits, and the admitted ones cover the pass.  So a
 *     co-tenant that holds CUs makes a pass slower, never a stall (tests/test_gpu_liveness.py
 *     launches tb_flow 8x over what the device holds).  tbgpu_init still checks once that a grid
 *     of that shape can be co-resident (within 200 ms) and fails with TBGPU_STATUS_DEVICE on a
 *     device other work holds; one engine process per device is the supported deployment.  Every
 *     wait stays bounded (PANIC_FLOW_STALL: an engine bug, never a hang).
 */
#ifndef TBGPU_H
#define TBGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBGPU_STATUS_OK 0
#define TBGPU_STATUS_INVALID 1
#define TBGPU_STATUS_PANIC 2
#define TBGPU_STATUS_DEVICE 3

#define TBGPU_OPERATION_CREATE_ACCOUNTS 128
#define TBGPU_OPERATION_CREATE_TRANSFERS 129
#define TBGPU_OPERATION_LOOKUP_ACCOUNTS 130
#define TBGPU_OPERATION_LOOKUP_TRANSFERS 131

/* batch_max.create_transfers for the production config (src/state_machine.zig:46-65). */
#define TBGPU_BATCH_EVENTS_MAX 8191u

/* Config flags. */
#define TBGPU_CONFIG_PROFILE (1u << 0) /* time every kernel with HIP events (tbgpu_get_stats) */
/* Ordered fallback on one lane in batch order (tb_replay) instead of the parallel flow path
 * (tb_flow); identical results, for cross-checking the two. */
#define TBGPU_CONFIG_SEQUENTIAL_FALLBACK (1u << 1)
/* Limit checks (tb_flow bounds): sweep whatever the first scan round leaves undecided in event
 * order (TBGPU_CONFIG_SWEEP_EARLY), or never sweep (TBGPU_CONFIG_SWEEP_OFF: rounds until they
 * converge, else the ordered run).  Identical results; for cross-checking the paths. */
#define TBGPU_CONFIG_SWEEP_EARLY (1u << 2)
#define TBGPU_CONFIG_SWEEP_OFF (1u << 3)
/* The sweep as one wave walking the undecided checks in event order, 64 a window (round 2's form),
 * instead of one walker per limit account.  Identical results; for cross-checking the two. */
#define TBGPU_CONFIG_SWEEP_WINDOW (1u << 4)

#define TBGPU_DEVICES_MAX 16u

typedef struct tbgpu_config {
    uint64_t accounts_max;      /* HBM account table capacity (the groove's object count) */
    uint64_t transfers_max;     /* HBM transfer store capacity (the whole ledger, over every device) */
    uint32_t pass_events_max;   /* max events in one device pass (tbgpu_commit_many); on a node: per
                                   source device and pass */
    uint32_t pass_batches_max;  /* max prepares in one device pass; on a node: per source device */
    int32_t device;             /* HIP device ordinal (device_count <= 1) */
    uint32_t flags;             /* TBGPU_CONFIG_* */
    /* SURVEY.md §8b device_mask.  device_count >= 2: a NODE engine over devices[0 .. device_count),
     * one shard per entry (an ordinal may repeat: logical shards sharing a GPU).  Every entry point
     * of this header works on a node engine with the same semantics: accounts hash-partitioned
     * (record and balances on their owner shard only), transfers on their home shard, each
     * create_transfers pass routed across the shards by kernels reading their peers' HBM over xGMI
     * (tigerbeetle_amd/csrc/node.h).  Not on a node: tbgpu_commit_device_async and the
     * tbgpu_shard.h primitives (they take one device's engine). */
    uint32_t device_count;
    int32_t devices[TBGPU_DEVICES_MAX];
} tbgpu_config;

typedef struct tbgpu tbgpu_t;

/* StateMachine.init: allocates every HBM table up front (static allocation). */
int tbgpu_init(const tbgpu_config* config, tbgpu_t** out);
void tbgpu_deinit(tbgpu_t* engine);
/* StateMachine.reset: empties every table, commit_timestamp = 0. */
int tbgpu_reset(tbgpu_t* engine);

/* StateMachine.commit for one prepare.  `input` holds `input_len` bytes (a multiple of 128 for
 * creates, of 16 for lookups); `output` receives the reply body and `*out_len` its size.
 * Byte-identical to the reference for every operation. */
int tbgpu_commit(tbgpu_t* engine, uint8_t operation, uint64_t timestamp, const void* input,
                 uint32_t input_len, void* output, uint32_t output_cap, uint32_t* out_len);

/* StateMachine.prefetch (src/state_machine.zig:345-506) for the prepare about to be committed.  The
 * objects are HBM-resident; what is staged is the body: a pageable create body starts its copy to
 * HBM at once, and the following tbgpu_commit of the same body (same pointer and length) only waits
 * for it.  A body in registered host memory (tbgpu_register_host: the message pool) is not staged:
 * the commit's first kernel reads it through, which measured faster than a DMA the replica's serial
 * prefetch -> commit leaves nothing to overlap with — except while the copy-out of an
 * asynchronous write-back written every few commits is in flight: then it is staged, so the commit
 * reads HBM and the copy-out need not wait for the commit's PCIe reads.  Completes
 * immediately (the reference allows the callback inside the call, src/lsm/groove.zig:723-742).
 * The staged copy belongs to the very next call only, if that call is tbgpu_commit of this body
 * (the replica's prefetch(op) -> commit(op)); any other call drops it.  The body must not change
 * between the two (a prepare message is immutable while its op commits, as in the reference). */
int tbgpu_prefetch(tbgpu_t* engine, uint8_t operation, const void* input, uint32_t input_len);

/* N consecutive prepares of the same create operation, pass_batches_max prepares per device pass
 * (tbgpu_commit_pipelined with chunk_batches = 0); identical results to N sequential tbgpu_commit
 * calls (timestamps strictly increasing). */
int tbgpu_commit_many(tbgpu_t* engine, uint8_t operation, uint32_t n, const uint64_t* timestamps,
                      const void* const* inputs, const uint32_t* input_lens, void* const* outputs,
                      uint32_t* out_lens);

/* Pipelined commit of N prepares from host memory: the replica's prefetch -> commit overlap
 * (src/state_machine.zig:345-506, src/vsr/replica.zig:3324-3665) with the objects HBM-resident.
 * Prepares are grouped into chunks of up to `chunk_batches` prepares (0: pass_batches_max); chunk
 * c+1's bodies cross PCIe while chunk c commits, and chunk c's replies come back as soon as it is
 * committed.  Bodies in memory registered with tbgpu_register_host (or otherwise pinned) move by
 * DMA; runs of address-contiguous prepares move as one copy.  Results are identical to N sequential
 * tbgpu_commit calls.  latency_ms (optional, N entries): per-prepare submit-to-reply time, from the
 * start of its chunk's PCIe copy to its reply landing in host memory (device clock).
 * On a node engine the bodies may also be in device memory (UVA pointers): a source shard's block of a
 * pass whose prepares sit back to back in that shard's own HBM is read in place (the node's
 * device-resident commit: prepares received or generated on each GPU), anything else is copied to it
 * (from another GPU over xGMI).  Replies still land in the host `outputs`. */
int tbgpu_commit_pipelined(tbgpu_t* engine, uint8_t operation, uint32_t n, const uint64_t* timestamps,
                           const void* const* inputs, const uint32_t* input_lens, void* const* outputs,
                           uint32_t* out_lens, uint32_t chunk_batches, double* latency_ms);

/* Device-resident throughput entry point: `events_dev` holds sum(batch_lens) events back to back
 * in HBM; batch k's reply is written to results_dev + 8*offset_k (offset_k = sum of earlier
 * batch lengths) and its byte count to reply_bytes_dev[k].  Enqueued on the engine's stream;
 * call tbgpu_sync() to wait and collect the status. */
int tbgpu_commit_device_async(tbgpu_t* engine, uint8_t operation, uint32_t n_batches,
                              const uint64_t* timestamps, const uint32_t* batch_lens,
                              const void* events_dev, void* results_dev, uint32_t* reply_bytes_dev);
int tbgpu_sync(tbgpu_t* engine);

/* Zero-copy create_transfers: the device address where the next `events` transfer records will be
 * stored (the transfer log from the engine's next position; the groove's insert,
 * src/lsm/groove.zig:950-1014, lands here).  Prepares placed there — by DMA from the message
 * buffers, by a peer, by a generator — and committed with tbgpu_commit_device_async(operation 129,
 * events_dev = *window) are committed IN PLACE: a committed transfer's record is its event with its
 * timestamp written, so the pass stores 8 bytes of it instead of copying 128 (results identical to
 * a copy commit).  The window is valid until the next call that stores transfers; INVALID when the
 * log cannot hold `events` more, or on a node engine. */
int tbgpu_log_window(tbgpu_t* engine, uint64_t events, void** window);

/* Host-memory registration for the replica's message pool (allocated once at init, like every
 * reference buffer): prepare bodies inside registered memory reach HBM by direct DMA. */
int tbgpu_register_host(tbgpu_t* engine, void* ptr, uint64_t bytes);
int tbgpu_unregister_host(tbgpu_t* engine, void* ptr);

/* StateMachine.commit_timestamp (src/state_machine.zig:251). */
uint64_t tbgpu_commit_timestamp(tbgpu_t* engine);

/* Test-only: the table harness `setup` action (src/state_machine.zig:1398-1407).
 * balances = {dp_lo, dp_hi, dpost_lo, dpost_hi, cp_lo, cp_hi, cpost_lo, cpost_hi}. */
int tbgpu_test_set_balances(tbgpu_t* engine, uint64_t id_lo, uint64_t id_hi,
                            const uint64_t balances[8]);

/* Parity read-back: every live record, sorted by id ascending; *count = records written. */
int tbgpu_export_accounts(tbgpu_t* engine, void* out, uint64_t cap, uint64_t* count);
int tbgpu_export_transfers(tbgpu_t* engine, void* out, uint64_t cap, uint64_t* count);
/* Posted groove (src/state_machine.zig:185-198): {pending_timestamp, fulfillment} pairs, sorted. */
int tbgpu_export_posted(tbgpu_t* engine, uint64_t* out_pairs, uint64_t cap, uint64_t* count);

/* Groove write-back for a durable replica (StateMachine.checkpoint / compact,
 * src/state_machine.zig:542-582; groove insert / upsert, src/lsm/groove.zig:902-963): the objects
 * changed since the previous call (or since init / reset) — accounts created or re-balanced (full
 * records, in no particular order: the groove sorts its mutable table itself), transfers created
 * (by timestamp), posted-groove entries created or changed ({pending timestamp, fulfillment} pairs,
 * by timestamp).  The cost follows the changes, not the tables.  If a buffer is too small the call
 * returns TBGPU_STATUS_INVALID with the sizes needed in *counts and nothing advances.  Buffers in
 * registered host memory (tbgpu_register_host) are filled by DMA. */
typedef struct tbgpu_delta_counts {
    uint64_t accounts;
    uint64_t transfers;
    uint64_t posted;
    uint64_t created_after;  /* accounts with a timestamp above this were created since the previous
                                write-back (groove insert); the others changed (groove upsert) */
} tbgpu_delta_counts;
int tbgpu_checkpoint_delta(tbgpu_t* engine, void* accounts_out, void* accounts_before_out, uint64_t accounts_cap,
                           void* transfers_out, uint64_t transfers_cap, uint64_t* posted_out, uint64_t posted_cap,
                           tbgpu_delta_counts* counts);
/* accounts_before_out (nullable, 64 B per account): {dp, dpost, cp, cpost} as of the previous
 * write-back (zero for accounts created since) — the old object a groove upsert diffs the balance
 * index trees against (src/lsm/groove.zig:925-963).
 * The buffers are checked before anything runs against what the write-back can emit at most
 * (transfers and posted entries: the transfer-log positions written since; accounts: two per such
 * position plus the listed creates, or every live account after creates the engine could not list):
 * a refused call returns those sizes in *counts and changes nothing. */

/* The same write-back without the wait (StateMachine.compact is asynchronous,
 * src/state_machine.zig:542-567; the replica's compact stage, src/vsr/replica.zig:3088-3091): the
 * state it describes is captured in stream order with the commits (the accounts the bar's transfers
 * name, with their balances; the next commits follow the capture), the rest is gathered on a
 * low-priority stream beside them, and the objects cross PCIe into the caller's buffers by DMA,
 * one slice after each one-prepare tbgpu_commit's body read (all at once after a commit whose body
 * tbgpu_prefetch staged; the rest at the wait).  A write-back every few commits whose objects
 * filled those bounds is sent at the bounds from the first commit after it (the bytes past the
 * counts land in the caller's buffers, unread; tbgpu_stats.write_backs_bound).
 * tbgpu_checkpoint_delta_wait returns the counts once the
 * objects have landed (transfers and posted entries sorted as above); until then the buffers belong
 * to the engine, and no other write-back may start.  Needs buffers registered with
 * tbgpu_register_host and large enough for the bounds above; otherwise (or past one slice of the
 * engine's write-back buffers) the call runs the synchronous write-back and the wait returns at
 * once.  A node engine (device_count >= 2) merges its shards' objects at the call (owners'
 * balances, homes' records, on the host) and its wait returns at once: the same contract, without the
 * single device's overlap with the next commits. */
int tbgpu_checkpoint_delta_async(tbgpu_t* engine, void* accounts_out, void* accounts_before_out, uint64_t accounts_cap,
                                 void* transfers_out, uint64_t transfers_cap, uint64_t* posted_out, uint64_t posted_cap);
int tbgpu_checkpoint_delta_wait(tbgpu_t* engine, tbgpu_delta_counts* counts);

/* Replica restart (StateMachine.open, src/state_machine.zig:322-334, then WAL replay from the
 * checkpoint): the HBM tables start empty while the forest holds the checkpointed objects.  The
 * wrapper's prefetch (src/state_machine.zig:345-506) reads the objects a prepare needs from the
 * forest and loads the ones the engine lacks: objects the engine already holds are newer and are
 * left as they are.  posted_state per transfer: 0 = no posted entry, 1 = posted, 2 = voided. */
int tbgpu_load_accounts(tbgpu_t* engine, const void* accounts, uint32_t n);
int tbgpu_load_transfers(tbgpu_t* engine, const void* transfers, const uint8_t* posted_state, uint32_t n);

/* Bounded residency.  The transfer log holds tbgpu_config.transfers_max records; a replica that
 * outlives it evicts what its forest already holds and loads it back when a prepare names it — the
 * reference's groove keeps every transfer reachable through its cache and LSM levels
 * (src/lsm/groove.zig:602-898), loaded by prefetch before commit (src/state_machine.zig:419-467).
 *   tbgpu_evict_transfers: drops the transfers the last write-back (tbgpu_checkpoint_delta) covered,
 *     except the newest `keep` log positions; the rest of the log is compacted and re-indexed.
 *     *evicted = transfers dropped.  Synchronous.  Only right after a write-back: with an
 *     asynchronous write-back in flight, or any log position written since the last one (a commit,
 *     a load), it returns TBGPU_STATUS_INVALID and changes nothing (an unwritten post / void may name
 *     a pending transfer the cut would drop, and the next write-back needs that record).
 *   tbgpu_transfers_maybe_cold: for n ids ({lo, hi} pairs), cold[i] = 1 when the engine does not
 *     hold id i and may have evicted it (a Bloom filter of evicted ids: false positives only).  The
 *     wrapper's prefetch loads the cold ids its forest holds (tbgpu_load_transfers, with their posted
 *     state) before the commit of a prepare that names them (its ids and post / void pending ids);
 *     an id it does not load is taken as absent, as the reference's groove would report it.
 * A node engine evicts per home shard (each shard's log keeps its share of `keep`; log_used in
 * tbgpu_stats is the fullest shard's fill in units of the node's capacity) and answers each id's
 * cold query on its home shard. */
int tbgpu_evict_transfers(tbgpu_t* engine, uint64_t keep, uint64_t* evicted);
int tbgpu_transfers_maybe_cold(tbgpu_t* engine, const uint64_t* ids, uint32_t n, uint8_t* cold);

/* The replica writes StateMachine.commit_timestamp itself: the header timestamp after every commit
 * (src/vsr/replica.zig:3664-3665) and the checkpoint's value on open / state sync.  The wrapper
 * pushes a changed value here before the next commit, so the engine asserts what the reference
 * asserts (timestamp > commit_timestamp, src/state_machine.zig:519). */
int tbgpu_set_commit_timestamp(tbgpu_t* engine, uint64_t timestamp);

typedef struct tbgpu_stats {
    uint64_t passes;
    uint64_t events;
    uint64_t dependent_events;   /* events replayed by the ordered fallback kernel */
    uint64_t accounts;           /* live accounts */
    uint64_t transfers;          /* live transfers */
    /* With TBGPU_CONFIG_PROFILE: total device ms and launch count per kernel. */
    double ms_validate;          /* tb_transfers_validate / tb_accounts_validate */
    double ms_resolve;           /* tb_*_resolve (classify + chains + apply + replies) */
    double ms_replay;            /* tb_replay (ordered fallback) */
    double ms_clear;             /* dedup table clears */
    uint64_t launches_validate, launches_resolve, launches_replay, launches_clear;
    double ms_apply;             /* tb_apply_legs (per-account sums of the balance legs) */
    uint64_t launches_apply;
    uint64_t flow_passes;        /* passes whose dependent events ran on the parallel flow path */
    uint64_t flow_units;         /* chains / single dependent events the flow path executed */
    uint64_t flow_runs;          /* runs: single-resource sequences walked with the balance in registers */
    uint64_t flow_run_units;     /* units covered by runs */
    double flow_plan_ms;         /* tb_flow wall time planning the dependent events (workgroup 0) */
    double flow_run_ms;          /* tb_flow wall time executing them in order (workgroup 0) */
    uint64_t bounds_passes;      /* passes whose limit checks were all decided by bounds scans (no ordered run) */
    uint64_t bounds_units;       /* dependent events they decided */
    uint64_t bounds_rounds;      /* scan rounds they took (and those of abandoned attempts) */
    uint64_t bounds_skipped;     /* dependent passes with an event the bounds do not cover */
    uint64_t bounds_abandoned;   /* passes whose bounds did not converge (ordered run instead) */
    uint64_t bounds_swept;       /* units decided by the in-order sweep after the rounds */
    double sweep_ms;             /* tb_flow wall time of the sweeps (one wave) */
    double sweep_loop_ms;        /* ... of it resolving windows in order */
    double sweep_wait_ms;        /* ... of it waiting for memory between windows */
    uint64_t sweep_u64_passes;   /* sweeps in the u64 X/Y form (bound + S >= 2^63: no signed slack) */
    double flow_exec_ms;         /* tb_flow run: time lanes spent executing units, summed over lanes */
    double flow_phase_ms[8];     /* tb_flow wall time by phase: plan, sort, link, bounds setup, bounds
                                    rounds, sweep, run (or applying the bounds), replies */
    /* The sweep's per-account walkers (k_flow.h fl_walk): segments walked, heavy segments (a wave
     * each); over the heavy walkers: positions, windows, stops at a partner's open unit, blocked
     * returns, blocked ms (summed over walkers), and the longest segment (positions). */
    uint64_t walk_segments, walk_heavy, walk_heavy_positions, walk_heavy_windows, walk_heavy_stops,
        walk_heavy_blocks;
    double walk_heavy_blocked_ms;
    uint64_t walk_longest;
    /* The critical walker (the longest segment's, a wave each): windows, waits at a partner's open
     * unit, ms spent waiting, ms in all (summed over passes). */
    uint64_t walk_crit_windows, walk_crit_blocks;
    double walk_crit_wait_ms, walk_crit_ms;
    uint64_t walk_dbg[4]; /* diagnostics: a stalled walker's kind | segment, unit, status, verdict bits */
    /* With TBGPU_CONFIG_PROFILE, the device clock of the launch itself (s_memrealtime): from the
     * first workgroup's start to the last workgroup's end, summed over launches, for validate,
     * resolve and apply (the HIP-event times above also hold the dispatch of each launch). */
    double span_ms[3];
    uint64_t span_launches[3];
    /* Node engines: create_transfers passes routed whole (clean), split (the dependent subsequence
     * committed by the sequencer, the rest routed), or sequenced whole (no overflow certificate);
     * events the sequencer committed. */
    uint64_t node_passes_clean, node_passes_split, node_passes_whole, node_sequenced_events;
    /* HBM bytes of the account table (hot records, balances, cold fields, marks): this engine's; on a
     * node engine the largest shard's, and each shard's in node_shard_account_bytes — the accounts it
     * owns (1/N of the ledger) plus an import room for foreign accounts' hot records (the ledger's
     * accounts, or two per event of a routed sub-pass when that is fewer). */
    uint64_t account_table_bytes;
    uint64_t node_shard_account_bytes[16];
    /* Bounded residency (tbgpu_evict_transfers): transfers evicted so far, transfer-log positions in
     * use and in all (a wrapper evicts when the log fills; a node: the sums over its shards, log_used
     * the fullest shard's fill times the node's capacity). */
    uint64_t transfers_evicted, log_used, log_capacity;
    /* Asynchronous write-backs started (tbgpu_checkpoint_delta_async), and of them those whose
     * copy-out was sent at its bounds from the first commit after it (a write-back every few ops;
     * the bytes past the counts land in the caller's buffers unread); since tbgpu_init. */
    uint64_t write_backs_async, write_backs_bound;
} tbgpu_stats;

int tbgpu_get_stats(tbgpu_t* engine, tbgpu_stats* stats);
void tbgpu_reset_stats(tbgpu_t* engine);

/* vsr.checksum (src/vsr/checksum.zig:50-74): Aegis-128L MAC, zero key and nonce, 16 tag bytes
 * (the u128 in little-endian order).  Host-only (touches no device): the AOF reader verifies
 * header and body checksums with it (src/aof.zig:214-218, src/vsr.zig:405-437). */
void tbgpu_checksum(const void* data, uint64_t len, uint8_t out[16]);

/* Last error message (thread-local, static storage). */
const char* tbgpu_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
