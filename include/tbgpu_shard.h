/*
 * tbgpu_shard.h — multi-GPU sharding primitives of the MI355X commit engine: one engine per GPU,
 * one process per GPU, the collectives (RCCL over xGMI) issued by the host between these calls
 * (tigerbeetle_amd/sharded.py).
 *
 * The reference commits on one thread of one replica (src/vsr/replica.zig:3045-3102); SURVEY.md
 * §8e asks for one 8-GPU node with cross-shard traffic routed by all-to-all.  Partition:
 *   - Account records are replicated (all fields but the balances are immutable after
 *     create_account, src/state_machine.zig:738-765): every rank commits every create_accounts
 *     prepare, with identical results.
 *   - Account balances are per-rank partial sums: each rank applies the legs of the transfers
 *     it owns; true balance = sum over ranks (every partial is non-negative, so every partial is
 *     <= the true balance, and the sum of the ranks' `bound`s bounds every true balance).
 *   - A transfer (record, id index entry, posted state) lives on tbgpu_home(id, world).
 *
 * A create_transfers pass is CLEAN when no event is linked / post / void / balancing, no debit or
 * credit account carries a limit flag, and (sum of bounds) + (sum of S) fits u128.  Each event's
 * result then depends only on state its home holds (create_transfer reads balances only for
 * balancing :826-846, overflow :848-861 and limits :863-868), so a clean pass is:
 *     tbgpu_route_plan         (every rank: classify + group its events by home)
 *     all-to-all of the events (each carrying its execute timestamp)
 *     tbgpu_commit_routed_async (every home: the normal kernels, per-event timestamps and codes)
 *     all-to-all of the result codes back
 *     tbgpu_route_replies_async (every rank: sparse replies per prepare).
 * A DIRTY pass is committed by rank 0 on a scratch engine after prefetching what it reads — the
 * reference's own prefetch -> commit split (src/state_machine.zig:345-506) — with the fetch and
 * upsert calls below, then written back to the homes.
 */
#ifndef TBGPU_SHARD_H
#define TBGPU_SHARD_H

#include <stdint.h>

#include "tbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TBGPU_WORLD_MAX 64u

/* Dirty bits of a route plan. */
#define TBGPU_DIRTY_FLAGS 1u /* linked / post / void / balancing event */
#define TBGPU_DIRTY_LIMIT 2u /* debit or credit account with a limit flag (tigerbeetle.zig:31-39) */

/* Certificate handed to a routed commit (the router's global overflow proof). */
#define TBGPU_CERT_U128 1u /* sum of bounds + sum of S < 2^128 */
#define TBGPU_CERT_U64 2u  /* ... and < 2^64: balance adds never carry out of the low word */

/* Home rank of a transfer id (host function; needs no device). */
uint32_t tbgpu_home(uint64_t id_lo, uint64_t id_hi, uint32_t world);
/* Vectorised: ids = n {lo, hi} pairs. */
void tbgpu_homes(const uint64_t* ids, uint64_t n, uint32_t world, uint32_t* out);

/* Allocate the routing scratch for passes of up to `events_max` local events (call once). */
int tbgpu_route_init(tbgpu_t* engine, uint32_t world, uint64_t events_max);

typedef struct tbgpu_route_plan {
    uint64_t send_counts[TBGPU_WORLD_MAX]; /* events for each home, in rank order */
    uint64_t sum_lo, sum_hi;               /* S: saturating sum of every amount of the pass */
    uint64_t bound_lo, bound_hi;           /* this engine's balance bound before the pass */
    uint32_t dirty;                        /* TBGPU_DIRTY_* */
    uint32_t reserved;
} tbgpu_route_plan;

/* Classify this rank's share of a create_transfers pass (n_batches prepares of batch_lens[k]
 * events at timestamps[k], back to back in events_dev) and group it by home: send_events_dev
 * receives the events home by home (128 B each, the timestamp field set to the event's execute
 * timestamp, state_machine.zig:645), each home's run in input order; slot_dev[e] = event e's send
 * position, or 0xFFFFFFFF for an event whose timestamp field was non-zero (it fails with
 * timestamp_must_be_zero, :643, before reading any state: answered here, never routed).
 * Synchronous (the plan is needed on the host for the collectives). */
int tbgpu_route_plan_build(tbgpu_t* engine, uint32_t n_batches, const uint64_t* timestamps,
                           const uint32_t* batch_lens, const void* events_dev, const uint8_t* skip_dev,
                           void* send_events_dev, uint32_t* slot_dev, tbgpu_route_plan* plan);
/* skip_dev (nullable, one byte per event): non-zero = a dependent event of a split dirty pass,
 * committed by the pass's sequencer instead: not routed, slot 0xFFFFFFFE (its amount still counts
 * in S). */

/* Dependency classes of this rank's share of a dirty pass (dep_dev, one byte per event, synchronous):
 * 1 linked-chain member, 2 post/void, 4 balancing, 8 touches an account with a limit flag, 16
 * touches one of the n_marked accounts (host array of {lo, hi} ids sorted by hi then lo: the
 * accounts the pass's balancing events touch, state_machine.zig:826-846). */
/* home(id) of n {lo, hi} ids held in device memory (out_dev: one byte each).  Synchronous. */
int tbgpu_route_homes(tbgpu_t* engine, const uint64_t* ids_dev, uint64_t n, uint32_t world, uint8_t* out_dev);

int tbgpu_route_dependents(tbgpu_t* engine, uint32_t n_batches, const uint32_t* batch_lens, const void* events_dev,
                           const uint64_t* marked_ids, uint32_t n_marked, uint8_t* dep_dev);

/* Commit `n` routed events (this home's share of a clean pass, in global order, each carrying its
 * execute timestamp); codes_dev[i] = result code of event i.  `cert` = TBGPU_CERT_*.  `ts_max` =
 * the last timestamp of the global pass (host-side ordering state).  Enqueued; tbgpu_sync() waits. */
int tbgpu_commit_routed_async(tbgpu_t* engine, uint64_t n, const void* events_dev, uint64_t ts_max,
                              uint32_t cert, uint8_t* codes_dev);

/* Owner-partitioned balances: an account's balances live on owner(id) =
 * tbgpu_home(id, world); every other rank holds zeros for it.  This is tbgpu_commit_routed_async
 * for rank `self` of `world`, except that the home applies no balance itself: every committed
 * transfer's two legs (state_machine.zig:870-880) are written to legs_dev, grouped by owner —
 * owner o's legs at legs_dev + o * legs_cap * 40 B, {id lo, id hi, amount lo, amount hi, field
 * (0 dp, 1 dpost, 2 cp, 3 cpost)} as u64 words — and leg_counts_dev[o] = their number.  legs_cap
 * >= 2 n.  Enqueued. */
int tbgpu_commit_routed_owner_async(tbgpu_t* engine, uint64_t n, const void* events_dev, uint64_t ts_max,
                                    uint32_t cert, uint8_t* codes_dev, uint32_t world, uint32_t self,
                                    void* legs_dev, uint64_t legs_cap, uint64_t* leg_counts_dev);

/* Owner side: add n received legs (the layout above, back to back) to this rank's balances.  A leg
 * for an account the table lacks is a PANIC (accounts are replicated).  Synchronous. */
int tbgpu_apply_owner_legs_async(tbgpu_t* engine, const void* legs_dev, uint64_t n, uint32_t cert);

/* Sparse per-prepare replies from the returned codes (codes_dev in send order): batch k's reply
 * at results_dev + 8*offset_k, its size in reply_bytes_dev[k]. Enqueued. */
int tbgpu_route_replies_async(tbgpu_t* engine, uint32_t n_batches, const uint32_t* batch_lens,
                              const uint32_t* slot_dev, const uint8_t* codes_dev, void* results_dev,
                              uint32_t* reply_bytes_dev);

/* Dirty-pass prefetch (host buffers, synchronous).  ids = n {lo, hi} pairs.
 * Accounts: out (128 B each, this rank's partial balances), found[i] in {0, 1}.
 * Transfers: out (128 B each), state[i] = 0 absent, 1 + {0 none, 1 posted, 2 voided}. */
int tbgpu_fetch_accounts(tbgpu_t* engine, const uint64_t* ids, uint32_t n, void* out, uint8_t* found);
int tbgpu_fetch_transfers(tbgpu_t* engine, const uint64_t* ids, uint32_t n, void* out, uint8_t* state);

/* Dirty-pass write-back (host buffers, synchronous).  Accounts: insert verbatim, or overwrite the
 * four balances of an existing account (keeps the balance bound).  Transfers: insert verbatim
 * (state as in fetch; 0 = no posted entry), or set the posted state of an existing one. */
int tbgpu_upsert_accounts(tbgpu_t* engine, const void* records, uint32_t n);
int tbgpu_upsert_transfers(tbgpu_t* engine, const void* records, const uint8_t* state, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
