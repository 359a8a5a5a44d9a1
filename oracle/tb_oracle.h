/*
 * tb_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of TigerBeetle's StateMachine commit path (create_accounts,
 * create_transfers, lookup_accounts, lookup_transfers), used as the parity
 * checker for the MI355X engine (tigerbeetle_amd/).  Only tests/, the smoke()
 * entry and bench.py's cpu_baseline leg may load this library.  It is never
 * part of the product path.
 *
 * Followed reference files (read-only snapshot under /root/reference):
 *   src/state_machine.zig:612-698   execute (batch loop, linked chains)
 *   src/state_machine.zig:700-736   execute_lookup_accounts / _transfers
 *   src/state_machine.zig:738-777   create_account / create_account_exists
 *   src/state_machine.zig:779-905   create_transfer / create_transfer_exists
 *   src/state_machine.zig:907-1077  post_or_void_pending_transfer (+ _exists)
 *   src/state_machine.zig:1152-1157 sum_overflows
 *   src/state_machine.zig:584-610   scope_open / scope_close
 *   src/lsm/cache_map.zig:266-309   scope rollback semantics (LIFO undo)
 *   src/tigerbeetle.zig:7-249       layouts, flags, result enums
 *
 * Parity pin: the 12 table-driven tests of src/state_machine.zig:1531-2074
 * (committed as tests/golden/state_machine_tables.txt) and the sum_overflows
 * vectors of :1164-1179.  The reference itself (Zig 0.11) cannot be built in
 * this image (no Zig toolchain, no network), so these fixtures are the pin.
 *
 * Panics: where the reference (ReleaseSafe) would trap on an integer overflow
 * or an `unreachable`/`.?`, the oracle returns TBO_STATUS_PANIC instead of
 * aborting the process.
 */
#ifndef TB_ORACLE_H
#define TB_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBO_STATUS_OK 0
#define TBO_STATUS_INVALID 1   /* bad arguments (operation, length, capacity) */
#define TBO_STATUS_PANIC 2     /* the reference would have panicked */

typedef struct tbo_state tbo_state;

tbo_state* tbo_init(uint64_t accounts_hint, uint64_t transfers_hint);
void tbo_deinit(tbo_state* s);
void tbo_reset(tbo_state* s);

/* StateMachine.commit (state_machine.zig:508-540). `operation` is 128..131.
 * `out_len` receives the reply size in bytes. */
int tbo_commit(tbo_state* s, uint8_t operation, uint64_t timestamp,
               const void* input, uint32_t input_len,
               void* output, uint32_t output_cap, uint32_t* out_len);

/* Test-only: the `setup` action of the table harness (state_machine.zig:1398-1407):
 * overwrite the four balances of an existing account.  balances = {dp, dpost, cp, cpost}
 * each as {lo, hi}.  Returns TBO_STATUS_PANIC if the account does not exist. */
int tbo_set_balances(tbo_state* s, uint64_t id_lo, uint64_t id_hi, const uint64_t balances[8]);

uint64_t tbo_commit_timestamp(const tbo_state* s);
uint64_t tbo_account_count(const tbo_state* s);
uint64_t tbo_transfer_count(const tbo_state* s);

/* Dump every account (128-B records) / transfer, sorted by id ascending.
 * Returns the number written (at most cap). */
uint64_t tbo_export_accounts(const tbo_state* s, void* out, uint64_t cap);
uint64_t tbo_export_transfers(const tbo_state* s, void* out, uint64_t cap);
/* Posted groove dump: pairs {pending_timestamp u64, fulfillment u64 (0 posted, 1 voided)},
 * sorted by timestamp. */
uint64_t tbo_export_posted(const tbo_state* s, uint64_t* out_pairs, uint64_t cap);

/* Shard test double (tests/harness/shard_double.py): CPU restatements of the per-rank primitives
 * of include/tbgpu_shard.h.  commit_routed: create_transfer for each event, whose timestamp
 * field holds its execute timestamp (execute's per-event body, state_machine.zig:641-662),
 * codes[i] = its result;
 * linked/post/void/balancing events are rejected (TBO_STATUS_INVALID).  fetch/upsert: as the
 * tbgpu_* calls of the same name.  balance_bound: max over accounts of dp+dpost, cp+cpost. */
int tbo_commit_routed(tbo_state* s, uint64_t n, const void* events, uint8_t* codes);
int tbo_fetch_accounts(const tbo_state* s, const uint64_t* ids, uint32_t n, void* out, uint8_t* found);
int tbo_fetch_transfers(const tbo_state* s, const uint64_t* ids, uint32_t n, void* out, uint8_t* state);
int tbo_upsert_accounts(tbo_state* s, const void* records, uint32_t n);
int tbo_upsert_transfers(tbo_state* s, const void* records, const uint8_t* state, uint32_t n);
void tbo_balance_bound(const tbo_state* s, uint64_t out[2]);

/* sum_overflows (state_machine.zig:1152-1157) exposed for its known-answer vectors. */
int tbo_sum_overflows_u64(uint64_t a, uint64_t b);
int tbo_sum_overflows_u128(uint64_t a_lo, uint64_t a_hi, uint64_t b_lo, uint64_t b_hi);

#ifdef __cplusplus
}
#endif
#endif
