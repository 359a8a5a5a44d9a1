// state_machine.hpp — C++ host mirror of the reference's StateMachine plugin interface, backed by
// the MI355X engine's C ABI (include/tbgpu.h).
//
// The reference's replica drives a comptime duck-typed `StateMachineType`
// (src/state_machine.zig:28-1150; contract in SURVEY.md §8b).  The host side stays in the
// reference's language there (Zig); no Zig toolchain exists in this image, so this is the same
// interface in C++ — what a Zig `@cImport` wrapper would call, one level up:
//
//   reference member (src/state_machine.zig)          here
//   ------------------------------------------------  ---------------------------------------------
//   Operation (:208-214)                               tb::Operation
//   Options (:216-221)                                 tb::Options (+ HBM sizing)
//   init(allocator, grid, options) !Self (:264-278)    StateMachine(const Options&) (throws DeviceError)
//   deinit (:280-289) / reset (:291-317)                ~StateMachine() / reset()
//   open(callback) (:319-334)                          open(cb)
//   prepare(operation, input) (:336-343)               prepare(op, input, len)
//   prefetch(callback, op, operation, input) (:345)    prefetch(cb, op, operation, input, len)
//   commit(client, op, timestamp, operation, input,    commit(client, op, timestamp, operation, input,
//          output) usize (:508-540)                           len, output) -> bytes written
//   compact(callback, op) / checkpoint(callback)       compact(cb, op) / checkpoint(cb)
//     (:542-582)
//   prepare_timestamp / commit_timestamp (:250-251)    prepare_timestamp / commit_timestamp
//
// Error behaviour follows the reference: invalid events are result codes; an invariant the
// reference asserts (or an integer overflow it would trap on in ReleaseSafe) throws tb::Panic —
// the replica's @panic; a HIP failure throws tb::DeviceError.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

extern "C" {
#include "../../include/tbgpu.h"
}

namespace tb {

using u128 = unsigned __int128;

// src/state_machine.zig:208-214 (vsr_operations_reserved = 128).
enum class Operation : uint8_t {
    create_accounts = 128,
    create_transfers = 129,
    lookup_accounts = 130,
    lookup_transfers = 131,
};

// config.zig:137 / vsr.zig:401: message_size_max (1 MiB) - header (128 B).
constexpr size_t message_body_size_max = (1u << 20) - 128;
// batch_max (state_machine.zig:46-65): body / max(sizeof(Event), sizeof(Result)) = 8191 for every
// operation of the production config.
constexpr uint32_t batch_max = message_body_size_max / 128;

// src/tigerbeetle.zig:7-29.
struct alignas(16) Account {
    u128 id;
    u128 debits_pending;
    u128 debits_posted;
    u128 credits_pending;
    u128 credits_posted;
    u128 user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t reserved;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
};
static_assert(sizeof(Account) == 128, "Account is a 128-byte extern struct");

// src/tigerbeetle.zig:64-89.
struct alignas(16) Transfer {
    u128 id;
    u128 debit_account_id;
    u128 credit_account_id;
    u128 amount;
    u128 pending_id;
    u128 user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t timeout;
    uint32_t ledger;
    uint16_t code;
    uint16_t flags;
    uint64_t timestamp;
};
static_assert(sizeof(Transfer) == 128, "Transfer is a 128-byte extern struct");

// Create*sResult (tigerbeetle.zig:224-249): {index, result}, only non-ok events.
struct CreateResult {
    uint32_t index;
    uint32_t result;
};
static_assert(sizeof(CreateResult) == 8, "8-byte result");

namespace AccountFlags {  // tigerbeetle.zig:31-62
constexpr uint16_t linked = 1 << 0;
constexpr uint16_t debits_must_not_exceed_credits = 1 << 1;
constexpr uint16_t credits_must_not_exceed_debits = 1 << 2;
}  // namespace AccountFlags

namespace TransferFlags {  // tigerbeetle.zig:91-104
constexpr uint16_t linked = 1 << 0;
constexpr uint16_t pending = 1 << 1;
constexpr uint16_t post_pending_transfer = 1 << 2;
constexpr uint16_t void_pending_transfer = 1 << 3;
constexpr uint16_t balancing_debit = 1 << 4;
constexpr uint16_t balancing_credit = 1 << 5;
}  // namespace TransferFlags

// Result names in declaration order (value == index, tigerbeetle.zig:109-249).
const std::vector<std::string>& create_account_result_names();
const std::vector<std::string>& create_transfer_result_names();

struct Options {
    // Reference options (state_machine.zig:216-221): accepted for interface parity; the HBM
    // tables hold every object, so there is no cache to size.
    uint32_t lsm_forest_node_count = 0;
    uint32_t cache_entries_accounts = 0;
    uint32_t cache_entries_transfers = 0;
    uint32_t cache_entries_posted = 0;
    // HBM sizing (static allocation at init, as the reference's grooves).
    uint64_t accounts_max = 1 << 16;
    uint64_t transfers_max = 1 << 20;
    uint32_t pass_events_max = 8190 * 64;
    uint32_t pass_batches_max = 512;
    int32_t device = 0;
    // Two or more entries: a node engine, one shard per listed device (tbgpu_config.devices).
    std::vector<int32_t> devices;
    bool profile = false;
};

struct Panic : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct DeviceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// One groove write-back (tbgpu_checkpoint_delta): what checkpoint() hands to the durable
// replica's forest — accounts (128-B records, in no particular order, each with its 64-B balances as
// of the previous write-back), transfers (128-B records, by timestamp), posted pairs {pending
// timestamp, fulfillment} (by timestamp).  Views of the state machine's registered write-back
// buffers: valid until the next write-back.
struct Delta {
    const uint8_t* accounts = nullptr;
    const uint8_t* accounts_before = nullptr;
    uint64_t account_count = 0;
    uint64_t created_after = 0;  // accounts with a later timestamp are new (insert)
    const uint8_t* transfers = nullptr;
    uint64_t transfer_count = 0;
    const uint64_t* posted = nullptr;
    uint64_t posted_count = 0;
};

class StateMachine {
public:
    using Callback = std::function<void(StateMachine&)>;
    using WriteBack = std::function<void(const Delta&)>;

    explicit StateMachine(const Options& options);
    ~StateMachine();
    StateMachine(const StateMachine&) = delete;
    StateMachine& operator=(const StateMachine&) = delete;

    void reset();
    void open(const Callback& callback);
    // Input / output buffers are the prepare body and the reply body (align 16 in the reference).
    void prepare(Operation operation, const void* input, size_t input_len);
    void prefetch(const Callback& callback, uint64_t op, Operation operation, const void* input, size_t input_len);
    size_t commit(u128 client, uint64_t op, uint64_t timestamp, Operation operation, const void* input,
                  size_t input_len, void* output);
    // N consecutive prepares of one create operation in one device pass: identical results to N
    // commit() calls (the throughput entry point; the replica may batch committed prepares).
    std::vector<size_t> commit_many(Operation operation, const std::vector<uint64_t>& timestamps,
                                    const std::vector<const void*>& inputs, const std::vector<size_t>& input_lens,
                                    const std::vector<void*>& outputs);
    // At the last op of every bar (config.zig:143 lsm_batch_multiple = 64) with `write_back` set:
    // hands the PREVIOUS bar's changes to write_back (they crossed PCIe while this bar committed)
    // and starts this bar's without waiting (tbgpu_checkpoint_delta_async: the reference's compact
    // is asynchronous, src/state_machine.zig:542-567); then calls back.  The forest so trails the
    // engine by at most one bar, and checkpoint() closes the gap.
    void compact(const Callback& callback, uint64_t op);
    // compact's write-back synchronous instead (tbgpu_checkpoint_delta at the bar's last op, its
    // objects handed over before compact calls back): the shape zig/state_machine_gpu.zig runs.
    bool compact_sync = false;
    // compact's write-back one OP (or chunk of ops) behind instead of one bar: every op starts the capture of its own
    // changes (tbgpu_checkpoint_delta_async) and hands the previous op's to write_back (they crossed
    // PCIe while this op committed); the last op of a bar waits for its own, so every bar's objects
    // reach the forest before compact calls back — each bar's table_mutable holds exactly that bar
    // (the groove's value_count_max, src/state_machine.zig:100-178), and nothing blocks for a bar.
    // The shape zig/state_machine_gpu.zig runs.
    bool compact_per_op = false;
    // With compact_per_op: capture every this many ops (a chunk of the bar) instead of every op; the
    // bar's last ops in chunks halving down to its last op alone, which waits for its own.
    uint32_t compact_every = 1;
    bool chunk_end(uint64_t op) const;
    // One bar behind, except the bar ending at a checkpoint op (a journal of this many slots:
    // vsr.Checkpoint.checkpoint_after, src/vsr.zig:2009-2021), written back synchronously (the
    // in-flight bar first): the shape zig/state_machine_gpu.zig runs with engine_write_back_behind.
    // 0: no checkpoint bars.
    uint32_t checkpoint_journal_slots = 0;
    bool checkpoint_trigger_sync = false;  // the trigger's bar synchronous too (A/B)
    static bool checkpoint_bar(uint64_t op, uint32_t journal_slots, uint32_t bar, bool trigger_too);
    // The replica's message pool (MessagePool.init_capacity, src/message_pool.zig:98-120): buffers
    // registered once, so prefetch stages a prepare body from its message by DMA.
    void register_message_buffer(void* buffer, size_t bytes);
    void unregister_message_buffer(void* buffer);
    uint32_t lsm_batch_multiple = 64;
    // prefetch stages a registered body by DMA (tbgpu_prefetch) — worth it when the replica has work
    // between prefetch and commit (its client-replies stage, src/vsr/replica.zig:3060); off (the
    // default): commit's first kernel reads the body straight from the registered message, which
    // is faster when commit follows prefetch at once (tb_replica_bench: 0.092 vs 0.115 ms per op).
    bool stage_bodies = false;
    // Hands every object changed since the previous write-back to `write_back` (if set) — the bar
    // still in flight, then the rest — then calls back (state_machine.zig:565-582).
    void checkpoint(const Callback& callback);
    // The synchronous write-back (a bar in flight is handed to write_back first).
    const Delta& checkpoint_delta();
    WriteBack write_back;
    // Allocates and registers both bar-sized write-back buffer sets now (the Zig wrapper does it in
    // init): otherwise the first bar's compact does.
    void reserve_write_back();

    // Test-only: the table harness `setup` action (state_machine.zig:1398-1407).
    void test_set_balances(u128 account_id, u128 debits_pending, u128 debits_posted, u128 credits_pending,
                           u128 credits_posted);

    uint64_t prepare_timestamp = 0;
    uint64_t commit_timestamp = 0;

    tbgpu_t* engine() const { return engine_; }

private:
    void check(int status, const char* what) const;
    struct WbSet {  // one set of registered write-back buffers
        uint64_t caps[3] = {0, 0, 0};  // accounts, transfers, posted
        std::vector<uint8_t> accounts, before, transfers, posted;
    };
    void wb_reserve(WbSet& w, const uint64_t caps[3]);
    const Delta& wb_view(const WbSet& w, const tbgpu_delta_counts& c);
    void wb_deliver_inflight();
    tbgpu_t* engine_ = nullptr;
    Delta delta_;
    WbSet wb_[2];          // [0]: synchronous write-backs and even bars, [1]: odd bars
    int wb_bar_ = 0;       // the set the next bar's asynchronous write-back uses
    int wb_inflight_ = -1; // the set of the write-back in flight, or -1
};

}  // namespace tb
