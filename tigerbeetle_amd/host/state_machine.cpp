// state_machine.cpp — tb::StateMachine over the C ABI (include/tbgpu.h).  See state_machine.hpp.
#include "state_machine.hpp"

#include <algorithm>
#include <cstring>

namespace tb {

const std::vector<std::string>& create_account_result_names() {
    static const std::vector<std::string> names = {
        "ok", "linked_event_failed", "linked_event_chain_open", "timestamp_must_be_zero", "reserved_field",
        "reserved_flag", "id_must_not_be_zero", "id_must_not_be_int_max", "flags_are_mutually_exclusive",
        "debits_pending_must_be_zero", "debits_posted_must_be_zero", "credits_pending_must_be_zero",
        "credits_posted_must_be_zero", "ledger_must_not_be_zero", "code_must_not_be_zero",
        "exists_with_different_flags", "exists_with_different_user_data_128", "exists_with_different_user_data_64",
        "exists_with_different_user_data_32", "exists_with_different_ledger", "exists_with_different_code", "exists",
    };
    return names;
}

const std::vector<std::string>& create_transfer_result_names() {
    static const std::vector<std::string> names = {
        "ok", "linked_event_failed", "linked_event_chain_open", "timestamp_must_be_zero", "reserved_flag",
        "id_must_not_be_zero", "id_must_not_be_int_max", "flags_are_mutually_exclusive",
        "debit_account_id_must_not_be_zero", "debit_account_id_must_not_be_int_max",
        "credit_account_id_must_not_be_zero", "credit_account_id_must_not_be_int_max", "accounts_must_be_different",
        "pending_id_must_be_zero", "pending_id_must_not_be_zero", "pending_id_must_not_be_int_max",
        "pending_id_must_be_different", "timeout_reserved_for_pending_transfer", "amount_must_not_be_zero",
        "ledger_must_not_be_zero", "code_must_not_be_zero", "debit_account_not_found", "credit_account_not_found",
        "accounts_must_have_the_same_ledger", "transfer_must_have_the_same_ledger_as_accounts",
        "pending_transfer_not_found", "pending_transfer_not_pending", "pending_transfer_has_different_debit_account_id",
        "pending_transfer_has_different_credit_account_id", "pending_transfer_has_different_ledger",
        "pending_transfer_has_different_code", "exceeds_pending_transfer_amount",
        "pending_transfer_has_different_amount", "pending_transfer_already_posted", "pending_transfer_already_voided",
        "pending_transfer_expired", "exists_with_different_flags", "exists_with_different_debit_account_id",
        "exists_with_different_credit_account_id", "exists_with_different_amount", "exists_with_different_pending_id",
        "exists_with_different_user_data_128", "exists_with_different_user_data_64",
        "exists_with_different_user_data_32", "exists_with_different_timeout", "exists_with_different_code", "exists",
        "overflows_debits_pending", "overflows_credits_pending", "overflows_debits_posted", "overflows_credits_posted",
        "overflows_debits", "overflows_credits", "overflows_timeout", "exceeds_credits", "exceeds_debits",
    };
    return names;
}

void StateMachine::check(int status, const char* what) const {
    if (status == TBGPU_STATUS_OK) return;
    const std::string msg = std::string(what) + ": " + tbgpu_last_error();
    if (status == TBGPU_STATUS_PANIC) throw Panic(msg);
    if (status == TBGPU_STATUS_DEVICE) throw DeviceError(msg);
    throw std::invalid_argument(msg);
}

StateMachine::StateMachine(const Options& o) {
    tbgpu_config cfg{};
    cfg.accounts_max = o.accounts_max;
    cfg.transfers_max = o.transfers_max;
    cfg.pass_events_max = o.pass_events_max;
    cfg.pass_batches_max = o.pass_batches_max;
    cfg.device = o.device;
    cfg.flags = o.profile ? TBGPU_CONFIG_PROFILE : 0;
    if (o.devices.size() > TBGPU_DEVICES_MAX) throw std::invalid_argument("tbgpu_init: too many devices");
    cfg.device_count = (uint32_t)o.devices.size();
    for (size_t d = 0; d < o.devices.size(); d++) cfg.devices[d] = o.devices[d];
    const int st = tbgpu_init(&cfg, &engine_);
    if (st != TBGPU_STATUS_OK) {
        // init is the reference's only fallible call (`!StateMachine`).
        throw DeviceError(std::string("tbgpu_init: ") + tbgpu_last_error());
    }
}

StateMachine::~StateMachine() {
    if (wb_inflight_ >= 0) {
        tbgpu_delta_counts c;
        (void)tbgpu_checkpoint_delta_wait(engine_, &c);  // its buffers go away with this object
    }
    for (WbSet& w : wb_) {
        for (std::vector<uint8_t>* b : {&w.accounts, &w.before, &w.transfers, &w.posted}) {
            if (!b->empty()) tbgpu_unregister_host(engine_, b->data());
        }
    }
    tbgpu_deinit(engine_);
}

void StateMachine::reset() {
    wb_inflight_ = -1;  // the engine drops a write-back in flight with its state
    check(tbgpu_reset(engine_), "reset");
    prepare_timestamp = 0;
    commit_timestamp = 0;
}

void StateMachine::open(const Callback& callback) { callback(*this); }

void StateMachine::prepare(Operation operation, const void* input, size_t input_len) {
    (void)input;
    // state_machine.zig:336-343: creates advance prepare_timestamp by the event count.
    if (operation == Operation::create_accounts || operation == Operation::create_transfers) {
        prepare_timestamp += input_len / 128;
    }
}

void StateMachine::prefetch(const Callback& callback, uint64_t op, Operation operation, const void* input,
                            size_t input_len) {
    if (op == 0) throw Panic("prefetch: op == 0");
    // Every object is HBM-resident; the body starts crossing PCIe now (tbgpu_prefetch: a DMA from a
    // registered message) and the prefetch completes at once (the reference allows the callback to
    // fire inside the call, src/lsm/groove.zig:723-742).
    if (stage_bodies) {
        check(tbgpu_prefetch(engine_, static_cast<uint8_t>(operation), input, static_cast<uint32_t>(input_len)),
              "prefetch");
    }
    callback(*this);
}

void StateMachine::register_message_buffer(void* buffer, size_t bytes) {
    check(tbgpu_register_host(engine_, buffer, bytes), "register_message_buffer");
}

void StateMachine::unregister_message_buffer(void* buffer) {
    check(tbgpu_unregister_host(engine_, buffer), "unregister_message_buffer");
}

size_t StateMachine::commit(u128 client, uint64_t op, uint64_t timestamp, Operation operation, const void* input,
                            size_t input_len, void* output) {
    (void)client;
    if (op == 0) throw Panic("commit: op == 0");  // state_machine.zig:518
    if (input_len > message_body_size_max) throw std::invalid_argument("commit: body larger than a message");
    uint32_t out_len = 0;
    check(tbgpu_commit(engine_, static_cast<uint8_t>(operation), timestamp, input, static_cast<uint32_t>(input_len),
                       output, static_cast<uint32_t>(message_body_size_max), &out_len),
          "commit");
    commit_timestamp = tbgpu_commit_timestamp(engine_);
    return out_len;
}

std::vector<size_t> StateMachine::commit_many(Operation operation, const std::vector<uint64_t>& timestamps,
                                              const std::vector<const void*>& inputs,
                                              const std::vector<size_t>& input_lens,
                                              const std::vector<void*>& outputs) {
    const size_t n = timestamps.size();
    if (inputs.size() != n || input_lens.size() != n || outputs.size() != n) {
        throw std::invalid_argument("commit_many: argument lengths differ");
    }
    std::vector<uint32_t> lens(n), out_lens(n);
    for (size_t k = 0; k < n; k++) lens[k] = static_cast<uint32_t>(input_lens[k]);
    check(tbgpu_commit_many(engine_, static_cast<uint8_t>(operation), static_cast<uint32_t>(n), timestamps.data(),
                            inputs.data(), lens.data(), outputs.data(), out_lens.data()),
          "commit_many");
    commit_timestamp = tbgpu_commit_timestamp(engine_);
    return std::vector<size_t>(out_lens.begin(), out_lens.end());
}

bool StateMachine::checkpoint_bar(uint64_t op, uint32_t journal_slots, uint32_t bar, bool trigger_too) {
    if (journal_slots == 0 || journal_slots <= bar + 1) return false;
    const uint64_t first = journal_slots - bar - 1, every = journal_slots - bar;  // checkpoint_after
    if (op < first) return false;
    const uint64_t r = (op - first) % every;
    // A checkpoint op (its bar is flushed by the trigger bar's compaction); optionally the trigger too.
    return r == 0 || (trigger_too && r == bar);
}

// In chunks of compact_every ops; the bar's last compact_every ops in chunks halving down to its
// last op alone (e.g. of 4: 2, 1, 1).  The bar's last chunk is waited for at once (its objects
// land before compact returns) and each chunk's copy-out overlaps the next chunk's commits, so a
// chunk shorter than the one before it waits for the difference: halving keeps both waits to about
// one op's objects.
bool StateMachine::chunk_end(uint64_t op) const {
    const uint64_t bar = lsm_batch_multiple, r = op % bar, rem = bar - 1 - r;
    const uint64_t every = std::max<uint32_t>(1, compact_every);
    if (rem < every) return rem == 0 || (rem & (rem - 1)) == 0;
    return (r + 1) % every == 0;
}

void StateMachine::compact(const Callback& callback, uint64_t op) {
    // The HBM tables need no compaction; the durable copy gets each bar's changes, one bar behind.
    const bool bar_end = lsm_batch_multiple && (op + 1) % lsm_batch_multiple == 0;
    if (write_back && lsm_batch_multiple && compact_per_op && !chunk_end(op)) {
        // inside a chunk: nothing to do
    } else if (write_back && lsm_batch_multiple && compact_per_op) {
        wb_deliver_inflight();  // the previous chunk's objects: landed while this one committed
        reserve_write_back();
        WbSet& w = wb_[wb_bar_];
        check(tbgpu_checkpoint_delta_async(engine_, w.accounts.data(), w.before.data(), w.caps[0], w.transfers.data(),
                                           w.caps[1], (uint64_t*)w.posted.data(), w.caps[2]),
              "checkpoint_delta_async");
        wb_inflight_ = wb_bar_;
        wb_bar_ ^= 1;
        if (bar_end) wb_deliver_inflight();  // the bar ends with its own objects
    } else if (write_back && lsm_batch_multiple && (op + 1) % lsm_batch_multiple == 0 &&
               (compact_sync || checkpoint_bar(op, checkpoint_journal_slots, lsm_batch_multiple, checkpoint_trigger_sync))) {
        // The bar's objects before compact returns (the in-flight bar first, in checkpoint_delta):
        // the Zig wrapper's synchronous shape, and its checkpoint bars with engine_write_back_behind.
        write_back(checkpoint_delta());
    } else if (write_back && lsm_batch_multiple && (op + 1) % lsm_batch_multiple == 0) {
        wb_deliver_inflight();  // the previous bar's objects: landed while this bar committed
        reserve_write_back();
        WbSet& w = wb_[wb_bar_];
        check(tbgpu_checkpoint_delta_async(engine_, w.accounts.data(), w.before.data(), w.caps[0], w.transfers.data(),
                                           w.caps[1], (uint64_t*)w.posted.data(), w.caps[2]),
              "checkpoint_delta_async");
        wb_inflight_ = wb_bar_;
        wb_bar_ ^= 1;
    }
    callback(*this);
}

// The write-back buffers are the state machine's own, registered once (grown only when a delta
// needs more room), so the objects land by DMA.
static void grow_registered(tbgpu_t* engine, std::vector<uint8_t>& buf, size_t bytes) {
    if (buf.size() >= bytes) return;
    if (!buf.empty()) tbgpu_unregister_host(engine, buf.data());
    std::vector<uint8_t>(bytes).swap(buf);
    if (tbgpu_register_host(engine, buf.data(), buf.size()) != TBGPU_STATUS_OK) {
        throw DeviceError(std::string("register write-back buffer: ") + tbgpu_last_error());
    }
}

void StateMachine::reserve_write_back() {
    // Room for a whole bar (what a bar of prepares can change at most, tbgpu.h), registered once.
    const uint64_t ev = (uint64_t)lsm_batch_multiple * TBGPU_BATCH_EVENTS_MAX;
    const uint64_t caps[3] = {2 * ev, ev, ev};
    for (WbSet& w : wb_) wb_reserve(w, caps);
}

void StateMachine::wb_reserve(WbSet& w, const uint64_t caps[3]) {
    for (int k = 0; k < 3; k++) w.caps[k] = std::max(w.caps[k], std::max<uint64_t>(caps[k], 1));
    grow_registered(engine_, w.accounts, w.caps[0] * 128);
    grow_registered(engine_, w.before, w.caps[0] * 64);
    grow_registered(engine_, w.transfers, w.caps[1] * 128);
    grow_registered(engine_, w.posted, w.caps[2] * 16);
}

const Delta& StateMachine::wb_view(const WbSet& w, const tbgpu_delta_counts& c) {
    delta_.accounts = w.accounts.data();
    delta_.accounts_before = w.before.data();
    delta_.account_count = c.accounts;
    delta_.transfers = w.transfers.data();
    delta_.transfer_count = c.transfers;
    delta_.posted = (const uint64_t*)w.posted.data();
    delta_.posted_count = c.posted;
    delta_.created_after = c.created_after;
    return delta_;
}

void StateMachine::wb_deliver_inflight() {
    if (wb_inflight_ < 0) return;
    tbgpu_delta_counts c{};
    const int set = wb_inflight_;
    wb_inflight_ = -1;
    check(tbgpu_checkpoint_delta_wait(engine_, &c), "checkpoint_delta_wait");
    const Delta& d = wb_view(wb_[set], c);
    if (write_back) write_back(d);
}

const Delta& StateMachine::checkpoint_delta() {
    wb_deliver_inflight();
    WbSet& w = wb_[0];
    if (!w.caps[0]) {
        const uint64_t first[3] = {1024, 1024, 1024};
        wb_reserve(w, first);
    }
    tbgpu_delta_counts counts{};
    for (;;) {
        const int st = tbgpu_checkpoint_delta(engine_, w.accounts.data(), w.before.data(), w.caps[0], w.transfers.data(),
                                              w.caps[1], (uint64_t*)w.posted.data(), w.caps[2], &counts);
        if (st == TBGPU_STATUS_INVALID &&
            (counts.accounts > w.caps[0] || counts.transfers > w.caps[1] || counts.posted > w.caps[2])) {
            const uint64_t need[3] = {counts.accounts, counts.transfers, counts.posted};
            wb_reserve(w, need);  // room for everything, then retry (nothing advanced)
            continue;
        }
        check(st, "checkpoint_delta");
        return wb_view(w, counts);
    }
}

void StateMachine::checkpoint(const Callback& callback) {
    wb_deliver_inflight();
    const Delta& d = checkpoint_delta();
    if (write_back) write_back(d);
    callback(*this);
}

void StateMachine::test_set_balances(u128 id, u128 dp, u128 dpost, u128 cp, u128 cpost) {
    const uint64_t b[8] = {(uint64_t)dp, (uint64_t)(dp >> 64), (uint64_t)dpost, (uint64_t)(dpost >> 64),
                           (uint64_t)cp, (uint64_t)(cp >> 64), (uint64_t)cpost, (uint64_t)(cpost >> 64)};
    check(tbgpu_test_set_balances(engine_, (uint64_t)id, (uint64_t)(id >> 64), b), "test_set_balances");
}

}  // namespace tb
