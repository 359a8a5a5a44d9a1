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
    for (std::vector<uint8_t>* b : {&wb_accounts_, &wb_before_, &wb_transfers_, &wb_posted_}) {
        if (!b->empty()) tbgpu_unregister_host(engine_, b->data());
    }
    tbgpu_deinit(engine_);
}

void StateMachine::reset() {
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

void StateMachine::compact(const Callback& callback, uint64_t op) {
    // The HBM tables need no compaction; the durable copy gets the bar's changes at its last op.
    if (write_back && lsm_batch_multiple && (op + 1) % lsm_batch_multiple == 0) write_back(checkpoint_delta());
    callback(*this);
}

// The write-back buffers are the state machine's own, allocated and registered once (grown when a
// delta needs more room: static allocation in the steady state), so the delta lands by DMA.
static void grow_registered(tbgpu_t* engine, std::vector<uint8_t>& buf, size_t bytes) {
    if (buf.size() >= bytes) return;
    if (!buf.empty()) tbgpu_unregister_host(engine, buf.data());
    std::vector<uint8_t>(bytes).swap(buf);
    if (tbgpu_register_host(engine, buf.data(), buf.size()) != TBGPU_STATUS_OK) {
        throw DeviceError(std::string("register write-back buffer: ") + tbgpu_last_error());
    }
}

const Delta& StateMachine::checkpoint_delta() {
    tbgpu_delta_counts counts{wb_caps_[0], wb_caps_[1], wb_caps_[2], 0};
    for (;;) {
        wb_caps_[0] = std::max<uint64_t>(wb_caps_[0], counts.accounts);
        wb_caps_[1] = std::max<uint64_t>(wb_caps_[1], counts.transfers);
        wb_caps_[2] = std::max<uint64_t>(wb_caps_[2], counts.posted);
        grow_registered(engine_, wb_accounts_, wb_caps_[0] * 128);
        grow_registered(engine_, wb_before_, wb_caps_[0] * 64);
        grow_registered(engine_, wb_transfers_, wb_caps_[1] * 128);
        grow_registered(engine_, wb_posted_, wb_caps_[2] * 16);
        const int st = tbgpu_checkpoint_delta(engine_, wb_accounts_.data(), wb_before_.data(), wb_caps_[0],
                                              wb_transfers_.data(), wb_caps_[1], (uint64_t*)wb_posted_.data(),
                                              wb_caps_[2], &counts);
        if (st == TBGPU_STATUS_INVALID &&
            (counts.accounts > wb_caps_[0] || counts.transfers > wb_caps_[1] || counts.posted > wb_caps_[2])) {
            continue;  // room for everything, then retry (nothing advanced)
        }
        check(st, "checkpoint_delta");
        delta_.accounts = wb_accounts_.data();
        delta_.accounts_before = wb_before_.data();
        delta_.account_count = counts.accounts;
        delta_.transfers = wb_transfers_.data();
        delta_.transfer_count = counts.transfers;
        delta_.posted = (const uint64_t*)wb_posted_.data();
        delta_.posted_count = counts.posted;
        delta_.created_after = counts.created_after;
        return delta_;
    }
}

void StateMachine::checkpoint(const Callback& callback) {
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
