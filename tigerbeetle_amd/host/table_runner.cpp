// table_runner.cpp — the reference's table-driven StateMachine tests, run through the C++ host
// mirror (tb::StateMachine) on the GPU engine.
//
//   tb_table_runner <tests/golden/state_machine_tables.txt> [device]
//
// The fixture holds the 18 check() tables of src/state_machine.zig:1531-2074 verbatim.  Row DSL:
// src/testing/table.zig:8-100 (tokens, `_` defaults, letter labels, `-N` = maxInt - N); action
// schema and harness: src/state_machine.zig:1247-1529 (TestAction, TestCreateAccount,
// TestCreateTransfer, check()).  Prints one line per table; exit status = number of failures.
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "state_machine.hpp"

namespace {

using tb::u128;

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// table.zig:37-47: one leading letter is a label; `-N` on an unsigned field is maxInt - N.
u128 parse_int(const std::string& tok, int bits) {
    size_t i = (!tok.empty() && std::isalpha((unsigned char)tok[0])) ? 1 : 0;
    const u128 maxv = bits == 128 ? ~(u128)0 : (((u128)1 << bits) - 1);
    bool neg = false;
    if (i < tok.size() && tok[i] == '-') {
        neg = true;
        i++;
    }
    if (i >= tok.size()) throw ParseError("empty integer: " + tok);
    u128 v = 0;
    for (; i < tok.size(); i++) {
        if (!std::isdigit((unsigned char)tok[i])) throw ParseError("bad integer: " + tok);
        v = v * 10 + (u128)(tok[i] - '0');
    }
    if (neg) {
        if (v > maxv) throw ParseError("out of range: " + tok);
        return maxv - v;
    }
    if (v > maxv) throw ParseError("out of range: " + tok);
    return v;
}

struct Tokens {
    std::vector<std::string> t;
    size_t i = 0;
    bool more() const { return i < t.size(); }
    const std::string& peek() const { return t[i]; }
    std::string next() {
        if (i >= t.size()) throw ParseError("row too short");
        return t[i++];
    }
};

// A column: bits > 0 integer, bits == 0 flag (token), bits < 0 result enum.
struct Column {
    const char* name;
    int bits;
    const char* flag;
    bool required;
};

const Column kAccountColumns[] = {  // TestCreateAccount (state_machine.zig:1281-1298)
    {"id", 128, nullptr, true},          {"debits_pending", 128, nullptr, false},
    {"debits_posted", 128, nullptr, false}, {"credits_pending", 128, nullptr, false},
    {"credits_posted", 128, nullptr, false}, {"user_data_128", 128, nullptr, false},
    {"user_data_64", 64, nullptr, false}, {"user_data_32", 32, nullptr, false},
    {"reserved", 1, nullptr, false},     {"ledger", 32, nullptr, true},
    {"code", 16, nullptr, true},         {"linked", 0, "LNK", false},
    {"debits_must_not_exceed_credits", 0, "D<C", false},
    {"credits_must_not_exceed_debits", 0, "C<D", false},
    {"flags_padding", 13, nullptr, false}, {"timestamp", 64, nullptr, false},
    {"result", -1, nullptr, true},
};

const Column kTransferColumns[] = {  // TestCreateTransfer (state_machine.zig:1324-1344)
    {"id", 128, nullptr, true},          {"debit_account_id", 128, nullptr, true},
    {"credit_account_id", 128, nullptr, true}, {"amount", 128, nullptr, false},
    {"pending_id", 128, nullptr, false}, {"user_data_128", 128, nullptr, false},
    {"user_data_64", 64, nullptr, false}, {"user_data_32", 32, nullptr, false},
    {"timeout", 32, nullptr, false},     {"ledger", 32, nullptr, true},
    {"code", 16, nullptr, true},         {"linked", 0, "LNK", false},
    {"pending", 0, "PEN", false},        {"post_pending_transfer", 0, "POS", false},
    {"void_pending_transfer", 0, "VOI", false}, {"balancing_debit", 0, "BDR", false},
    {"balancing_credit", 0, "BCR", false}, {"flags_padding", 10, nullptr, false},
    {"timestamp", 64, nullptr, false},   {"result", -2, nullptr, true},
};

uint32_t result_index(const std::vector<std::string>& names, const std::string& tok) {
    for (size_t i = 0; i < names.size(); i++) {
        if (names[i] == tok) return (uint32_t)i;
    }
    throw ParseError("unknown result: " + tok);
}

// table.zig:49-71: `_` selects a field's default, only for fields that have one.
template <size_t N>
std::map<std::string, u128> parse_struct(Tokens& toks, const Column (&cols)[N]) {
    std::map<std::string, u128> row;
    for (const Column& c : cols) {
        if (!c.required && toks.more() && toks.peek() == "_") {
            toks.next();
            row[c.name] = 0;
            continue;
        }
        const std::string tok = toks.next();
        if (c.bits > 0) {
            row[c.name] = parse_int(tok, c.bits);
        } else if (c.bits == 0) {
            if (tok != c.flag) throw ParseError("unknown flag " + tok + " (expected " + c.flag + ")");
            row[c.name] = 1;
        } else {
            row[c.name] = result_index(c.bits == -1 ? tb::create_account_result_names() : tb::create_transfer_result_names(),
                                       tok);
        }
    }
    return row;
}

tb::Account account_event(std::map<std::string, u128>& r) {  // state_machine.zig:1300-1321
    tb::Account a{};
    a.id = r["id"];
    a.debits_pending = r["debits_pending"];
    a.debits_posted = r["debits_posted"];
    a.credits_pending = r["credits_pending"];
    a.credits_posted = r["credits_posted"];
    a.user_data_128 = r["user_data_128"];
    a.user_data_64 = (uint64_t)r["user_data_64"];
    a.user_data_32 = (uint32_t)r["user_data_32"];
    a.reserved = (uint32_t)r["reserved"];
    a.ledger = (uint32_t)r["ledger"];
    a.code = (uint16_t)r["code"];
    a.flags = (uint16_t)((r["linked"] ? tb::AccountFlags::linked : 0) |
                         (r["debits_must_not_exceed_credits"] ? tb::AccountFlags::debits_must_not_exceed_credits : 0) |
                         (r["credits_must_not_exceed_debits"] ? tb::AccountFlags::credits_must_not_exceed_debits : 0) |
                         ((uint16_t)r["flags_padding"] << 3));
    a.timestamp = (uint64_t)r["timestamp"];
    return a;
}

tb::Transfer transfer_event(std::map<std::string, u128>& r) {  // state_machine.zig:1346-1370
    tb::Transfer t{};
    t.id = r["id"];
    t.debit_account_id = r["debit_account_id"];
    t.credit_account_id = r["credit_account_id"];
    t.amount = r["amount"];
    t.pending_id = r["pending_id"];
    t.user_data_128 = r["user_data_128"];
    t.user_data_64 = (uint64_t)r["user_data_64"];
    t.user_data_32 = (uint32_t)r["user_data_32"];
    t.timeout = (uint32_t)r["timeout"];
    t.ledger = (uint32_t)r["ledger"];
    t.code = (uint16_t)r["code"];
    t.flags = (uint16_t)((r["linked"] ? tb::TransferFlags::linked : 0) | (r["pending"] ? tb::TransferFlags::pending : 0) |
                         (r["post_pending_transfer"] ? tb::TransferFlags::post_pending_transfer : 0) |
                         (r["void_pending_transfer"] ? tb::TransferFlags::void_pending_transfer : 0) |
                         (r["balancing_debit"] ? tb::TransferFlags::balancing_debit : 0) |
                         (r["balancing_credit"] ? tb::TransferFlags::balancing_credit : 0) |
                         ((uint16_t)r["flags_padding"] << 6));
    t.timestamp = (uint64_t)r["timestamp"];
    return t;
}

template <typename T>
void append(std::vector<uint8_t>& buf, const T& v) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
    buf.insert(buf.end(), p, p + sizeof(T));
}

std::string describe(const std::vector<uint8_t>& b, bool creates) {
    std::ostringstream os;
    if (creates) {
        for (size_t i = 0; i + 8 <= b.size(); i += 8) {
            uint32_t idx, res;
            memcpy(&idx, &b[i], 4);
            memcpy(&res, &b[i + 4], 4);
            os << "(" << idx << "," << res << ")";
        }
    } else {
        os << b.size() / 128 << " records";
    }
    return os.str();
}

// check() (state_machine.zig:1373-1529) for one table.
std::string run_table(tb::StateMachine& sm, const std::string& text) {
    std::map<u128, tb::Account> accounts;
    std::map<u128, tb::Transfer> transfers;
    std::vector<uint8_t> request, reply;
    int operation = 0;  // 0 = none yet
    uint64_t prepare_timestamp = 0;
    std::vector<uint8_t> output(tb::message_body_size_max);
    uint64_t op_number = 0;

    std::istringstream lines(text);
    std::string line;
    while (std::getline(lines, line)) {
        Tokens toks;
        std::istringstream ls(line);
        for (std::string w; ls >> w;) toks.t.push_back(w);
        if (toks.t.empty()) continue;
        const std::string variant = toks.next();
        if (variant == "setup") {
            u128 v[5];
            for (u128& x : v) x = parse_int(toks.next(), 128);
            sm.test_set_balances(v[0], v[1], v[2], v[3], v[4]);
        } else if (variant == "tick") {
            prepare_timestamp += (uint64_t)parse_int(toks.next(), 64);
        } else if (variant == "account") {
            auto r = parse_struct(toks, kAccountColumns);
            operation = (int)tb::Operation::create_accounts;
            const tb::Account a = account_event(r);
            append(request, a);
            if (r["result"] == 0) accounts[a.id] = a;
            else append(reply, tb::CreateResult{(uint32_t)(request.size() / 128 - 1), (uint32_t)r["result"]});
        } else if (variant == "transfer") {
            auto r = parse_struct(toks, kTransferColumns);
            operation = (int)tb::Operation::create_transfers;
            const tb::Transfer t = transfer_event(r);
            append(request, t);
            if (r["result"] == 0) transfers[t.id] = t;
            else append(reply, tb::CreateResult{(uint32_t)(request.size() / 128 - 1), (uint32_t)r["result"]});
        } else if (variant == "lookup_account") {
            operation = (int)tb::Operation::lookup_accounts;
            const u128 id = parse_int(toks.next(), 128);
            append(request, id);
            if (toks.peek() == "_") {
                toks.next();
            } else {
                tb::Account a = accounts.at(id);
                a.debits_pending = parse_int(toks.next(), 128);
                a.debits_posted = parse_int(toks.next(), 128);
                a.credits_pending = parse_int(toks.next(), 128);
                a.credits_posted = parse_int(toks.next(), 128);
                append(reply, a);
            }
        } else if (variant == "lookup_transfer") {
            operation = (int)tb::Operation::lookup_transfers;
            const u128 id = parse_int(toks.next(), 128);
            append(request, id);
            const std::string kind = toks.next();
            if (kind == "exists") {
                const std::string v = toks.next();
                if (v == "true" || v == "T" || v == "1") append(reply, transfers.at(id));
            } else if (kind == "amount") {
                tb::Transfer t = transfers.at(id);
                t.amount = parse_int(toks.next(), 128);
                append(reply, t);
            } else {
                throw ParseError("unknown lookup_transfer variant " + kind);
            }
        } else if (variant == "commit") {
            const std::string name = toks.next();
            const tb::Operation op = name == "create_accounts"    ? tb::Operation::create_accounts
                                     : name == "create_transfers" ? tb::Operation::create_transfers
                                     : name == "lookup_accounts"  ? tb::Operation::lookup_accounts
                                     : name == "lookup_transfers" ? tb::Operation::lookup_transfers
                                                                  : throw ParseError("unknown operation " + name);
            if (operation != 0 && operation != (int)op) throw ParseError("commit of a different operation");
            prepare_timestamp += 1;
            sm.prepare_timestamp = prepare_timestamp;
            sm.prepare(op, request.data(), request.size());  // state_machine.zig:336-343
            prepare_timestamp = sm.prepare_timestamp;
            sm.prefetch([](tb::StateMachine&) {}, ++op_number, op, request.data(), request.size());
            size_t n = sm.commit(0, op_number, prepare_timestamp, op, request.data(), request.size(), output.data());
            std::vector<uint8_t> actual(output.begin(), output.begin() + n);
            const bool creates = op == tb::Operation::create_accounts || op == tb::Operation::create_transfers;
            if (!creates) {  // :1500-1506 lookups zero every returned timestamp
                for (size_t off = 0; off + 128 <= actual.size(); off += 128) memset(&actual[off + 120], 0, 8);
            }
            if (actual != reply) {
                return "reply mismatch for " + name + ": expected " + describe(reply, creates) + " got " +
                       describe(actual, creates);
            }
            request.clear();
            reply.clear();
            operation = 0;
        } else {
            throw ParseError("unknown row variant " + variant);
        }
        if (toks.more() && toks.peek() != "//") throw ParseError("trailing token " + toks.peek());
    }
    return "";
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <state_machine_tables.txt> [device]\n", argv[0]);
        return 2;
    }
    std::ifstream in(argv[1]);
    if (!in) {
        fprintf(stderr, "cannot open %s\n", argv[1]);
        return 2;
    }
    tb::Options o;
    o.accounts_max = 4096;
    o.transfers_max = 1 << 14;
    o.pass_events_max = 8192 * 4;
    o.pass_batches_max = 64;
    o.device = argc > 2 ? atoi(argv[2]) : 0;
    std::unique_ptr<tb::StateMachine> owner;
    try {
        owner.reset(new tb::StateMachine(o));  // StateMachine.init: the only fallible call
    } catch (const std::exception& e) {
        fprintf(stderr, "init failed: %s\n", e.what());
        return 255;
    }
    tb::StateMachine& sm = *owner;

    // Fixture: `@table <name>` ... `@end` blocks (tests/golden/extract_tables.py).
    int failures = 0, tables = 0;
    std::string line, name, body;
    bool inside = false;
    while (std::getline(in, line)) {
        if (line.rfind("@table ", 0) == 0) {
            name = line.substr(7);
            body.clear();
            inside = true;
        } else if (line == "@end" && inside) {
            inside = false;
            tables++;
            std::string err;
            try {
                sm.reset();
                err = run_table(sm, body);
            } catch (const tb::Panic& e) {
                err = std::string("panic: ") + e.what();
            } catch (const std::exception& e) {
                err = std::string("error: ") + e.what();
            }
            if (err.empty()) {
                printf("ok   %s\n", name.c_str());
            } else {
                printf("FAIL %s: %s\n", name.c_str(), err.c_str());
                failures++;
            }
        } else if (inside) {
            body += line + "\n";
        }
    }
    printf("%d tables, %d failed\n", tables, failures);
    return failures;
}
