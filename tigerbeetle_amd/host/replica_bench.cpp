// tb_replica_bench — the replica's own call path through the C++ mirror (tb::StateMachine): one op
// at a time, prepare -> prefetch -> commit -> compact, serially, as the replica's commit stage
// machine drives the state machine (src/vsr/replica.zig:3045-3102; commit_op_prefetch :3324-3354,
// commit_op :3581-3665).  Prepare bodies sit in a message pool registered once (one 1-MiB message
// per prepare, the body after its 128-B header: src/message_pool.zig:98-120), so commit's first
// kernel reads each body straight from its message (or, with --stage, prefetch starts its DMA and
// commit waits for it).  With --write-back, compact hands each bar's changes to a sink (the durable
// replica's forest; here the sink touches nothing).
//
// Usage: tb_replica_bench [--accounts N] [--prepares N] [--warmup N] [--write-back | --write-back-sync |
//                         --write-back-per-op] [--stage]
//                         [--device D]
// (--write-back-sync: compact writes each bar back synchronously, as zig/state_machine_gpu.zig did in
// round 4; --write-back-per-op: one op behind, each bar complete at its last op — the Zig wrapper's
// shape since round 5.)
// (--stage: prefetch stages the body by DMA; default: commit reads it straight from the message.)
// Prints one JSON line: per-op latency (host clock around prefetch+commit+compact) and throughput.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tbgpu.h"
#include "../../include/tbgpu_bench.h"
#include "state_machine.hpp"

namespace {

void need(int st, const char* what) {
    if (st != TBGPU_STATUS_OK) {
        fprintf(stderr, "%s: %s\n", what, tbgpu_last_error());
        exit(1);
    }
}

// The reference's percentile pick (src/benchmark.zig:454-471): latencies[len * p / 100 -| 1].
double pick(const std::vector<double>& sorted, int p) {
    if (sorted.empty()) return 0;
    size_t i = sorted.size() * (size_t)p / 100;
    return sorted[i ? i - 1 : 0];
}

}  // namespace

int main(int argc, char** argv) {
    uint64_t accounts = 1000000, prepares = 2000, warmup = 64;
    int device = 0;
    bool write_back = false, stage = false, sync_wb = false, per_op_wb = false, trigger_sync = false;
    uint32_t every = 1, journal_slots = 0;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? strtoull(argv[++i], nullptr, 10) : 0ULL; };
        if (a == "--accounts") accounts = next();
        else if (a == "--prepares") prepares = next();
        else if (a == "--warmup") warmup = next();
        else if (a == "--device") device = (int)next();
        else if (a == "--write-back") write_back = true;
        else if (a == "--write-back-sync") write_back = sync_wb = true;
        else if (a == "--write-back-per-op") write_back = per_op_wb = true;
        else if (a == "--write-back-every") { write_back = per_op_wb = true; every = (uint32_t)next(); }
        else if (a == "--checkpoint-journal-slots") { write_back = true; journal_slots = (uint32_t)next(); }
        else if (a == "--checkpoint-trigger-sync") trigger_sync = true;
        else if (a == "--no-stage") stage = false;
        else if (a == "--stage") stage = true;
    }
    const uint32_t batch = 8190;
    const uint64_t total_ops = warmup + prepares;

    tb::Options o;
    o.accounts_max = accounts;
    o.transfers_max = total_ops * batch + 1024;
    o.pass_events_max = batch * 64;
    o.pass_batches_max = 64;
    o.device = device;
    tb::StateMachine sm(o);
    sm.stage_bodies = stage;
    sm.compact_sync = sync_wb;
    sm.compact_per_op = per_op_wb;
    sm.compact_every = every;
    sm.checkpoint_journal_slots = journal_slots;
    sm.checkpoint_trigger_sync = trigger_sync;
    tbgpu_t* E = sm.engine();

    // Workload: the engine's generator (C2 shapes, tbgpu_bench.h), copied to host memory.
    const uint64_t gen_n = std::max<uint64_t>(accounts, (uint64_t)batch * 64);
    void* dev = nullptr;
    need(tbgpu_device_alloc(E, gen_n * 128, &dev), "alloc");
    tbgpu_workload w{};
    w.seed = 42;
    w.account_count = accounts;
    std::vector<uint8_t> acct(accounts * 128);
    need(tbgpu_bench_generate_accounts(E, dev, 0, accounts, &w), "generate accounts");
    need(tbgpu_copy_to_host(E, acct.data(), dev, accounts * 128), "copy");
    uint64_t ts = 1000000000;
    for (uint64_t a0 = 0; a0 < accounts; a0 += (uint64_t)batch * 512) {
        std::vector<uint64_t> stamps;
        std::vector<const void*> ins;
        std::vector<size_t> lens;
        std::vector<std::vector<uint8_t>> outs;
        std::vector<void*> outp;
        for (uint64_t k = a0; k < std::min<uint64_t>(accounts, a0 + (uint64_t)batch * 512); k += batch) {
            const uint64_t L = std::min<uint64_t>(batch, accounts - k);
            ts += 1 + L;
            stamps.push_back(ts);
            ins.push_back(acct.data() + k * 128);
            lens.push_back(L * 128);
            outs.emplace_back(L * 8);
        }
        for (auto& v : outs) outp.push_back(v.data());
        for (size_t r : sm.commit_many(tb::Operation::create_accounts, stamps, ins, lens, outp)) {
            if (r) {
                fprintf(stderr, "account creation failed\n");
                return 1;
            }
        }
    }
    sm.prepare_timestamp = ts;

    // The message pool: one message per op, the body after a 128-B header.
    const size_t message = 1u << 20;
    std::vector<uint8_t> pool(total_ops * message);
    w.kind = 0;
    for (uint64_t k0 = 0; k0 < total_ops; k0 += 64) {
        const uint64_t m = std::min<uint64_t>(64, total_ops - k0);
        need(tbgpu_bench_generate_transfers(E, dev, k0 * batch, m * batch, &w), "generate transfers");
        std::vector<uint8_t> tmp(m * batch * 128);
        need(tbgpu_copy_to_host(E, tmp.data(), dev, tmp.size()), "copy");
        for (uint64_t k = 0; k < m; k++) memcpy(&pool[(k0 + k) * message + 128], &tmp[k * batch * 128], batch * 128);
    }
    need(tbgpu_device_free(E, dev), "free");
    sm.register_message_buffer(pool.data(), pool.size());

    uint64_t wb_objects = 0;
    if (write_back) {
        sm.write_back = [&](const tb::Delta& d) { wb_objects += d.account_count + d.transfer_count + d.posted_count; };
        sm.reserve_write_back();      // both bar-sized buffer sets, registered before the timed ops
        (void)sm.checkpoint_delta();  // the accounts' creation: written back before the timed ops
    }
    std::vector<uint8_t> reply(tb::message_body_size_max);
    std::vector<double> lat;
    lat.reserve(prepares);
    uint64_t failed = 0;
    double compact_ms = 0, compact_max = 0;  // inside compact (the write-back's host side)
    const auto run0 = std::chrono::steady_clock::now();
    auto t_timed = run0;
    for (uint64_t op = 1; op <= total_ops; op++) {
        if (op == warmup + 1) t_timed = std::chrono::steady_clock::now();
        const uint8_t* body = &pool[(op - 1) * message + 128];
        const size_t len = (size_t)batch * 128;
        const auto t0 = std::chrono::steady_clock::now();
        sm.prepare(tb::Operation::create_transfers, body, len);
        sm.prefetch([](tb::StateMachine&) {}, op, tb::Operation::create_transfers, body, len);
        const size_t n = sm.commit(0, op, sm.prepare_timestamp, tb::Operation::create_transfers, body, len, reply.data());
        const auto tc = std::chrono::steady_clock::now();
        sm.compact([](tb::StateMachine&) {}, op);
        const auto t1 = std::chrono::steady_clock::now();
        if (op > warmup) {
            const double c = std::chrono::duration<double, std::milli>(t1 - tc).count();
            compact_ms += c;
            compact_max = std::max(compact_max, c);
        }
        failed += n / 8;
        sm.prepare_timestamp += 1;
        if (op > warmup) lat.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    const double total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_timed).count();
    if (write_back) sm.checkpoint([](tb::StateMachine&) {});  // the last bar's objects (untimed)
    sm.unregister_message_buffer(pool.data());
    std::vector<double> sorted(lat);
    std::sort(sorted.begin(), sorted.end());
    printf("{\"call_path\": \"prepare -> prefetch -> commit -> compact per op (tb::StateMachine, C++)\", "
           "\"ops\": %llu, \"events_per_op\": %u, \"write_back\": %s, \"write_back_sync\": %s, \"write_back_per_op\": %s, \"write_back_every_ops\": %u, \"checkpoint_journal_slots\": %u, \"prefetch_stages_body\": %s, \"transfers_per_s\": %.1f, "
           "\"ms_per_op\": %.4f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"p100_ms\": %.4f, \"failed_events\": %llu, "
           "\"written_back_objects\": %llu, \"compact_ms_per_op\": %.4f, \"compact_ms_max\": %.4f}\n",
           (unsigned long long)prepares, batch, write_back ? "true" : "false", sync_wb ? "true" : "false",
           per_op_wb ? "true" : "false", per_op_wb ? every : 0u, journal_slots, stage ? "true" : "false",
           prepares * batch / (total_ms / 1e3),
           total_ms / prepares, pick(sorted, 50), pick(sorted, 99), pick(sorted, 100), (unsigned long long)failed,
           (unsigned long long)wb_objects, compact_ms / prepares, compact_max);
    return failed ? 1 : 0;
}
