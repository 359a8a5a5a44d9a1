// node.h — the multi-device engine behind include/tbgpu.h (tbgpu_config.device_count > 1).
//
// The reference commits on one thread of one replica (src/vsr/replica.zig:3654, serial stages
// :3045-3102), and SURVEY.md §8e asks for one 8-GPU node with accounts hash-partitioned and
// cross-shard legs exchanged over xGMI.  Here the replica's single caller keeps its single call:
// tbgpu_commit / _many / _pipelined on a node engine route every pass across N shards (one per
// device listed in the config) inside the library — the exchange is kernels reading their peers'
// HBM (k_node.h), so no host staging, no collective library and no Python sit on the data path.
//
// Partition: an account — record and balances — on owner(id) only, a transfer on
// home(id).  create_accounts prepares are committed in order by the sequencer (below) with the
// existing records they name loaded from their owners, and each new account goes to its owner; a home
// imports the hot records of the foreign accounts a routed pass names from their owners before it
// validates and keeps them for later passes, until an account is inserted on a shard or the room
// fills (k_node.h tb_node_import, tb_node_import_flush).  Per-shard account memory is the owned 1/N
// of the ledger plus the import room (the ledger's accounts, or a routed sub-pass's two per event
// when fewer).  A create_transfers call is cut into passes: pass p takes up to
// N blocks of `chunk` prepares (block d -> source shard d, in order, so the pass's global order is
// block-major = prepare order).  Per pass, on every device:
//   copy stream   H2D of the source block's bodies (registered host memory: DMA)
//   route stream  route plan (classify / offsets / scatter) + its counts to pinned host memory
//   engine stream gather from the sources -> routed commit with owner legs -> apply the legs it
//                 owns from every home -> its sources' replies -> reply arena (pinned, mapped)
// The host reads pass p's plan counts (the one round trip per pass) while pass p-1 commits, and
// pass p+1's bodies cross PCIe meanwhile.  Cross-device order is hipStreamWaitEvent on events of
// the peers' streams.
//
// A pass is CLEAN when no event is linked / post / void / balancing, no account it touches carries
// a limit flag, and (sum of the shards' bounds) + S < 2^128 (host-tracked, conservative).  A
// dirty pass is SPLIT (node_split_pass, k_node.h): every source classifies its events on the device,
// the independent ones are routed and committed by their homes as in a clean pass, and the
// dependent subsequence is committed in order by the sequencer — an engine on the first device,
// allocated at init, that the pass loads with exactly the transfers and accounts those events read
// (peer reads from their homes and owners: the reference's prefetch -> commit split,
// src/state_machine.zig:345-506) — whose changes are written back to homes and owners by kernels
// on those devices.  No host code walks the events.  Without the overflow certificate every event of
// the pass is sequenced.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>

#include "k_node.h"

struct NodeDev {
    tbgpu* E = nullptr;
    int device = 0;
    hipStream_t rs = nullptr;   // route stream (plans); E->copy_stream: H2D; E->stream: the pass
    // Source side, by pass parity.
    u8* stage[2] = {};
    const u8* ev[2] = {};        // the block's events this pass parity: stage[], or the caller's HBM
    u8* send[2] = {};
    u32* slot[2] = {};
    u8* home[2] = {};
    u64* words[2] = {};          // zero between plans (tb_route_publish clears them)
    u64* h_words[2] = {};        // pinned, device-mapped: the plan words back on the host
    u64* d_words_host[2] = {};   // h_words' device address
    // Completion words (pinned, device-mapped) the host spins on: [par] a plan's words published,
    // [2 + tri] a one-workgroup reply arena written.  Each use gets a new non-zero sequence number.
    u32* h_flags = nullptr;
    u32* d_flags = nullptr;
    u32 flag_seq = 0;
    u32 plan_seq[2] = {};
    u32 reply_seq[3] = {};       // 0: the arena of that slot is waited for by its event
    u64* meta[2] = {};           // device: the block's offsets then timestamps
    u64* h_meta[2] = {};         // pinned mirror
    u32* block_counts = nullptr;
    u32* results = nullptr;      // the block's sparse replies (tb_node_replies)
    u32* reply_bytes = nullptr;
    // Home / owner side.
    u8* recv = nullptr;
    u8* codes = nullptr;
    u64* legs = nullptr;
    u64* leg_counts = nullptr;
    u64* hmeta_dev[3] = {};      // routed commit pseudo-prepares (offsets, timestamps), by pass mod 3
    u64* hmeta_host[3] = {};
    // Reply arenas by pass mod 3 (pinned, device-mapped; tb_reply_out's layout).
    u8* h_arena[3] = {};
    u8* d_arena[3] = {};
    hipEvent_t ev_start[3] = {}, ev_done[3] = {}, ev_planned[2] = {}, ev_copied = nullptr;
    hipEvent_t ev_gathered = nullptr, ev_committed = nullptr, ev_applied = nullptr, ev_replied = nullptr;
    // Dirty passes (k_node.h): the block's classification and this device's key sets.
    u8* dep1 = nullptr;
    u8* dep[2] = {};             // by pass parity: the sequencer reads pass p's while pass p + 1 classifies
    u64* dkeys = nullptr;        // [2 pe_src][2]
    u64* dbal = nullptr;         // [2 pe_src][2]
    u64* dcounts = nullptr;      // [NODE_DC_WORDS] (k_node.h NodeDepArgs)
    u64* h_dcounts = nullptr;    // pinned
    u64* keyset = nullptr;
    u64* markset = nullptr;
    u64 set_mask = 0;
    u64* wb_count = nullptr;     // sequencer write-back: records appended here
    hipEvent_t ev_cls = nullptr, ev_marked = nullptr;
    hipEvent_t ev_pre = nullptr;  // split pass: this stream before the pass's routed part (the sequencer's loads wait)
    hipEvent_t ev_xwb = nullptr;  // split pass: this shard's write-back of the sequencer's results done
    // Partitioned account records: the foreign accounts a routed sub-pass imports (k_node.h
    // tb_node_import), and the replicated limit-account bitmap.
    u32* imp_flag = nullptr;   // tb_pass_clear's import gate -> tb_node_import_flush
    u64* imp_count = nullptr;  // live imports (they stay across passes)
    u64 imp_cap = 0;           // the table's import room
    u32* imp_os = nullptr;  // [account_cap] an imported slot's slot on the account's owner (owner legs)
    u64* limbits = nullptr;
    u64 limmask = 0;             // bits - 1
};

struct NodeBlock {
    u32 k0 = 0, k1 = 0;  // global prepares [k0, k1)
    u64 events = 0;
};

struct NodePass {
    u32 k0 = 0, k1 = 0;
    NodeBlock blk[NODE_WORLD_MAX];
    u64* off[NODE_WORLD_MAX] = {};  // block-relative event offsets of its prepares (pb_src + 1, init-time)
    bool issued = false, consumed = false;
};
#define NODE_PASS_RING 4  // passes alive at once in a call: p - 2 (replies), p - 1, p, p + 1 (planned)

struct TbNode;
// The node's issue pool: one host thread per shard beyond the first (created at init), so a pass's
// per-shard work — a source's route plan, a home's routed commit, an owner's legs and a source's
// replies, each a chain of launches and event operations on that shard's streams — is issued for
// every shard at once instead of shard after shard (on N GPUs the host would otherwise issue ~N x
// the work of one pass per pass).  A phase runs its function for every shard and returns when all
// have; phases that wait on another shard's events of the same pass come after the phase that
// records them.  Idle workers spin briefly, then sleep on a condition variable.
typedef int (*NodeShardFn)(TbNode* N, u32 shard, void* ctx);
struct NodePool {
    std::vector<std::thread> threads;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<u64> gen{0};
    std::atomic<u32> done{0};
    std::atomic<bool> stop{false};
    u32 spin_us = 50;  // TBGPU_NODE_SPIN_US
    NodeShardFn fn = nullptr;
    void* ctx = nullptr;
    int status[NODE_WORLD_MAX] = {};
    std::string err[NODE_WORLD_MAX];
};

struct TbNode {
    u32 world = 0;
    NodeDev D[NODE_WORLD_MAX];
    u64 pe_src = 0;        // source events per pass per shard
    u32 pb_src = 0;        // source prepares per pass per shard
    u64 recv_cap = 0;      // events a home can receive in one pass (world * pe_src)
    u64 commit_ts = 0;
    // The sequencer (first device), sized at init for a whole pass: its log holds the loaded
    // transfers at [0, seq_tcap) and the pass at [seq_tcap, ...).
    tbgpu* X = nullptr;
    u64 seq_tcap = 0;
    SeqEntry* tset_e = nullptr;
    SeqEntry* aset_e = nullptr;
    u64 tset_mask = 0, aset_mask = 0;
    u32* tset_list = nullptr;
    u32* aset_list = nullptr;
    u64* seq_counts = nullptr;   // [0..1] tset, [2..3] aset, [4] loaded transfers
    u64* tset_dups = nullptr;
    u64* aset_dups = nullptr;
    u8* seq_codes = nullptr;     // [world * pe_src] the pass's dense codes from the sequencer (pass positions)
    u8* seq_xcodes = nullptr;    // [world * pe_src] its dense codes in compacted order
    u32* seq_map = nullptr;      // [world * pe_src] compacted index of each sequenced event
    u64* seq_ts = nullptr;       // [world * pe_src] execute timestamps of the compacted events
    u32* seq_blk = nullptr;      // [world * pe_src / 256 + 2] compaction counts / prefix
    AccountBal* seq_bal0 = nullptr;  // [6 * world * pe_src] balances as loaded (delta write-back)
    u32* xclr_list = nullptr;    // [xclr_cap] the sequencer's index entries a split pass claimed (tb_seq_xidx_list)
    u64* xclr_count = nullptr;
    u64 xclr_cap = 0;
    bool x_index_clean = true;   // the sequencer's transfer index, collision marks and posted states are empty
    hipEvent_t ev_xread = nullptr;   // the sequencer has read the split pass's source buffers
    hipEvent_t ev_x = nullptr;       // the sequencer's results (codes expanded) are final
    u64* h_seq = nullptr;        // pinned scratch words
    u64 passes_clean = 0, passes_split = 0, passes_whole = 0, seq_events = 0;
    bool limit_any = false;          // some account carries a limit flag (the bitmaps are consulted)
    // tbgpu_checkpoint_delta_async on a node: the merged delta is produced at the call (the shards'
    // objects are merged on the host, node_api_checkpoint_delta); the wait returns its counts.
    bool wb_inflight = false;
    tbgpu_delta_counts wb_counts{};
    u64 x_limit_seen = 0;            // the sequencer's limit_accounts count when last read
    const u64* api_calls = nullptr;  // the node handle's entry-point count (tbgpu::api_calls)
    NodePass ring[NODE_PASS_RING];   // a call's passes, built as they are planned (no per-call allocation)
    std::vector<u64> ring_off;       // their offset tables
    u64 drained_at = ~0ULL;          // its value when a create_transfers call last ended drained
    // TBGPU_NODE_TIMING=1 (set at init): host time per phase of create_transfers calls, printed at
    // deinit — plan issue, plan wait, commit issue, replies issue, consume wait, whole call.
    bool timing = false;
    NodePool* pool = nullptr;  // null: every phase issued shard after shard (TBGPU_NODE_THREADS=0)
    bool latency_on = false;  // the current call asked for per-prepare latencies (ev_start recorded)
    // Host memory registered through the node (node_api_register_host): a block in it is not in
    // HBM, known without asking the runtime per pass.
    struct HostRegion {
        const u8* p;
        u64 n;
    } host_reg[64];
    u32 n_host_reg = 0;
    double t_us[6] = {};
    u64 t_calls = 0;
    unsigned __int128 bound_carry = 0;  // the node's balance bound at that point (host-tracked)
};

static int node_fail_dev(const char* what, hipError_t e) {
    return fail(TBGPU_STATUS_DEVICE, "node: %s: %s", what, hipGetErrorString(e));
}

#define NCK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return node_fail_dev(#x, e_);                                        \
    } while (0)

static u32 node_home(const u8* rec16, u32 world) {
    const u64* w = (const u64*)rec16;
    return tb_home(w[0], w[1], world);
}

struct NodeTimer {  // adds the scope's host time to N->t_us[k] when N->timing
    TbNode* N;
    int k;
    std::chrono::steady_clock::time_point t0;
    NodeTimer(TbNode* n, int kk) : N(n), k(kk) {
        if (N->timing) t0 = std::chrono::steady_clock::now();
    }
    ~NodeTimer() {
        if (N->timing) N->t_us[k] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
};

static void node_pool_worker(TbNode* N, u32 d) {
    NodePool& Q = *N->pool;
    u64 seen = 0;
    for (;;) {
        // A job (gen past `seen`) or stop: spin Q.spin_us, then sleep until notified.
        const auto t0 = std::chrono::steady_clock::now();
        for (u32 spin = 0; Q.gen.load(std::memory_order_acquire) == seen && !Q.stop.load(); spin++) {
            __builtin_ia32_pause();
            if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(Q.spin_us)) break;
        }
        if (Q.gen.load(std::memory_order_acquire) == seen && !Q.stop.load()) {
            std::unique_lock<std::mutex> lk(Q.mu);
            Q.cv.wait(lk, [&] { return Q.gen.load(std::memory_order_acquire) != seen || Q.stop.load(); });
        }
        if (Q.stop.load()) return;
        seen = Q.gen.load(std::memory_order_acquire);
        const int st = Q.fn(N, d, Q.ctx);
        Q.status[d] = st;
        if (st) Q.err[d] = g_err;  // (the error text is per thread)
        Q.done.fetch_add(1, std::memory_order_acq_rel);
    }
}

// fn for every shard: shard 0 on the calling thread, the others on the pool.  The first failure's
// status and text come back to the caller.
static int node_run(TbNode* N, NodeShardFn fn, void* ctx) {
    const u32 W = N->world;
    if (!N->pool) {
        for (u32 d = 0; d < W; d++) {
            const int st = fn(N, d, ctx);
            if (st) return st;
        }
        return TBGPU_STATUS_OK;
    }
    NodePool& Q = *N->pool;
    Q.fn = fn;
    Q.ctx = ctx;
    Q.done.store(0, std::memory_order_relaxed);
    Q.gen.fetch_add(1, std::memory_order_acq_rel);
    { std::lock_guard<std::mutex> lk(Q.mu); }  // a worker checking its wait predicate sees the new gen
    Q.cv.notify_all();
    int status = fn(N, 0, ctx);
    while (Q.done.load(std::memory_order_acquire) < W - 1) __builtin_ia32_pause();
    for (u32 d = 1; d < W; d++) {
        if (Q.status[d] && !status) {
            status = Q.status[d];
            g_err = Q.err[d];
        }
    }
    return status;
}

static void node_pool_stop(TbNode* N) {
    if (!N->pool) return;
    N->pool->stop.store(true);
    { std::lock_guard<std::mutex> lk(N->pool->mu); }
    N->pool->cv.notify_all();
    for (std::thread& t : N->pool->threads) t.join();
    delete N->pool;
    N->pool = nullptr;
}

static void node_free(TbNode* N) {
    if (!N) return;
    node_pool_stop(N);
    if (N->timing && N->t_calls) {
        const double c = (double)N->t_calls;
        fprintf(stderr, "tbgpu node timing (us per create_transfers call, %llu calls): plan_issue %.1f plan_wait %.1f "
                        "commit_issue %.1f replies_issue %.1f consume_wait %.1f call %.1f\n",
                (unsigned long long)N->t_calls, N->t_us[0] / c, N->t_us[1] / c, N->t_us[2] / c, N->t_us[3] / c,
                N->t_us[4] / c, N->t_us[5] / c);
    }
    for (u32 d = 0; d < N->world; d++) {
        NodeDev& D = N->D[d];
        if (D.E) {
            (void)hipSetDevice(D.device);
            (void)hipDeviceSynchronize();
        }
        void* dev[] = {D.stage[0], D.stage[1], D.send[0], D.send[1], D.slot[0], D.slot[1], D.home[0], D.home[1],
                       D.words[0], D.words[1], D.meta[0], D.meta[1], D.block_counts, D.results, D.reply_bytes,
                       D.recv, D.codes, D.legs, D.leg_counts, D.hmeta_dev[0], D.hmeta_dev[1], D.hmeta_dev[2],
                       D.dep1, D.dep[0], D.dep[1], D.dkeys, D.dbal, D.dcounts, D.keyset, D.markset, D.wb_count,
                       D.imp_flag, D.imp_count, D.imp_os, D.limbits};
        for (void* p : dev) if (p) (void)hipFree(p);
        void* host[] = {D.h_words[0], D.h_words[1], D.h_meta[0], D.h_meta[1], D.hmeta_host[0], D.hmeta_host[1],
                        D.hmeta_host[2], D.h_arena[0], D.h_arena[1], D.h_arena[2], D.h_dcounts, D.h_flags};
        for (void* p : host) if (p) (void)hipHostFree(p);
        hipEvent_t evs[] = {D.ev_start[0], D.ev_start[1], D.ev_start[2], D.ev_done[0], D.ev_done[1], D.ev_done[2],
                            D.ev_planned[0], D.ev_planned[1], D.ev_copied, D.ev_gathered, D.ev_committed,
                            D.ev_applied, D.ev_replied, D.ev_cls, D.ev_marked, D.ev_pre, D.ev_xwb};
        for (hipEvent_t e : evs) if (e) (void)hipEventDestroy(e);
        if (D.rs) (void)hipStreamDestroy(D.rs);
        if (D.E) tbgpu_deinit(D.E);
    }
    if (N->X) {
        (void)hipSetDevice(N->D[0].device);
        void* dev[] = {N->tset_e, N->aset_e, N->tset_list, N->aset_list, N->seq_counts, N->tset_dups, N->aset_dups,
                       N->seq_codes, N->seq_xcodes, N->seq_map, N->seq_ts, N->seq_blk, N->seq_bal0, N->xclr_list,
                       N->xclr_count};
        for (void* p : dev) if (p) (void)hipFree(p);
        if (N->ev_xread) (void)hipEventDestroy(N->ev_xread);
        if (N->ev_x) (void)hipEventDestroy(N->ev_x);
        if (N->h_seq) (void)hipHostFree(N->h_seq);
        tbgpu_deinit(N->X);
    }
    delete N;
}

static u64 node_arena_bytes(const TbNode* N) { return 16 + (u64)N->pb_src * 4 + N->pe_src * 8; }

static int node_init(const tbgpu_config* config, TbNode** out) {
    *out = nullptr;
    const u32 W = config->device_count;
    if (W < 2 || W > NODE_WORLD_MAX) return fail(TBGPU_STATUS_INVALID, "device_count %u out of range (2..%u)", W, NODE_WORLD_MAX);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(TBGPU_STATUS_DEVICE, "tbgpu_init: no HIP device visible");
    for (u32 d = 0; d < W; d++) {
        if (config->devices[d] < 0 || config->devices[d] >= ndev) {
            return fail(TBGPU_STATUS_INVALID, "tbgpu_init: devices[%u] = %d out of range (%d devices)", d, config->devices[d], ndev);
        }
    }
    TbNode* N = new TbNode();
    if (const char* t = getenv("TBGPU_NODE_TIMING")) N->timing = atoi(t) != 0;
    {
        const char* t = getenv("TBGPU_NODE_THREADS");
        if (!(t && atoi(t) == 0) && W >= 2) {
            N->pool = new NodePool();
            if (const char* us = getenv("TBGPU_NODE_SPIN_US")) N->pool->spin_us = (u32)atoi(us);
            for (u32 d = 1; d < W; d++) N->pool->threads.emplace_back(node_pool_worker, N, d);
        }
    }
    N->world = W;
    N->pe_src = config->pass_events_max;
    N->pb_src = config->pass_batches_max;
    N->recv_cap = (u64)W * N->pe_src;
    N->ring_off.assign((u64)NODE_PASS_RING * W * (N->pb_src + 1), 0);
    for (u32 r = 0; r < NODE_PASS_RING; r++) {
        for (u32 d = 0; d < W; d++) N->ring[r].off[d] = N->ring_off.data() + ((u64)r * W + d) * (N->pb_src + 1);
    }
    // Shard engines: the accounts owned there (below), the transfer log of the transfers homed there
    // (1/N of the ledger, with room for hash imbalance), routed passes of up to ~1.25x a source
    // block (larger receipts are committed in several passes).
    tbgpu_config sc = *config;
    sc.device_count = 0;
    sc.transfers_max = std::min<u64>(1ULL << 31, config->transfers_max / W + config->transfers_max / (8 * W) + N->recv_cap + 4096);
    sc.pass_events_max = (u32)std::min<u64>(N->recv_cap, N->pe_src + N->pe_src / 4 + 8192);
    sc.pass_batches_max = (u32)std::min<u64>(FLOW_NB_MAX, (sc.pass_events_max + BATCH_EVENTS_MAX - 2) / (BATCH_EVENTS_MAX - 1) + 2);
    sc.pass_batches_max = std::max(sc.pass_batches_max, N->pb_src);
    // Accounts: the ones this shard owns (1/N of the ledger, with room for hash imbalance) plus the
    // import room — every account of the ledger when that is smaller than a routed sub-pass's two per
    // event (imports then never need a flush, and the table stays as dense as the ledger allows: its
    // random probes hit the MALL), else the sub-pass's two per event (k_node.h tb_node_import_flush).
    const u64 owned = std::min<u64>(config->accounts_max, config->accounts_max / W + config->accounts_max / (8 * W) + 4096);
    const u64 import_room = std::min<u64>(config->accounts_max, 2 * (u64)sc.pass_events_max);
    sc.accounts_max = std::min<u64>(1ULL << 31, owned + import_room);
    int st = TBGPU_STATUS_OK;
    for (u32 d = 0; d < W && st == TBGPU_STATUS_OK; d++) {
        NodeDev& D = N->D[d];
        D.device = config->devices[d];
        sc.device = D.device;
        st = tbgpu_init(&sc, &D.E);
    }
    if (st) {
        node_free(N);
        return st;
    }
    // Peer access between distinct devices (a kernel on one reads the other's HBM over xGMI).
    for (u32 a = 0; a < W; a++) {
        for (u32 b = 0; b < W; b++) {
            const int da = N->D[a].device, db = N->D[b].device;
            if (da == db) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, da, db) != hipSuccess || !can) {
                node_free(N);
                return fail(TBGPU_STATUS_DEVICE, "tbgpu_init: device %d cannot access device %d (no xGMI/P2P path)", da, db);
            }
            (void)hipSetDevice(da);
            const hipError_t e = hipDeviceEnablePeerAccess(db, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                node_free(N);
                return node_fail_dev("hipDeviceEnablePeerAccess", e);
            }
            (void)hipGetLastError();  // clear "already enabled"
        }
    }
    const u64 pe = N->pe_src, nblocks = (pe + ROUTE_THREADS - 1) / ROUTE_THREADS;
    const u64 legs_cap_total = (u64)W * 2 * N->recv_cap;  // W regions of up to 2 legs per received event
    hipError_t e = hipSuccess;
#define NALLOC(x) \
    if (e == hipSuccess) e = (x)
    for (u32 d = 0; d < W && e == hipSuccess; d++) {
        NodeDev& D = N->D[d];
        NALLOC(hipSetDevice(D.device));
        NALLOC(hipStreamCreateWithFlags(&D.rs, hipStreamNonBlocking));
        for (int k = 0; k < 2; k++) {
            NALLOC(tbMalloc(&D.stage[k], pe * 128));
            NALLOC(tbMalloc(&D.send[k], pe * 128));
            NALLOC(tbMalloc(&D.slot[k], pe * 4));
            NALLOC(tbMalloc(&D.home[k], pe));
            NALLOC(tbMalloc(&D.words[k], ROUTE_WORDS * 8));
            NALLOC(hipMemsetAsync(D.words[k], 0, ROUTE_WORDS * 8, D.rs));
            NALLOC(tbHostMalloc(&D.h_words[k], ROUTE_WORDS * 8, hipHostMallocMapped));
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&D.d_words_host[k], D.h_words[k], 0);
            NALLOC(tbMalloc(&D.meta[k], (2 * (u64)N->pb_src + 1) * 8));
            NALLOC(tbHostMalloc(&D.h_meta[k], (2 * (u64)N->pb_src + 1) * 8, hipHostMallocDefault));
            NALLOC(tbEventCreateWithFlags(&D.ev_planned[k], hipEventDisableTiming));
        }
        NALLOC(tbMalloc(&D.block_counts, 2 * nblocks * W * 4));
        NALLOC(tbMalloc(&D.results, pe * 8));
        NALLOC(tbMalloc(&D.reply_bytes, (u64)N->pb_src * 4));
        NALLOC(tbMalloc(&D.codes, N->recv_cap));
        NALLOC(tbMalloc(&D.legs, legs_cap_total * NODE_LEG_WORDS * 8));
        NALLOC(tbMalloc(&D.leg_counts, (u64)W * 8));
        const u64 hm = 2 * ((N->recv_cap + BATCH_EVENTS_MAX - 2) / (BATCH_EVENTS_MAX - 1) + 2) + 1;
        for (int k = 0; k < 3; k++) {
            NALLOC(tbMalloc(&D.hmeta_dev[k], hm * 8));
            NALLOC(tbHostMalloc(&D.hmeta_host[k], hm * 8, hipHostMallocDefault));
            NALLOC(tbHostMalloc(&D.h_arena[k], node_arena_bytes(N), hipHostMallocMapped));
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&D.d_arena[k], D.h_arena[k], 0);
            NALLOC(tbEventCreate(&D.ev_start[k]));
            NALLOC(tbEventCreate(&D.ev_done[k]));
        }
        NALLOC(tbHostMalloc(&D.h_flags, 64, hipHostMallocMapped));
        if (e == hipSuccess) {
            memset(D.h_flags, 0, 64);
            e = hipHostGetDevicePointer((void**)&D.d_flags, D.h_flags, 0);
        }
        NALLOC(tbEventCreateWithFlags(&D.ev_copied, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_gathered, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_committed, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_applied, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_replied, hipEventDisableTiming));
        // The events of "the previous pass" exist before the first pass: record them once.
        NALLOC(hipEventRecord(D.ev_gathered, D.E->stream));
        NALLOC(hipEventRecord(D.ev_applied, D.E->stream));
        NALLOC(hipEventRecord(D.ev_replied, D.E->stream));
        // Dirty passes: the block's classification, the key sets (every source's keys), the
        // sequencer write-back counter.
        D.set_mask = pow2_at_least(std::max<u64>(1024, 4 * (u64)W * pe)) - 1;
        NALLOC(tbMalloc(&D.dep1, pe));
        NALLOC(tbMalloc(&D.dep[0], pe));
        NALLOC(tbMalloc(&D.dep[1], pe));
        NALLOC(tbMalloc(&D.dkeys, 2 * pe * 16));
        NALLOC(tbMalloc(&D.dbal, 2 * pe * 16));
        NALLOC(tbMalloc(&D.dcounts, NODE_DC_WORDS * 8));
        NALLOC(tbHostMalloc(&D.h_dcounts, NODE_DC_WORDS * 8, hipHostMallocDefault));
        NALLOC(tbMalloc(&D.keyset, (D.set_mask + 1) * 8));
        NALLOC(tbMalloc(&D.markset, (D.set_mask + 1) * 8));
        NALLOC(tbMalloc(&D.wb_count, 8));
        NALLOC(tbEventCreateWithFlags(&D.ev_cls, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_marked, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_pre, hipEventDisableTiming));
        NALLOC(tbEventCreateWithFlags(&D.ev_xwb, hipEventDisableTiming));
        D.imp_cap = import_room;
        NALLOC(tbMalloc(&D.imp_flag, 4));
        NALLOC(tbMalloc(&D.imp_count, 8));
        NALLOC(hipMemset(D.imp_count, 0, 8));
        NALLOC(tbMalloc(&D.imp_os, D.E->account_cap * 4));
        // 16 bits per account of the ledger: a false positive (which only sequences an event) is at
        // most 1 in 16 even when every account is limited.
        const u64 lim_bits = std::min<u64>(1ULL << 34, pow2_at_least(std::max<u64>(1ULL << 16, 16 * config->accounts_max)));
        D.limmask = lim_bits - 1;
        NALLOC(tbMalloc(&D.limbits, lim_bits / 8));
        NALLOC(hipMemset(D.limbits, 0, lim_bits / 8));
    }
#undef NALLOC
    if (e != hipSuccess) {
        node_free(N);
        return node_fail_dev("tbgpu_init (node buffers)", e);
    }
    // The sequencer: one whole pass (every source's block) with the objects it can read — two
    // transfers (id, pending id) and up to four accounts per event.
    {
        const u64 pass = (u64)W * pe;
        tbgpu_config xc = sc;
        xc.device = N->D[0].device;
        xc.flags &= ~(u32)TBGPU_CONFIG_PROFILE;
        xc.accounts_max = std::max<u64>(1024, std::min<u64>(config->accounts_max, 4 * pass));
        N->seq_tcap = 2 * pass;
        xc.transfers_max = N->seq_tcap + pass;
        xc.pass_events_max = (u32)std::min<u64>(pass, 0xFFFFFFFFull);
        xc.pass_batches_max = W * N->pb_src;
        int st2 = tbgpu_init(&xc, &N->X);
        if (st2) {
            node_free(N);
            return st2;
        }
        // The sequencer's passes are the dependent events of a node pass: a tenth to a quarter of it
        // in C3 / C4, Zipf-hot.  Balance legs (per-account LDS sums) from 8K events on: below the
        // single engine's threshold, atomics on the hot accounts would serialise.
        N->X->legs_min = 8192;
        (void)hipSetDevice(N->D[0].device);
        N->tset_mask = pow2_at_least(4 * pass) - 1;
        N->aset_mask = pow2_at_least(2 * (xc.accounts_max + 2 * pass)) - 1;
#define XALLOC(x) \
    if (e == hipSuccess) e = (x)
        XALLOC(tbMalloc(&N->tset_e, (N->tset_mask + 1) * sizeof(SeqEntry)));
        XALLOC(tbMalloc(&N->aset_e, (N->aset_mask + 1) * sizeof(SeqEntry)));
        XALLOC(tbMalloc(&N->tset_list, 2 * pass * 4));
        XALLOC(tbMalloc(&N->aset_list, 6 * pass * 4));
        XALLOC(tbMalloc(&N->seq_counts, 8 * 8));
        XALLOC(tbMalloc(&N->tset_dups, 2 * pass * 24));
        XALLOC(tbMalloc(&N->aset_dups, 6 * pass * 24));
        XALLOC(tbMalloc(&N->seq_codes, pass));
        XALLOC(tbMalloc(&N->seq_xcodes, pass));
        XALLOC(tbMalloc(&N->seq_map, pass * 4));
        XALLOC(tbMalloc(&N->seq_ts, pass * 8));
        XALLOC(tbMalloc(&N->seq_blk, (pass / 256 + 2) * 4));
        XALLOC(tbMalloc(&N->seq_bal0, 6 * pass * sizeof(AccountBal)));
        N->xclr_cap = 2 * (N->seq_tcap + pass);  // two entries per log position (a withdrawn claim and a new one)
        XALLOC(tbMalloc(&N->xclr_list, N->xclr_cap * 4));
        XALLOC(tbMalloc(&N->xclr_count, 8));
        XALLOC(tbEventCreateWithFlags(&N->ev_xread, hipEventDisableTiming));
        XALLOC(tbEventCreateWithFlags(&N->ev_x, hipEventDisableTiming));
        XALLOC(hipEventRecord(N->ev_xread, N->X->stream));  // "the previous split pass" exists before the first
        XALLOC(tbHostMalloc(&N->h_seq, 16 * 8, hipHostMallocDefault));
        XALLOC(hipMemset(N->tset_e, 0, (N->tset_mask + 1) * sizeof(SeqEntry)));
        XALLOC(hipMemset(N->aset_e, 0, (N->aset_mask + 1) * sizeof(SeqEntry)));
#undef XALLOC
        if (e != hipSuccess) {
            node_free(N);
            return node_fail_dev("tbgpu_init (node sequencer)", e);
        }
    }
    *out = N;
    return TBGPU_STATUS_OK;
}

// Drain every device (and the sequencer) and read back its globals (panic, commit_timestamp).
static int node_sync(TbNode* N) {
    int status = TBGPU_STATUS_OK;
    if (N->X) {
        NCK(hipSetDevice(N->D[0].device));
        NCK(hipStreamSynchronize(N->X->stream));
    }
    for (u32 d = 0; d < N->world; d++) {
        NodeDev& D = N->D[d];
        NCK(hipSetDevice(D.device));
        NCK(hipStreamSynchronize(D.rs));
        NCK(hipStreamSynchronize(D.E->copy_stream));
        const int st = engine_sync(D.E);
        if (st && status == TBGPU_STATUS_OK) status = st;
        N->commit_ts = std::max(N->commit_ts, D.E->commit_ts);
    }
    return status;
}

// Every shard's imports out of its table (k_node.h tb_node_import_flush), on its engine stream:
// before an account is inserted on a shard (so no import sits on an owned probe chain) and before a
// table is read whole.  Routed passes import again what they name.
static int node_imports_flush(TbNode* N) {
    for (u32 d = 0; d < N->world; d++) {
        NodeDev& D = N->D[d];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        hipLaunchKernelGGL(tb_node_import_flush, dim3((u32)std::min<u64>(1024, (E->account_cap + 255) / 256)), dim3(256), 0,
                           E->stream, E->T, E->account_cap, N->world, d, (const u32*)nullptr);
        NCK(hipGetLastError());
        NCK(hipMemsetAsync(D.imp_count, 0, 8, E->stream));
    }
    return TBGPU_STATUS_OK;
}

// Sum of the shards' balance bounds (every true, owner-held balance is below it).
static unsigned __int128 node_bound(TbNode* N) {
    typedef unsigned __int128 h128;
    h128 total = 0;
    for (u32 d = 0; d < N->world; d++) {
        const Globals& g = *N->D[d].E->h_globals;  // read back by engine_sync
        const h128 b = ((h128)g.bound_hi << 64) | g.bound_lo;
        total = total + b < total ? ~(h128)0 : total + b;
    }
    return total;
}

// Every shard's commit_timestamp := the node's (host field and device global), on its stream.
static int node_publish_commit_ts(TbNode* N) {
    for (u32 d = 0; d < N->world; d++) {
        tbgpu* E = N->D[d].E;
        NCK(hipSetDevice(N->D[d].device));
        E->commit_ts = N->commit_ts;
        E->last_batch_ts = N->commit_ts;
        // Not waited for: the shard's next work follows it on the stream, and a later push that
        // overwrites the staging word before this copy runs only carries a newer timestamp.
        *E->h_pub = N->commit_ts;
        NCK(hipMemcpyAsync(&E->g->commit_timestamp, E->h_pub, 8, hipMemcpyHostToDevice, E->stream));
    }
    return TBGPU_STATUS_OK;
}

// -- create_accounts: committed in order by the sequencer, each new account to its owner -----------
// The reference's create_account reads only the account's own id (exists, :757-765) and the batch's
// earlier events (linked chains, :628-692): the sequencer gets the pass verbatim, loads from their
// owners the existing accounts the events name (prefetch, src/state_machine.zig:345-506), commits it
// with the normal kernels, and each shard takes the accounts it created that the shard owns; every
// shard's limit bitmap learns the new limit accounts.  The sequencer's account table is emptied after
// each pass (tombstones of rolled-back chains included).
static int node_commit_accounts(TbNode* N, u32 n, const u64* ts, const void* const* inputs, const u32* lens,
                                void* const* outputs, u32* out_lens) {
    const u32 W = N->world;
    tbgpu* X = N->X;
    const int dev0 = N->D[0].device;
    int st = node_imports_flush(N);  // new accounts go into the owners' tables below
    if (!st) st = node_sync(N);      // the owners' tables are read below
    if (st) return st;
    for (u32 k = 0; k < n; k++) ckpt_note_ids(N->D[0].E, (const u8*)inputs[k], lens[k]);  // the next write-back
    NodeTablesArgs NT{};
    NT.world = W;
    for (u32 d = 0; d < W; d++) NT.T[d] = N->D[d].E->T;
    SeqSet tset{N->tset_e, N->tset_mask, N->tset_list, N->seq_counts, N->tset_dups};
    SeqSet aset{N->aset_e, N->aset_mask, N->aset_list, N->seq_counts + 2, N->aset_dups};
    for (u32 k0 = 0; k0 < n;) {
        u32 k1 = k0;
        u64 ev = 0;
        while (k1 < n && k1 - k0 < X->pb_max && k1 - k0 < X->meta_cap && ev + lens[k1] <= X->pe_max) ev += lens[k1++];
        if (k1 == k0) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
        const u32 nb = k1 - k0;
        NCK(hipSetDevice(dev0));
        hipStream_t xs = X->stream;
        u64* h_off = X->h_meta;
        u64* h_ts = X->h_meta + nb + 1;
        h_off[0] = 0;
        for (u32 k = k0; k < k1; k++) {
            h_off[k - k0 + 1] = h_off[k - k0] + lens[k];
            h_ts[k - k0] = ts[k];
        }
        for (u32 k = k0; k < k1; k++) {
            if (lens[k]) NCK(hipMemcpyAsync(X->staging + h_off[k - k0] * 128, inputs[k], (u64)lens[k] * 128, hipMemcpyDefault, xs));
        }
        NCK(hipMemcpyAsync(X->meta, X->h_meta, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, xs));
        NCK(hipMemsetAsync(N->seq_counts, 0, 8 * 8, xs));
        const u64 ne = h_off[nb];
        if (ne) {
            hipLaunchKernelGGL(tb_seq_account_ids, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, xs, X->staging, ne, aset);
            hipLaunchKernelGGL(tb_seq_verify, dim3(256), dim3(256), 0, xs, aset, (u64*)&X->g->panic);
            hipLaunchKernelGGL(tb_seq_load_accounts, dim3(1024), dim3(256), 0, xs, NT, aset, X->T, (AccountBal*)nullptr);
            NCK(hipGetLastError());
        }
        N->h_seq[0] = N->commit_ts;
        NCK(hipMemcpyAsync(&X->g->commit_timestamp, N->h_seq, 8, hipMemcpyHostToDevice, xs));
        X->commit_ts = N->commit_ts;
        X->last_batch_ts = N->commit_ts;
        if ((st = enqueue_call(X, OP_CREATE_ACCOUNTS, nb, h_off, X->staging, X->results, X->reply_bytes, false, nullptr, 0,
                               nullptr, X->meta))) {
            return st;
        }
        hipLaunchKernelGGL(tb_seq_locate_new, dim3(1024), dim3(256), 0, xs, aset, X->T);
        NCK(hipGetLastError());
        NCK(hipMemcpyAsync(X->h_rb, X->reply_bytes, (u64)nb * 4, hipMemcpyDeviceToHost, xs));
        if ((st = engine_sync(X))) return st;
        for (u32 k = k0; k < k1; k++) {
            const u32 bytes = X->h_rb[k - k0];
            if (bytes) NCK(hipMemcpy(outputs[k], X->results + 2 * h_off[k - k0], bytes, hipMemcpyDeviceToHost));
            out_lens[k] = bytes;
        }
        N->commit_ts = std::max(N->commit_ts, X->commit_ts);
        if (X->h_globals->limit_accounts != N->x_limit_seen) {  // a limit account was created (or loaded)
            N->x_limit_seen = X->h_globals->limit_accounts;
            N->limit_any = true;
        }
        // Each shard takes the accounts it owns (its own stream, reading the sequencer over xGMI).
        for (u32 d = 0; d < W; d++) {
            NodeDev& D = N->D[d];
            NCK(hipSetDevice(D.device));
            hipLaunchKernelGGL(tb_seq_writeback_new_accounts, dim3(1024), dim3(256), 0, D.E->stream, X->T, aset, D.E->T, d,
                               W, D.limbits, D.limmask);
            NCK(hipGetLastError());
        }
        for (u32 d = 0; d < W; d++) {
            NCK(hipSetDevice(N->D[d].device));
            NCK(hipStreamSynchronize(N->D[d].E->stream));
        }
        // The sequencer empty again: its entries, the sets, and (by one sweep) the tombstones of
        // rolled-back creates.
        NCK(hipSetDevice(dev0));
        hipLaunchKernelGGL(tb_seq_clear, dim3(1024), dim3(256), 0, xs, tset, aset, X->T);
        NCK(hipGetLastError());
        NCK(hipMemsetAsync(X->T.acct_hot, 0, X->account_cap * sizeof(AccountHot), xs));
        NCK(hipStreamSynchronize(xs));
        k0 = k1;
    }
    return node_sync(N);
}

// -- create_transfers ----------------------------------------------------------------------------

// Is source d's block of the pass already in d's HBM, its prepares back to back?  (Then the route
// kernels read it in place: the node's device-resident commit, the prepares generated or received
// on each GPU.)
static bool node_block_resident(const TbNode* N, const NodeDev& D, const NodePass& P, u32 d, const void* const* inputs,
                                const u32* lens) {
    const NodeBlock& B = P.blk[d];
    if (B.k1 == B.k0 || B.events == 0) return false;
    const u8* base = (const u8*)inputs[B.k0];
    for (u32 i = 0; i < N->n_host_reg; i++) {
        if (base >= N->host_reg[i].p && base < N->host_reg[i].p + N->host_reg[i].n) return false;
    }
    for (u32 k = B.k0; k < B.k1; k++) {
        if ((const u8*)inputs[k] != base + P.off[d][k - B.k0] * 128) return false;
    }
    hipPointerAttribute_t attr{};
    if (hipPointerGetAttributes(&attr, base) != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory: not a HIP allocation
        return false;
    }
    (void)lens;
    return attr.type == hipMemoryTypeDevice && attr.device == D.device;
}

static u32 node_next_seq(NodeDev& D) {
    if (++D.flag_seq == 0) ++D.flag_seq;
    return D.flag_seq;
}

// Spin until a kernel wrote `seq` into a completion word (a stream's completion signal reaches a
// waiting host thread later).  False after 2 s: the caller waits on the stream's event instead,
// which reports a fault.
static bool node_spin(const u32* word, u32 seq) {
    volatile const u32* w = word;
    const auto t0 = std::chrono::steady_clock::now();
    for (u32 spin = 0; *w != seq; spin++) {
        if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return false;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return true;
}

// H2D of source d's block of pass p and its route plan (enqueued; ev_planned[p & 1] fires, and the
// plan flag takes plan_seq[p & 1], when the plan's words are in pinned host memory).
struct NodePlanJob {
    NodePass* P;
    u32 p;
    const u64* ts;
    const void* const* inputs;
    const u32* lens;
    bool single;  // the call is this one pass: its bodies cross on the route stream (no event hop)
};

static int node_plan_one(TbNode* N, u32 d, void* ctx) {
    const NodePlanJob& J = *(const NodePlanJob*)ctx;
    NodePass& P = *J.P;
    const u32 p = J.p, par = p & 1;
    const u64* ts = J.ts;
    const void* const* inputs = J.inputs;
    const u32* lens = J.lens;
    {
        NodeDev& D = N->D[d];
        const NodeBlock& B = P.blk[d];
        const u32 nb = B.k1 - B.k0;
        if (nb == 0) return TBGPU_STATUS_OK;
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        u64* h_off = D.h_meta[par];
        u64* h_ts = h_off + nb + 1;
        for (u32 k = 0; k <= nb; k++) h_off[k] = P.off[d][k];
        for (u32 k = 0; k < nb; k++) h_ts[k] = ts[B.k0 + k];
        // The block's bodies.  Already in this device's HBM, back to back (a device-resident call):
        // read where they are.  Otherwise the copy stream moves them (runs of address-contiguous
        // prepares as one DMA; host memory over the device's own PCIe link, another device's HBM
        // over xGMI).
        // A one-pass call has no next plan to overlap: its copy goes on the route stream itself (a
        // cross-stream event hop costs ~15 us on the device between the copy and the plan).
        hipStream_t cs = J.single ? D.rs : E->copy_stream;
        if (N->latency_on) NCK(hipEventRecord(D.ev_start[p % 3], cs));
        // The sequencer of the split pass two passes back may still be reading this parity's buffers.
        if (!J.single) NCK(hipStreamWaitEvent(E->copy_stream, N->ev_xread, 0));
        NCK(hipStreamWaitEvent(D.rs, N->ev_xread, 0));
        D.ev[par] = D.stage[par];
        if (node_block_resident(N, D, P, d, inputs, lens)) {
            D.ev[par] = (const u8*)inputs[B.k0];
        } else {
            for (u32 k = B.k0; k < B.k1;) {
                u32 j = k + 1;
                const u8* base = (const u8*)inputs[k];
                u64 bytes = (u64)lens[k] * 128;
                while (j < B.k1 && (const u8*)inputs[j] == base + bytes) bytes += (u64)lens[j++] * 128;
                if (bytes) NCK(hipMemcpyAsync(D.stage[par] + P.off[d][k - B.k0] * 128, base, bytes, hipMemcpyDefault, cs));
                k = j;
            }
        }
        if (!J.single) {
            NCK(hipEventRecord(D.ev_copied, E->copy_stream));
            NCK(hipStreamWaitEvent(D.rs, D.ev_copied, 0));
        }
        // Route stream: wait for the buffers' previous users (pass p-2's gathers on every home and
        // this source's replies), then the plan.
        NCK(hipStreamWaitEvent(D.rs, D.ev_replied, 0));
        for (u32 h = 0; h < N->world; h++) {
            NCK(hipSetDevice(D.device));
            NCK(hipStreamWaitEvent(D.rs, N->D[h].ev_gathered, 0));
        }
        // One prepare with events (the replica's commit): its metadata written by the classification
        // from kernel arguments, no copy.  The words are zero already (tb_route_publish).
        const bool im = nb == 1 && B.events > 0;
        if (!im) NCK(hipMemcpyAsync(D.meta[par], h_off, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, D.rs));
        RouteArgs A{};
        if (im) {
            A.im_meta = D.meta[par];
            A.im_ts = h_ts[0];
        }
        A.events = D.ev[par];
        A.n = (u32)B.events;
        A.nb = nb;
        A.batch_off = D.meta[par];
        A.batch_ts = D.meta[par] + nb + 1;
        A.world = N->world;
        A.nblocks = (u32)((B.events + ROUTE_THREADS - 1) / ROUTE_THREADS);
        A.home = D.home[par];
        A.block_counts = D.block_counts;
        A.block_base = D.block_counts + (u64)A.nblocks * N->world;
        A.words = D.words[par];
        A.T = E->T;
        A.skip = nullptr;
        A.limbits = D.limbits;
        A.limmask = D.limmask;
        A.limit_any = N->limit_any ? 1u : 0u;
        if (B.events) {
            hipLaunchKernelGGL(tb_route_classify, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A);
            NCK(hipGetLastError());
            hipLaunchKernelGGL(tb_route_offsets, dim3(A.world), dim3(1024), 0, D.rs, A);
            NCK(hipGetLastError());
            hipLaunchKernelGGL(tb_route_scatter, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A, D.send[par], D.slot[par]);
            NCK(hipGetLastError());
        }
        D.plan_seq[par] = node_next_seq(D);
        hipLaunchKernelGGL(tb_route_publish, dim3(1), dim3(64), 0, D.rs, D.words[par], D.d_words_host[par], D.d_flags + par,
                           D.plan_seq[par]);
        NCK(hipGetLastError());
        NCK(hipEventRecord(D.ev_planned[par], D.rs));
    }
    return TBGPU_STATUS_OK;
}

static int node_issue_plan(TbNode* N, NodePass& P, u32 p, const u64* ts, const void* const* inputs, const u32* lens,
                           bool single) {
    NodeTimer timer(N, 0);
    NodePlanJob J{&P, p, ts, inputs, lens, single};
    return node_run(N, node_plan_one, &J);
}

struct NodePlan {
    u64 C[NODE_WORLD_MAX][NODE_WORLD_MAX];  // events of source s for home h
    unsigned __int128 S = 0;                // saturating sum of every amount of the pass
    u32 dirty = 0;
    bool huge = false;
};

// spin: the words are all the caller reads (a clean plan); otherwise (a split pass, which reads its
// classification counts too) the route stream's event is waited for.
static int node_read_plan(TbNode* N, const NodePass& P, u32 p, NodePlan* out, bool spin = true) {
    typedef unsigned __int128 h128;
    memset(out->C, 0, sizeof(out->C));
    out->S = 0;
    out->dirty = 0;
    out->huge = false;
    const u32 par = p & 1;
    for (u32 d = 0; d < N->world; d++) {
        if (P.blk[d].k1 == P.blk[d].k0) continue;
        NodeDev& D = N->D[d];
        NCK(hipSetDevice(D.device));
        {
            NodeTimer timer(N, 1);
            if (!spin || !node_spin(D.h_flags + par, D.plan_seq[par])) NCK(hipEventSynchronize(D.ev_planned[par]));
        }
        const u64* w = D.h_words[par];
        if (w[RW_HUGE]) out->huge = true;
        for (int i = 0; i < SUM_SHARDS && !out->huge; i++) {
            const h128 v = ((h128)w[2 * i + 1] << 64) | w[2 * i];
            const h128 r = out->S + v;
            if (r < out->S) out->huge = true;
            out->S = r;
        }
        out->dirty |= (u32)w[RW_DIRTY];
        for (u32 h = 0; h < N->world; h++) out->C[d][h] = w[RW_COUNTS + h];
    }
    if (out->huge) out->S = ~(h128)0;
    return TBGPU_STATUS_OK;
}

// Where each source's run for each home sits, on both sides of the exchange.
struct NodeRoute {
    u64 R[NODE_WORLD_MAX][NODE_WORLD_MAX];    // R[h][s]: where source s's run starts in home h's receipt
    u64 off[NODE_WORLD_MAX][NODE_WORLD_MAX];  // off[s][h]: where home h's run starts in source s's send buffer
    u64 nh[NODE_WORLD_MAX];
};

static void node_route(const TbNode* N, const NodePlan& PL, NodeRoute& X) {
    const u32 W = N->world;
    for (u32 h = 0; h < W; h++) {
        u64 r = 0;
        for (u32 s = 0; s < W; s++) {
            X.R[h][s] = r;
            r += PL.C[s][h];
        }
        X.nh[h] = r;
    }
    for (u32 s = 0; s < W; s++) {
        u64 o = 0;
        for (u32 h = 0; h < W; h++) {
            X.off[s][h] = o;
            o += PL.C[s][h];
        }
    }
}

static int node_issue_replies(TbNode* N, NodePass& P, u32 p, const NodeRoute& X, const u8* seq_codes);

struct NodeCommitJob {
    NodePass* P;
    u32 p;
    const NodeRoute* RT;
    u32 cert;
    u64 ts_max;
    bool replies;
};
struct NodeReplyJob {
    NodePass* P;
    u32 p;
    const NodeRoute* RT;
    const u8* seq_codes;
};
static int node_reply_one(TbNode* N, u32 s, void* ctx);

// 1. Home h: gather, then (after the previous pass's readers of codes / legs) the routed commit.
static int node_home_one(TbNode* N, u32 h, void* ctx) {
    const NodeCommitJob& J = *(const NodeCommitJob*)ctx;
    const u32 W = N->world, par = J.p & 1, tri = J.p % 3;
    const u32 cert = J.cert;
    const u64 ts_max = J.ts_max;
    const auto& R = J.RT->R;
    const auto& off = J.RT->off;
    const auto& nh = J.RT->nh;
    {
        NodeDev& D = N->D[h];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        // The home's run lands at its transfer-log positions (the log window) and is committed in
        // place: validate stamps each committed record's timestamp instead of storing the record
        // (128 B an event less), as the single engine's in-place commit does.
        u8* window = (u8*)(E->T.xlog + E->log_next);
        if (nh[h]) {
            NodeGatherArgs G{};
            G.world = W;
            G.recv = window;
            for (u32 s = 0; s < W; s++) {
                G.src[s] = N->D[s].send[par] + off[s][h] * 128;
                G.start[s] = R[h][s];
            }
            G.start[W] = nh[h];
            hipLaunchKernelGGL(tb_node_gather, dim3((unsigned)((nh[h] * 8 + 256 * GATHER_PER - 1) / (256 * GATHER_PER))),
                               dim3(256), 0, E->stream, G);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_gathered, E->stream));
        // The previous pass's readers of this home's legs and codes: every shard's owner apply and
        // replies.  Both run on that shard's stream, the replies after the apply (node_issue_replies,
        // also for a split pass), so its latest replies event covers both.
        for (u32 o = 0; o < W; o++) {
            NCK(hipSetDevice(D.device));
            NCK(hipStreamWaitEvent(E->stream, N->D[o].ev_replied, 0));
        }
        NCK(hipSetDevice(D.device));
        if (!nh[h]) NCK(hipMemsetAsync(D.leg_counts, 0, (u64)W * 8, E->stream));  // (otherwise: tb_pass_clear)
        if (nh[h]) {
            const u64 per = BATCH_EVENTS_MAX - 1;
            const u64 nb = (nh[h] + per - 1) / per;
            u64* h_off = D.hmeta_host[tri];
            u64* h_ts = h_off + nb + 1;
            h_off[0] = 0;
            for (u64 k = 0; k < nb; k++) {  // routed events carry their own timestamps
                h_off[k + 1] = std::min<u64>(nh[h], h_off[k] + per);
                h_ts[k] = ts_max;
            }
            // One pseudo-prepare (a pass of up to 8191 routed events, the one-prepare call's): its
            // offsets and timestamp written by tb_pass_clear from kernel arguments, no copy.
            const u64 im[3] = {0, nh[h], ts_max};
            if (nb > 1) NCK(hipMemcpyAsync(D.hmeta_dev[tri], h_off, (2 * nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
            OwnerLegArgs O{W, h, D.legs, 2 * nh[h], D.leg_counts, D.imp_os, NODE_LEG_WORDS};
            NodeImport imp{};
            imp.N.world = W;
            for (u32 d = 0; d < W; d++) imp.N.T[d] = N->D[d].E->T;
            imp.self = h;
            imp.count = D.imp_count;
            imp.room = D.imp_cap;
            imp.flag = D.imp_flag;
            imp.os_of = D.imp_os;
            imp.leg_counts = D.leg_counts;
            imp.legs_n = W;
            imp.ev_legs = (void*)D.ev_committed;  // the owners need not wait for the import clear
            E->inplace_call = true;
            const int st = enqueue_call(E, OP_CREATE_TRANSFERS, (u32)nb, h_off, window, E->results, E->reply_bytes,
                                        true, D.codes, cert, nullptr, D.hmeta_dev[tri], &O, nb == 1 ? im : nullptr, &imp);
            E->inplace_call = false;
            if (st) return st;
        } else {
            NCK(hipEventRecord(D.ev_committed, E->stream));
        }
    }
    return TBGPU_STATUS_OK;
}

// 2. Owner o: the legs it owns, from every home (after every home's commit of the pass); then, unless
// the pass is split, source o's replies (the same stream: after the homes' codes).
static int node_owner_one(TbNode* N, u32 o, void* ctx) {
    const NodeCommitJob& J = *(const NodeCommitJob*)ctx;
    const u32 W = N->world;
    const u32 cert = J.cert;
    const auto& nh = J.RT->nh;
    {
        NodeDev& D = N->D[o];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        NodeLegArgs L{};
        L.world = W;
        L.cert64 = cert == TBGPU_CERT_U64 ? 1u : 0u;
        u64 legs_max = 0;
        for (u32 h = 0; h < W; h++) {
            if (h != o) NCK(hipStreamWaitEvent(E->stream, N->D[h].ev_committed, 0));
            L.legs[h] = N->D[h].legs + (u64)o * 2 * nh[h] * NODE_LEG_WORDS;
            L.region[h] = 2 * nh[h];
            L.counts[h] = N->D[h].leg_counts + o;
            legs_max += 2 * nh[h];
        }
        if (legs_max) {
            // A chunk of NAL_CHUNK legs per workgroup at twice the mean load (grid-stride past it).
            const u32 grid = (u32)std::min<u64>(4096, std::max<u64>(1, (2 * legs_max / W + NAL_CHUNK - 1) / NAL_CHUNK));
            hipLaunchKernelGGL(tb_node_apply_legs, dim3(grid), dim3(256), 0, E->stream, E->T, L);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_applied, E->stream));
    }
    if (!J.replies) return TBGPU_STATUS_OK;
    NodeReplyJob RJ{J.P, J.p, J.RT, nullptr};
    return node_reply_one(N, o, &RJ);
}

// Gather, routed commit with owner legs, legs to owners, replies to sources — every device, enqueued.
// replies = false (a split pass): the sources' replies wait for the sequencer (node_issue_replies).
static int node_issue_commit(TbNode* N, NodePass& P, u32 p, const NodePlan& PL, u32 cert, u64 ts_max,
                             bool replies = true) {
    NodeTimer timer(N, 2);
    const u32 W = N->world;
    NodeRoute RT;
    node_route(N, PL, RT);
    const auto& nh = RT.nh;
    for (u32 h = 0; h < W; h++) {
        if (nh[h] > N->recv_cap) return fail(TBGPU_STATUS_INVALID, "node: home %u receives %llu events > %llu", h,
                                             (unsigned long long)nh[h], (unsigned long long)N->recv_cap);
        if (N->D[h].E->log_next + nh[h] > N->D[h].E->xlog_cap) {
            return fail(TBGPU_STATUS_INVALID, "node: transfer log of shard %u full (%llu + %llu > %llu)", h,
                        (unsigned long long)N->D[h].E->log_next, (unsigned long long)nh[h],
                        (unsigned long long)N->D[h].E->xlog_cap);
        }
    }
    NodeCommitJob J{&P, p, &RT, cert, ts_max, replies};
    int st = node_run(N, node_home_one, &J);
    if (st) return st;
    // Every home's commit event is recorded: the owners may wait on them.
    st = node_run(N, node_owner_one, &J);
    if (st) return st;
    P.issued = true;
    return TBGPU_STATUS_OK;
}

// 3. Sources: replies from the codes their homes wrote (and, for a split pass, the sequencer's codes
// of the events it committed: seq_codes, the whole pass block-major), into the reply arena.
static int node_reply_one(TbNode* N, u32 s, void* ctx) {
    const NodeReplyJob& J = *(const NodeReplyJob*)ctx;
    const NodePass& P = *J.P;
    const NodeRoute& RT = *J.RT;
    const u8* seq_codes = J.seq_codes;
    const u32 W = N->world, par = J.p & 1, tri = J.p % 3;
    u64 base = 0;  // the pass's events of the sources before s (seq_codes is the whole pass, block-major)
    for (u32 d = 0; d < s; d++) base += P.blk[d].events;
    {
        NodeDev& D = N->D[s];
        tbgpu* E = D.E;
        const u32 nb = P.blk[s].k1 - P.blk[s].k0;
        NCK(hipSetDevice(D.device));
        if (nb) {
            NodeReplyArgs A{};
            for (u32 h = 0; h < W; h++) {
                A.codes[h] = N->D[h].codes;
                A.delta[h] = (i64)RT.R[h][s] - (i64)RT.off[s][h];
            }
            A.seq = seq_codes ? seq_codes + base : nullptr;
            hipLaunchKernelGGL(tb_node_replies, dim3(nb), dim3(1024), 0, E->stream, D.meta[par], D.home[par], D.slot[par], A,
                               D.results, D.reply_bytes);
            NCK(hipGetLastError());
        }
        // Every shard's arena, with or without a block: its head carries the shard's panic word after
        // its whole part of the pass (home commit, owner legs, replies: one stream), so consuming the
        // pass reads every shard's verdict and the call needs no drain at its end.
        // One workgroup (a block of at most one prepare): it flags its arena for the host to spin on.
        D.reply_seq[tri] = nb <= 1 ? node_next_seq(D) : 0;
        hipLaunchKernelGGL(tb_reply_out, dim3(std::max<u32>(nb, 1)), dim3(64), 0, E->stream, D.meta[par], nb,
                           D.reply_bytes, D.results, E->g, D.d_arena[tri], D.d_flags + 2 + tri, D.reply_seq[tri]);
        NCK(hipGetLastError());
        // After tb_reply_out too: it reads this parity's prepare offsets, which the route stream
        // rewrites two passes on once it has waited for this event.
        NCK(hipEventRecord(D.ev_replied, E->stream));
        NCK(hipEventRecord(D.ev_done[tri], E->stream));
    }
    return TBGPU_STATUS_OK;
}

static int node_issue_replies(TbNode* N, NodePass& P, u32 p, const NodeRoute& RT, const u8* seq_codes) {
    NodeTimer timer(N, 3);
    NodeReplyJob J{&P, p, &RT, seq_codes};
    const int st = node_run(N, node_reply_one, &J);
    if (st) return st;
    P.issued = true;
    return TBGPU_STATUS_OK;
}

// Replies of an issued pass into the caller's buffers.
static int node_consume(TbNode* N, NodePass& P, u32 p, void* const* outputs, u32* out_lens, double* latency_ms, bool take) {
    const u32 tri = p % 3;
    int status = TBGPU_STATUS_OK;
    for (u32 s = 0; s < N->world; s++) {
        NodeDev& D = N->D[s];
        const NodeBlock& B = P.blk[s];
        const u32 nb = B.k1 - B.k0;
        NCK(hipSetDevice(D.device));
        {
            NodeTimer timer(N, 4);
            // The arena's flag when it has one (and no device-clock latency is asked for).
            const bool spun = D.reply_seq[tri] && !(latency_ms && nb) && node_spin(D.h_flags + 2 + tri, D.reply_seq[tri]);
            if (!spun) NCK(hipEventSynchronize(D.ev_done[tri]));
        }
        if (!take || status) continue;
        const u64* head = (const u64*)D.h_arena[tri];
        const u32* rb = (const u32*)(D.h_arena[tri] + 16);
        const u8* res = D.h_arena[tri] + 16 + (u64)nb * 4;
        float ms = 0;
        if (latency_ms && nb) NCK(hipEventElapsedTime(&ms, D.ev_start[tri], D.ev_done[tri]));
        for (u32 k = B.k0; k < B.k1; k++) {
            const u32 bytes = rb[k - B.k0];
            if (bytes) memcpy(outputs[k], res + 8 * P.off[s][k - B.k0], bytes);
            out_lens[k] = bytes;
            if (latency_ms) latency_ms[k] = ms;
        }
        N->commit_ts = std::max(N->commit_ts, head[1]);
        if (head[0]) D.E->poisoned = true;
        if (head[0]) status = fail(TBGPU_STATUS_PANIC, "device panic 0x%llx on shard %u (the reference would have trapped)",
                                   (unsigned long long)head[0], s);
    }
    P.consumed = true;
    return status;
}

// A dirty pass, SPLIT (k_node.h): the dependent subsequence is committed in order by the sequencer,
// every other event is routed to its home as in a clean pass.  Enqueued, nothing drained: the
// sequencer runs on its own stream beside the routed part, on the pass's sequenced events only
// (compacted, each with its execute timestamp), loaded with the state from before the pass (every
// shard's stream is marked before the routed part is issued), and writes its results back as deltas
// (balances) and into log room reserved per home; the replies wait for it.  all: no overflow
// certificate — every event goes to the sequencer.  One host round trip: the plan (the routed part's
// counts, the sequenced events per home), as in a clean pass.
// plan_next() issues the next pass's route plan; it is called once this pass's classification is
// enqueued on the route streams, so the plan queues BEHIND it: the plan waits for the replies of
// the pass two back (its buffers' previous users), which for a split pass wait for that pass's
// sequencer, and a classification queued behind it would wait too — serialising the sequencer of
// pass p with the classification of pass p + 1 (C3 on 2 logical shards: 4.45 ms a pass).
template <class PlanNext>
static int node_split_pass(TbNode* N, NodePass& P, u32 p, const u64* ts, u64 bound_lo, u64 bound_hi, bool all,
                           PlanNext plan_next) {
    const u32 W = N->world, par = p & 1;
    tbgpu* X = N->X;
    auto route_args = [&](NodeDev& D, const NodeBlock& B) {
        RouteArgs A{};
        A.events = D.ev[par];
        A.n = (u32)B.events;
        A.nb = B.k1 - B.k0;
        A.batch_off = D.meta[par];
        A.batch_ts = D.meta[par] + A.nb + 1;
        A.world = W;
        A.T = D.E->T;
        A.limbits = D.limbits;
        A.limmask = D.limmask;
        A.limit_any = N->limit_any ? 1u : 0u;
        return A;
    };
    // -- 1. classification on every source: primary classes, then the events on balancing-marked
    //       accounts, then the key set, the final mask and the route plan of the rest.
    for (u32 d = 0; d < W; d++) {
        NodeDev& D = N->D[d];
        const NodeBlock& B = P.blk[d];
        NCK(hipSetDevice(D.device));
        NCK(hipMemsetAsync(D.dcounts, 0, NODE_DC_WORDS * 8, D.rs));
        if (B.events) {
            const RouteArgs A = route_args(D, B);
            NodeDepArgs Dp{D.dep1, D.dep[par], D.dkeys, D.dbal, D.dcounts, all ? 1u : 0u};
            hipLaunchKernelGGL(tb_node_classify1, dim3((unsigned)((B.events + ROUTE_THREADS - 1) / ROUTE_THREADS)),
                               dim3(ROUTE_THREADS), 0, D.rs, A, Dp);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_cls, D.rs));
    }
    NodeSetArgs S{};
    S.world = W;
    for (u32 d = 0; d < W; d++) {
        S.keys[d] = N->D[d].dkeys;
        S.bal[d] = N->D[d].dbal;
        S.counts[d] = N->D[d].dcounts;
    }
    // Events on a balancing-marked account become primary-dependent (their ids join the key lists),
    // once every source's balancing accounts are known: every sequenced event's id is then a key, so
    // no routed event creates an id a sequenced event reads.
    for (u32 d = 0; d < W; d++) {
        NodeDev& D = N->D[d];
        const NodeBlock& B = P.blk[d];
        NCK(hipSetDevice(D.device));
        for (u32 s = 0; s < W; s++) NCK(hipStreamWaitEvent(D.rs, N->D[s].ev_cls, 0));
        NCK(hipMemsetAsync(D.markset, 0, (D.set_mask + 1) * 8, D.rs));
        NodeSetArgs Sd = S;
        Sd.markset = D.markset;
        Sd.markset_mask = D.set_mask;
        hipLaunchKernelGGL(tb_node_sets, dim3(512), dim3(256), 0, D.rs, Sd);
        if (B.events) {
            const RouteArgs A = route_args(D, B);
            NodeDepArgs Dp{D.dep1, D.dep[par], D.dkeys, D.dbal, D.dcounts, all ? 1u : 0u};
            hipLaunchKernelGGL(tb_node_classify_marked, dim3((unsigned)((B.events + ROUTE_THREADS - 1) / ROUTE_THREADS)),
                               dim3(ROUTE_THREADS), 0, D.rs, A, Dp, D.markset, D.set_mask);
        }
        NCK(hipGetLastError());
        NCK(hipEventRecord(D.ev_marked, D.rs));
    }
    for (u32 d = 0; d < W; d++) {
        NodeDev& D = N->D[d];
        const NodeBlock& B = P.blk[d];
        NCK(hipSetDevice(D.device));
        for (u32 s = 0; s < W; s++) NCK(hipStreamWaitEvent(D.rs, N->D[s].ev_marked, 0));
        NCK(hipMemsetAsync(D.keyset, 0, (D.set_mask + 1) * 8, D.rs));
        NodeSetArgs Sd = S;
        Sd.keyset = D.keyset;
        Sd.keyset_mask = D.set_mask;
        hipLaunchKernelGGL(tb_node_sets, dim3(512), dim3(256), 0, D.rs, Sd);
        NCK(hipGetLastError());
        NCK(hipMemsetAsync(D.words[par], 0, ROUTE_WORDS * 8, D.rs));
        if (B.events) {
            RouteArgs A = route_args(D, B);
            A.nblocks = (u32)((B.events + ROUTE_THREADS - 1) / ROUTE_THREADS);
            A.home = D.home[par];
            A.block_counts = D.block_counts;
            A.block_base = D.block_counts + (u64)A.nblocks * W;
            A.words = D.words[par];
            NodeDepArgs Dp{D.dep1, D.dep[par], D.dkeys, D.dbal, D.dcounts, all ? 1u : 0u};
            hipLaunchKernelGGL(tb_node_classify2, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A, Dp, D.keyset, D.set_mask);
            A.skip = D.dep[par];
            hipLaunchKernelGGL(tb_route_classify, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A);
            hipLaunchKernelGGL(tb_route_offsets, dim3(A.world), dim3(1024), 0, D.rs, A);
            hipLaunchKernelGGL(tb_route_scatter, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A, D.send[par], D.slot[par]);
            NCK(hipGetLastError());
        }
        D.plan_seq[par] = node_next_seq(D);
        hipLaunchKernelGGL(tb_route_publish, dim3(1), dim3(64), 0, D.rs, D.words[par], D.d_words_host[par], D.d_flags + par,
                           D.plan_seq[par]);
        NCK(hipGetLastError());
        NCK(hipMemcpyAsync(D.h_dcounts, D.dcounts, NODE_DC_WORDS * 8, hipMemcpyDeviceToHost, D.rs));
        NCK(hipEventRecord(D.ev_planned[par], D.rs));
    }
    int st = plan_next();
    if (st) return st;
    NodePlan PL;
    if ((st = node_read_plan(N, P, p, &PL, false))) return st;
    u64 n_seq = 0, n_pass = 0, room[NODE_WORLD_MAX] = {};
    for (u32 d = 0; d < W; d++) {
        // A source with an empty block (the call's last pass) sequences nothing; its counts' copy is
        // not waited for (node_read_plan waits for the sources with events), so its host words may
        // still hold an earlier pass's counts: reading them reserved too little log room on the
        // homes and sized the sequencer's pass wrong (8-shard C3 / C4, tests/test_gpu_node.py).
        if (P.blk[d].k1 == P.blk[d].k0) continue;
        n_seq += N->D[d].h_dcounts[2];
        n_pass += P.blk[d].events;
        for (u32 h = 0; h < W; h++) room[h] += N->D[d].h_dcounts[NODE_DC_HOME + h];
    }
    // -- 2. the routed part, committed by the homes (legs to the owners); its certificate covers the
    //       whole pass's amounts.  First every shard's stream is marked: the sequencer's loads see the
    //       state before the pass (every earlier pass applied), not the routed part, which touches no
    //       id, pending transfer or constrained balance a sequenced event reads.
    typedef unsigned __int128 h128;
    const h128 bound = ((h128)bound_hi << 64) | bound_lo;
    const h128 total = bound + PL.S < bound ? ~(h128)0 : bound + PL.S;
    const u32 cert = (total >> 64) == 0 ? TBGPU_CERT_U64 : TBGPU_CERT_U128;
    for (u32 d = 0; d < W; d++) {
        NCK(hipSetDevice(N->D[d].device));
        NCK(hipEventRecord(N->D[d].ev_pre, N->D[d].E->stream));
    }
    if (!all && (st = node_issue_commit(N, P, p, PL, cert, ts[P.k1 - 1], false))) return st;
    // Log room on every home for the transfers the sequencer may create there (one per sequenced
    // event homed there), after the routed part's.
    u64 wb_base[NODE_WORLD_MAX];
    for (u32 h = 0; h < W; h++) {
        tbgpu* E = N->D[h].E;
        if (E->log_next + room[h] > E->xlog_cap) {
            return fail(TBGPU_STATUS_INVALID, "node: transfer log of shard %u full", h);
        }
        wb_base[h] = E->log_next;
        E->log_next += room[h];
    }
    // -- 3. the sequencer (its own stream, beside the routed part): the pass's sequenced events
    //       compacted, loaded with what they read, committed in order.
    const int dev0 = N->D[0].device;
    NCK(hipSetDevice(dev0));
    hipStream_t xs = X->stream;
    for (u32 d = 0; d < W; d++) {
        NCK(hipStreamWaitEvent(xs, N->D[d].ev_pre, 0));
        NCK(hipStreamWaitEvent(xs, N->D[d].ev_planned[par], 0));  // the classification
    }
    if (!N->x_index_clean) {  // an earlier split pass ended before its clear (tb_seq_xidx_zero)
        NCK(hipMemsetAsync(X->T.xidx, 0, X->xidx_cap * 8, xs));
        NCK(hipMemsetAsync(X->T.xdup, 0, X->xidx_cap, xs));
        NCK(hipMemsetAsync(X->T.xposted, 0, X->xlog_cap, xs));
    }
    N->x_index_clean = false;
    NCK(hipMemsetAsync(N->seq_counts, 0, 8 * 8, xs));
    NCK(hipMemsetAsync(&X->g->commit_timestamp, 0, 8, xs));
    SeqSet tset{N->tset_e, N->tset_mask, N->tset_list, N->seq_counts, N->tset_dups};
    SeqSet aset{N->aset_e, N->aset_mask, N->aset_list, N->seq_counts + 2, N->aset_dups};
    const u32 nb = P.k1 - P.k0;
    SeqCompactArgs C{};
    C.world = W;
    {
        u64 at = 0;
        u32 pk = 0;
        for (u32 d = 0; d < W; d++) {
            C.src[d] = N->D[d].ev[par];
            C.dep[d] = N->D[d].dep[par];
            C.meta[d] = N->D[d].meta[par];
            C.nb[d] = P.blk[d].k1 - P.blk[d].k0;
            C.start[d] = at;
            C.pstart[d] = pk;
            at += P.blk[d].events;
            pk += C.nb[d];
        }
        C.start[W] = at;
        C.pstart[W] = pk;
    }
    C.nblk = (u32)((n_pass + 255) / 256);
    C.blk = N->seq_blk;
    C.out = X->staging;
    C.out_ts = N->seq_ts;
    C.map = N->seq_map;
    C.xmeta = X->meta;
    NodeTablesArgs NT{};
    NT.world = W;
    for (u32 d = 0; d < W; d++) NT.T[d] = N->D[d].E->T;
    if (n_pass) {
        hipLaunchKernelGGL(tb_seq_count, dim3(C.nblk), dim3(256), 0, xs, C);
        hipLaunchKernelGGL(tb_seq_scan, dim3(1), dim3(1024), 0, xs, C);
        hipLaunchKernelGGL(tb_seq_compact, dim3(C.nblk), dim3(256), 0, xs, C, tset);
        hipLaunchKernelGGL(tb_seq_meta, dim3((nb + 256) / 256), dim3(256), 0, xs, C);
        NCK(hipGetLastError());
    }
    NCK(hipEventRecord(N->ev_xread, xs));  // the sources' buffers of this pass may be reused
    if (n_seq) {
        hipLaunchKernelGGL(tb_seq_load_transfers, dim3(1024), dim3(256), 0, xs, NT, tset, X->T, N->seq_counts + 4, aset);
        hipLaunchKernelGGL(tb_seq_event_accounts, dim3((unsigned)((n_seq + 255) / 256)), dim3(256), 0, xs, X->staging,
                           n_seq, aset);
        hipLaunchKernelGGL(tb_seq_verify, dim3(256), dim3(256), 0, xs, tset, (u64*)&X->g->panic);
        hipLaunchKernelGGL(tb_seq_verify, dim3(256), dim3(256), 0, xs, aset, (u64*)&X->g->panic);
        hipLaunchKernelGGL(tb_seq_load_accounts, dim3(1024), dim3(256), 0, xs, NT, aset, X->T, N->seq_bal0);
        NCK(hipGetLastError());
    }
    // Its balance bound: the node's (its commit timestamp: from its own events, folded below).
    u64* hs = N->h_seq + 8 * (p & 1);  // by pass parity: the previous pass's copy may be in flight
    hs[0] = bound_lo;
    hs[1] = bound_hi;
    NCK(hipMemcpyAsync(&X->g->bound_lo, hs, 16, hipMemcpyHostToDevice, xs));
    X->commit_ts = 0;
    X->last_batch_ts = 0;
    X->log_next = N->seq_tcap;
    // One pass of the compacted prepares (nb of them, offsets on the device from tb_seq_meta; the
    // host needs only the total).
    u64* h_off = X->h_meta;
    for (u32 k = 0; k < nb; k++) h_off[k] = 0;
    h_off[nb] = n_seq;
    if (n_seq && (st = enqueue_call(X, OP_CREATE_TRANSFERS, nb, h_off, X->staging, X->results, X->reply_bytes, false,
                                    N->seq_xcodes, 0, nullptr, X->meta, nullptr, nullptr, nullptr, N->seq_ts))) {
        return st;
    }
    if (n_pass) {
        hipLaunchKernelGGL(tb_seq_expand, dim3(1024), dim3(256), 0, xs, C, N->seq_xcodes, N->seq_codes);
        NCK(hipGetLastError());
    }
    NCK(hipEventRecord(N->ev_x, xs));
    // -- 4. write-back on every shard's stream once the sequencer is done: its new transfers and
    //       posted states to their homes (into the room reserved above), its balance deltas to the
    //       owners; the first shard folds in its panic bits, timestamp and bound growth.
    for (u32 d = 0; d < W; d++) {
        NodeDev& D = N->D[d];
        NCK(hipSetDevice(D.device));
        NCK(hipStreamWaitEvent(D.E->stream, N->ev_x, 0));
        if (n_seq) {
            NCK(hipMemsetAsync(D.wb_count, 0, 8, D.E->stream));
            hipLaunchKernelGGL(tb_seq_writeback_transfers, dim3(1024), dim3(256), 0, D.E->stream, X->T, N->seq_tcap, n_seq,
                               tset, D.E->T, d, W, wb_base[d], D.wb_count);
            hipLaunchKernelGGL(tb_seq_writeback_accounts, dim3(1024), dim3(256), 0, D.E->stream, X->T, aset, D.E->T, d, W,
                               (const AccountBal*)N->seq_bal0);
            NCK(hipGetLastError());
        }
        if (d == 0) {
            hipLaunchKernelGGL(tb_seq_fold, dim3(1), dim3(64), 0, D.E->stream, (const Globals*)X->g, D.E->g, bound_lo, bound_hi);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_xwb, D.E->stream));
    }
    // -- 5. replies (the homes' codes and the sequencer's), then the sequencer's tables empty once
    //       every shard has written back.
    NodeRoute RT;
    node_route(N, PL, RT);
    if ((st = node_issue_replies(N, P, p, RT, N->seq_codes))) return st;
    NCK(hipSetDevice(dev0));
    for (u32 d = 0; d < W; d++) NCK(hipStreamWaitEvent(xs, N->D[d].ev_xwb, 0));
    hipLaunchKernelGGL(tb_seq_clear, dim3(1024), dim3(256), 0, xs, tset, aset, X->T);
    NCK(hipGetLastError());
    // The sequencer's transfer index, entry by entry (its claims; the next split pass needs it empty).
    NCK(hipMemsetAsync(N->xclr_count, 0, 8, xs));
    hipLaunchKernelGGL(tb_seq_xidx_list, dim3(1024), dim3(256), 0, xs, X->T, (const u64*)(N->seq_counts + 4), X->staging,
                       N->seq_tcap, n_seq, N->xclr_list, N->xclr_count, N->xclr_cap);
    hipLaunchKernelGGL(tb_seq_xidx_zero, dim3(1024), dim3(256), 0, xs, X->T, N->xclr_list, N->xclr_count,
                       (const u64*)(N->seq_counts + 4), N->seq_tcap, n_seq, N->xclr_cap);
    NCK(hipGetLastError());
    N->x_index_clean = true;
    if (all) N->passes_whole++;
    else N->passes_split++;
    N->seq_events += n_seq;
    return TBGPU_STATUS_OK;
}

// The node's commit of n create_transfers prepares from host memory.
static int node_commit_transfers(TbNode* N, u32 n, const u64* ts, const void* const* inputs, const u32* lens,
                                 void* const* outputs, u32* out_lens, u32 chunk, double* latency_ms) {
    NodeTimer timer(N, 5);
    N->t_calls++;
    N->latency_on = latency_ms != nullptr;
    typedef unsigned __int128 h128;
    const u32 W = N->world;
    const u32 per = std::max<u32>(1, std::min<u32>(chunk ? chunk : N->pb_src, N->pb_src));
    // Passes: W blocks of up to `per` prepares and pe_src events each, in prepare order, built in a
    // ring as they are planned.  Every prepare fits a block (checked before anything runs).
    for (u32 k = 0; k < n; k++) {
        if (lens[k] > N->pe_src) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
    }
    auto build = [&](u32 p, u32 k) -> NodePass& {
        NodePass& P = N->ring[p % NODE_PASS_RING];
        P.k0 = k;
        P.issued = P.consumed = false;
        for (u32 d = 0; d < W; d++) {
            NodeBlock& B = P.blk[d];
            B.k0 = B.k1 = k;
            B.events = 0;
            P.off[d][0] = 0;
            while (k < n && B.k1 - B.k0 < per && B.events + lens[k] <= N->pe_src) {
                B.events += lens[k];
                P.off[d][B.k1 - B.k0 + 1] = B.events;
                k++;
                B.k1 = k;
            }
        }
        P.k1 = k;
        return P;
    };
    // Drain the shards and read their bounds back — unless the previous call on this handle was a
    // create_transfers call that ended with nothing in flight and nothing ran since: its bound (the
    // host-tracked sum, conservative) still holds.
    const bool drained = N->api_calls && *N->api_calls == N->drained_at + 1;
    h128 bound = N->bound_carry;
    if (!drained) {
        const int st0 = node_sync(N);
        if (st0) return st0;
        bound = node_bound(N);
    }
    int status = TBGPU_STATUS_OK;
    u32 NP = 1;  // passes built so far (the last one planned)
    u32 next_consume = 0;
    auto pass = [&](u32 p) -> NodePass& { return N->ring[p % NODE_PASS_RING]; };
    auto consume_upto = [&](u32 end) {  // consume every issued pass < end
        for (; next_consume < end; next_consume++) {
            NodePass& P = pass(next_consume);
            if (P.issued && !P.consumed) {
                const int c = node_consume(N, P, next_consume, outputs, out_lens, latency_ms, status == TBGPU_STATUS_OK);
                if (status == TBGPU_STATUS_OK) status = c;
            }
        }
    };
    {
        NodePass& P0 = build(0, 0);
        if ((status = node_issue_plan(N, P0, 0, ts, inputs, lens, P0.k1 >= n))) return status;
    }
    for (u32 p = 0; p < NP && status == TBGPU_STATUS_OK; p++) {
        if (p >= 2) consume_upto(p - 1);  // pass p-2: its arena slot, start event and meta are reused next
        if (status) break;
        NodePass& Pp = pass(p);
        NodePlan PL;
        if ((status = node_read_plan(N, Pp, p, &PL))) break;
        // The next pass's plan, issued once this pass's work on the route streams (a split pass's
        // classification) is queued ahead of it.
        auto plan_next = [&]() -> int {
            if (pass(p).k1 >= n) return TBGPU_STATUS_OK;
            NP = p + 2;  // its ring slot held pass p - 3, consumed above
            return node_issue_plan(N, build(p + 1, pass(p).k1), p + 1, ts, inputs, lens, false);
        };
        const h128 total = bound + PL.S < bound ? ~(h128)0 : bound + PL.S;
        if (PL.dirty || PL.huge || total == ~(h128)0) {
            // Split: issued like a clean pass, nothing drained (node_split_pass).  Without the overflow
            // certificate every event is sequenced, and the shards' bounds are read back after it.
            const bool all = PL.huge || total == ~(h128)0;
            if ((status = node_split_pass(N, Pp, p, ts, (u64)bound, (u64)(bound >> 64), all, plan_next))) break;
            if (!all) {
                bound = total;
                continue;
            }
            consume_upto(p + 1);
            if (status) break;
            if ((status = node_sync(N))) break;
            bound = node_bound(N);
            continue;
        }
        if ((status = plan_next())) break;
        const u32 cert = (total >> 64) == 0 ? TBGPU_CERT_U64 : TBGPU_CERT_U128;
        if ((status = node_issue_commit(N, Pp, p, PL, cert, ts[Pp.k1 - 1]))) break;
        bound = total;
        N->passes_clean++;
    }
    consume_upto(NP);
    // Every pass consumed = every shard's stream past its last reply arena (node_issue_replies), every
    // plan read: nothing is in flight and every shard's panic word was read.  The end-of-call drain
    // stays only after a failure (plans issued ahead) or to collect profiling events.
    bool profiling = false;
    for (u32 d = 0; d < W; d++) profiling |= N->D[d].E->profile;
    if (status != TBGPU_STATUS_OK || profiling) {
        const int s2 = node_sync(N);
        if (status == TBGPU_STATUS_OK) status = s2;
    }
    const int s3 = node_publish_commit_ts(N);
    if (status == TBGPU_STATUS_OK && s3 == TBGPU_STATUS_OK && N->api_calls) {
        N->drained_at = *N->api_calls;
        N->bound_carry = bound;
    }
    return status ? status : s3;
}

// A device panic on any shard stops the node (tbgpu.h: until tbgpu_reset).
static int node_poisoned(TbNode* N) {
    for (u32 d = 0; d < N->world; d++) {
        if (N->D[d].E->poisoned) {
            return fail(TBGPU_STATUS_PANIC, "node stopped by an earlier device panic on shard %u (tbgpu_reset or tbgpu_deinit it)", d);
        }
    }
    return TBGPU_STATUS_OK;
}

static int node_commit_pipelined(TbNode* N, u8 op, u32 n, const u64* ts, const void* const* inputs, const u32* input_lens,
                                 void* const* outputs, u32* out_lens, u32 chunk, double* latency_ms) {
    if (const int st = node_poisoned(N)) return st;
    if (op != OP_CREATE_ACCOUNTS && op != OP_CREATE_TRANSFERS) {
        return fail(TBGPU_STATUS_INVALID, "operation %u is not a create operation", op);
    }
    std::vector<u32> lens(n);
    u64 prev = N->commit_ts;
    for (u32 k = 0; k < n; k++) {  // the commit asserts of every prepare (state_machine.zig:518-519, :645)
        if (input_lens[k] % 128 != 0) return fail(TBGPU_STATUS_INVALID, "create body not a multiple of 128");
        const u32 L = input_lens[k] / 128;
        if (L > BATCH_EVENTS_MAX) return fail(TBGPU_STATUS_INVALID, "batch %u has %u events (max %u)", k, L, BATCH_EVENTS_MAX);
        if (!(ts[k] > prev)) return fail(TBGPU_STATUS_PANIC, "timestamp %llu <= commit timestamp %llu",
                                         (unsigned long long)ts[k], (unsigned long long)prev);
        if (L > 0) {
            if (ts[k] < L) return fail(TBGPU_STATUS_PANIC, "timestamp %llu < batch length %u", (unsigned long long)ts[k], L);
            if (!(ts[k] - L + 1 > prev)) return fail(TBGPU_STATUS_PANIC, "first event timestamp <= commit timestamp");
        }
        prev = ts[k];
        lens[k] = L;
        out_lens[k] = 0;
    }
    if (op == OP_CREATE_ACCOUNTS) {
        const int st = node_commit_accounts(N, n, ts, inputs, lens.data(), outputs, out_lens);
        const int s2 = node_publish_commit_ts(N);
        return st ? st : s2;
    }
    return node_commit_transfers(N, n, ts, inputs, lens.data(), outputs, out_lens, chunk, latency_ms);
}

// -- lookups, exports, write-back, test setup ------------------------------------------------------

// Every account, from its owner (the only copy), in id order.
static int node_export_accounts(TbNode* N, std::vector<u8>& out) {
    out.clear();
    if (const int st = node_imports_flush(N)) return st;  // each table read whole: its own accounts only
    for (u32 d = 0; d < N->world; d++) {
        if (hipSetDevice(N->D[d].device) != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "hipSetDevice");
        std::vector<u8> r;
        const int st = export_records<true>(N->D[d].E, r, nullptr);
        if (st) return st;
        const u64 m = r.size() / 128;
        for (u64 i = 0; i < m; i++) {
            if (node_home(&r[i * 128], N->world) != d) return fail(TBGPU_STATUS_PANIC, "node: shard %u holds a foreign account", d);
        }
        out.insert(out.end(), r.begin(), r.end());
    }
    const u64 n = out.size() / 128;
    std::vector<u64> idx(n);
    for (u64 i = 0; i < n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](u64 a, u64 b) { return id_less(&out[a * 128], &out[b * 128]); });
    std::vector<u8> sorted(out.size());
    for (u64 i = 0; i < n; i++) memcpy(&sorted[i * 128], &out[idx[i] * 128], 128);
    out.swap(sorted);
    return TBGPU_STATUS_OK;
}

static int node_export_transfers(TbNode* N, std::vector<u8>& out, std::vector<u64>* posted) {
    out.clear();
    for (u32 d = 0; d < N->world; d++) {
        if (hipSetDevice(N->D[d].device) != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "hipSetDevice");
        std::vector<u8> r;
        const int st = export_records<false>(N->D[d].E, r, posted);
        if (st) return st;
        out.insert(out.end(), r.begin(), r.end());
    }
    const u64 n = out.size() / 128;
    std::vector<u64> idx(n);
    for (u64 i = 0; i < n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](u64 a, u64 b) { return id_less(&out[a * 128], &out[b * 128]); });
    std::vector<u8> sorted(out.size());
    for (u64 i = 0; i < n; i++) memcpy(&sorted[i * 128], &out[idx[i] * 128], 128);
    out.swap(sorted);
    return TBGPU_STATUS_OK;
}

// Records by id from their owners (accounts) or homes (transfers), in input order.
static int node_fetch(TbNode* N, bool accounts, const u64* ids, u32 n, u8* out, u8* found) {
    std::vector<std::vector<u64>> part(N->world);
    std::vector<std::vector<u32>> where(N->world);
    for (u32 i = 0; i < n; i++) {
        const u32 o = tb_home(ids[2 * i], ids[2 * i + 1], N->world);
        part[o].push_back(ids[2 * i]);
        part[o].push_back(ids[2 * i + 1]);
        where[o].push_back(i);
    }
    for (u32 o = 0; o < N->world; o++) {
        const u32 m = (u32)where[o].size();
        if (!m) continue;
        std::vector<u8> r((u64)m * 128), f(m);
        const int st = accounts ? tbgpu_fetch_accounts(N->D[o].E, part[o].data(), m, r.data(), f.data())
                                : tbgpu_fetch_transfers(N->D[o].E, part[o].data(), m, r.data(), f.data());
        if (st) return st;
        for (u32 j = 0; j < m; j++) {
            memcpy(out + (u64)where[o][j] * 128, &r[(u64)j * 128], 128);
            found[where[o][j]] = f[j];
        }
    }
    return TBGPU_STATUS_OK;
}

static int node_lookup(TbNode* N, bool accounts, const void* input, u32 input_len, void* output, u32 output_cap,
                       u32* out_len) {
    if (input_len % 16 != 0) return fail(TBGPU_STATUS_INVALID, "lookup body not a multiple of 16");
    const u32 n = input_len / 16;
    std::vector<u64> ids(2 * (u64)n);
    if (n) memcpy(ids.data(), input, (u64)n * 16);
    std::vector<u8> recs((u64)n * 128), found(n);
    const int st = node_fetch(N, accounts, ids.data(), n, recs.data(), found.data());
    if (st) return st;
    const u32 slots = output_cap / 128;
    u32 m = 0;
    for (u32 i = 0; i < n; i++) {
        if (found[i] && m < slots) {
            memcpy((u8*)output + (u64)m * 128, &recs[(u64)i * 128], 128);
            m++;
        }
    }
    *out_len = m * 128;
    return TBGPU_STATUS_OK;
}

// -- the tbgpu.h entry points of a node engine --------------------------------------------------------

static int node_api_init(const tbgpu_config* config, tbgpu_t** out) {
    TbNode* N = nullptr;
    const int st = node_init(config, &N);
    if (st) return st;
    tbgpu* E = new tbgpu();
    E->cfg = *config;
    E->node = N;
    N->api_calls = &E->api_calls;
    E->device = N->D[0].device;
    *out = E;
    return TBGPU_STATUS_OK;
}

static int node_api_reset(TbNode* N) {
    for (u32 d = 0; d < N->world; d++) {
        const int st = tbgpu_reset(N->D[d].E);
        if (st) return st;
        NCK(hipSetDevice(N->D[d].device));
        NCK(hipMemset(N->D[d].imp_count, 0, 8));  // (the tables are empty again)
    }
    N->commit_ts = 0;
    return TBGPU_STATUS_OK;
}

static int node_api_commit(TbNode* N, u8 op, u64 timestamp, const void* input, u32 input_len, void* output,
                           u32 output_cap, u32* out_len) {
    *out_len = 0;
    if (const int st = node_poisoned(N)) return st;
    if (op < OP_CREATE_ACCOUNTS || op > OP_LOOKUP_TRANSFERS) return fail(TBGPU_STATUS_INVALID, "unknown operation %u", op);
    if (!(timestamp > N->commit_ts)) {  // state_machine.zig:519
        return fail(TBGPU_STATUS_PANIC, "timestamp %llu <= commit timestamp %llu", (unsigned long long)timestamp,
                    (unsigned long long)N->commit_ts);
    }
    if (op == OP_LOOKUP_ACCOUNTS || op == OP_LOOKUP_TRANSFERS) {
        return node_lookup(N, op == OP_LOOKUP_ACCOUNTS, input, input_len, output, output_cap, out_len);
    }
    if (input_len == 0) return TBGPU_STATUS_OK;
    if (input_len % 128 != 0) return fail(TBGPU_STATUS_INVALID, "create body not a multiple of 128");
    if ((u64)output_cap < (u64)(input_len / 128) * 8) return fail(TBGPU_STATUS_INVALID, "output too small");
    const void* ins[1] = {input};
    void* outs[1] = {output};
    return node_commit_pipelined(N, op, 1, &timestamp, ins, &input_len, outs, out_len, 1, nullptr);
}

// The setup action (state_machine.zig:1398-1407): on the owner, the account's only copy.
static int node_api_set_balances(TbNode* N, u64 id_lo, u64 id_hi, const u64 b[8]) {
    return tbgpu_test_set_balances(N->D[tb_home(id_lo, id_hi, N->world)].E, id_lo, id_hi, b);
}

static int node_api_export(TbNode* N, int what, void* out, u64 cap, u64* count) {
    std::vector<u8> recs;
    std::vector<u64> posted;
    const int st = what == 0 ? node_export_accounts(N, recs) : node_export_transfers(N, recs, what == 2 ? &posted : nullptr);
    if (st) return st;
    if (what < 2) {
        const u64 n = std::min<u64>(recs.size() / 128, cap);
        memcpy(out, recs.data(), n * 128);
        *count = n;
        return TBGPU_STATUS_OK;
    }
    const u64 n = posted.size() / 2;
    std::vector<std::pair<u64, u64>> pairs(n);
    for (u64 i = 0; i < n; i++) pairs[i] = {posted[2 * i], posted[2 * i + 1]};
    std::sort(pairs.begin(), pairs.end());
    const u64 m = std::min<u64>(n, cap);
    u64* o = (u64*)out;
    for (u64 i = 0; i < m; i++) {
        o[2 * i] = pairs[i].first;
        o[2 * i + 1] = pairs[i].second;
    }
    *count = m;
    return TBGPU_STATUS_OK;
}

// Groove write-back of the node, O(changes) like a single engine's (engine.hip wb_*, the same
// preallocated buffers on every shard): the new transfers of every shard's log, merged by timestamp;
// the posted entries their post / void records make (the pending transfer may live on another
// shard: its timestamp is fetched from its home); the accounts the new transfers moved — wherever
// those transfers live — plus the listed creates and direct writes, each looked up on its OWNER,
// whose copy holds its balances (a whole-table diff of a shard keeps only the accounts it owns).
// The caller's buffers are checked up front against the most the write-back can emit.
static int node_api_checkpoint_delta(TbNode* N, void* accounts_out, void* accounts_before_out, u64 accounts_cap,
                                     void* transfers_out, u64 transfers_cap, u64* posted_out, u64 posted_cap,
                                     tbgpu_delta_counts* counts) {
    memset(counts, 0, sizeof(*counts));
    const u32 W = N->world;
    if (N->wb_inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight (tbgpu_checkpoint_delta_wait)");
    int st = node_sync(N);
    if (st) return st;
    WbBounds bd{0, 0, 0};
    u64 listed = 0;
    bool scan = false;
    for (u32 d = 0; d < W; d++) {
        tbgpu* E = N->D[d].E;
        NCK(hipSetDevice(N->D[d].device));
        if (E->wb.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight");
        if ((st = ckpt_snapshot_ready(E))) return st;
        const WbBounds b = wb_bounds(E, E->h_globals->account_count);
        bd.transfers += b.transfers;
        bd.posted += b.posted;
        listed += E->ckpt_ids.size() / 2;
        scan |= E->ckpt_scan;
    }
    bd.accounts = std::min<u64>(N->D[0].E->h_globals->account_count, scan ? ~0ULL : 2 * bd.transfers + listed);
    counts->created_after = N->D[0].E->ckpt_ts;
    if (bd.accounts > accounts_cap || bd.transfers > transfers_cap || bd.posted > posted_cap) {  // nothing moved
        counts->accounts = bd.accounts;
        counts->transfers = bd.transfers;
        counts->posted = bd.posted;
        return fail(TBGPU_STATUS_INVALID, "checkpoint delta: buffers must hold %llu accounts, %llu transfers, %llu posted",
                    (unsigned long long)bd.accounts, (unsigned long long)bd.transfers, (unsigned long long)bd.posted);
    }
    // 1. Every shard's new transfers (records, their account ids, post / void records), slice by slice.
    std::vector<std::vector<u8>> runs(W);
    std::vector<u64> ids_all, pv_all;
    u64 nt = 0;
    for (u32 d = 0; d < W; d++) {
        tbgpu* E = N->D[d].E;
        NCK(hipSetDevice(N->D[d].device));
        if ((st = wb_next_epoch(E))) return st;
        NCK(hipMemsetAsync(E->wb.d_cnt, 0, WB_COUNT_WORDS * 8, E->stream));
        for (u64 a = E->ckpt_pos; a < E->log_next; a += E->wb.cap_t) {
            const u64 b = std::min<u64>(E->log_next, a + E->wb.cap_t);
            if ((st = wb_gather_slice(E, a, b, true, false))) return st;
            if ((st = wb_read_counts(E))) return st;
            const u64 k = E->wb.h_cnt[WB_RECORDS], q = E->wb.h_cnt[WB_PV];
            const size_t r0 = runs[d].size(), i0 = ids_all.size(), p0 = pv_all.size();
            runs[d].resize(r0 + k * 128);
            ids_all.resize(i0 + k * 4);
            pv_all.resize(p0 + q * 3);
            if (k) NCK(hipMemcpyAsync(runs[d].data() + r0, E->wb.d_out, k * 128, hipMemcpyDeviceToHost, E->stream));
            if (k) NCK(hipMemcpyAsync(ids_all.data() + i0, E->wb.d_ids, k * 32, hipMemcpyDeviceToHost, E->stream));
            if (q) NCK(hipMemcpyAsync(pv_all.data() + p0, E->wb.d_pv, q * 24, hipMemcpyDeviceToHost, E->stream));
            NCK(hipStreamSynchronize(E->stream));
        }
        delta_sort_by_timestamp(runs[d].data(), runs[d].size() / 128);
        nt += runs[d].size() / 128;
        ids_all.insert(ids_all.end(), E->ckpt_ids.begin(), E->ckpt_ids.end());
    }
    // 2. The accounts, on their owners: the ids routed there, or the owner's whole-table diff.
    std::vector<std::vector<u64>> owned(W);
    for (size_t i = 0; i + 1 < ids_all.size(); i += 2) {
        const u32 o = tb_home(ids_all[i], ids_all[i + 1], W);
        owned[o].push_back(ids_all[i]);
        owned[o].push_back(ids_all[i + 1]);
    }
    u64 na = 0;
    for (u32 o = 0; o < W; o++) {
        tbgpu* E = N->D[o].E;
        NCK(hipSetDevice(N->D[o].device));
        if ((st = wb_listed_ids(E, owned[o], (u8*)accounts_out, (u8*)accounts_before_out, &na))) return st;
        if ((st = wb_scan(E, W, o, (u8*)accounts_out, (u8*)accounts_before_out, &na))) return st;
    }
    // 3. The posted pairs: each post / void record's pending transfer, from its home.
    const u64 npv = pv_all.size() / 3;
    if (npv) {
        std::vector<u64> ids(2 * npv);
        for (u64 i = 0; i < npv; i++) {
            ids[2 * i] = pv_all[3 * i];
            ids[2 * i + 1] = pv_all[3 * i + 1];
        }
        std::vector<u8> rec(npv * 128), found(npv);
        if ((st = node_fetch(N, false, ids.data(), (u32)npv, rec.data(), found.data()))) return st;
        for (u64 i = 0; i < npv; i++) {
            if (!found[i]) return fail(TBGPU_STATUS_PANIC, "checkpoint delta: a posted pending transfer is missing");
            posted_out[2 * i] = *(const u64*)&rec[i * 128 + 120];
            posted_out[2 * i + 1] = pv_all[3 * i + 2];
        }
        delta_sort_pairs(posted_out, npv);
    }
    // 4. Transfers: each shard's in timestamp order, merged.
    {
        std::vector<size_t> pos(W, 0);
        auto ts_at = [&](u32 d) { return *(const u64*)&runs[d][pos[d] * 128 + 120]; };
        for (u64 k = 0; k < nt; k++) {
            u32 best = W;
            for (u32 d = 0; d < W; d++) {
                if (pos[d] < runs[d].size() / 128 && (best == W || ts_at(d) < ts_at(best))) best = d;
            }
            memcpy((u8*)transfers_out + k * 128, &runs[best][pos[best] * 128], 128);
            pos[best]++;
        }
    }
    // 5. Every shard's snapshot advances.
    for (u32 d = 0; d < W; d++) {
        NCK(hipSetDevice(N->D[d].device));
        if ((st = wb_advance(N->D[d].E))) return st;
        NCK(hipStreamSynchronize(N->D[d].E->stream));
    }
    counts->accounts = na;
    counts->transfers = nt;
    counts->posted = npv;
    return TBGPU_STATUS_OK;
}

static void node_reset_stats(TbNode* N) {
    tbgpu_reset_stats(N->X);
    N->passes_clean = N->passes_split = N->passes_whole = N->seq_events = 0;
}

static int node_api_get_stats(TbNode* N, tbgpu_stats* s) {
    memset(s, 0, sizeof(*s));
    s->node_passes_clean = N->passes_clean;
    s->node_passes_split = N->passes_split;
    s->node_passes_whole = N->passes_whole;
    s->node_sequenced_events = N->seq_events;
    double fill = 0;
    for (u32 d = 0; d <= N->world; d++) {  // every shard, then the sequencer (its ordered-path work)
        const bool seq = d == N->world;
        tbgpu_stats x;
        const int st = tbgpu_get_stats(seq ? N->X : N->D[d].E, &x);
        if (st) return st;
        s->dependent_events += x.dependent_events;
        if (!seq) {
            // Bounded residency per home shard: the log is as full as its fullest shard (a commit that
            // overruns any shard's log is refused), in units of the node's total capacity.
            s->transfers_evicted += x.transfers_evicted;
            s->log_capacity += x.log_capacity;
            if (x.log_capacity) fill = std::max(fill, (double)x.log_used / (double)x.log_capacity);
            s->node_shard_account_bytes[d] = x.account_table_bytes;
            s->account_table_bytes = std::max(s->account_table_bytes, x.account_table_bytes);
            s->passes += x.passes;
            s->events += x.events;
            s->accounts += x.accounts;  // each on its owner only
            s->transfers += x.transfers;
        }
        s->ms_validate += x.ms_validate;
        s->ms_resolve += x.ms_resolve;
        s->ms_replay += x.ms_replay;
        s->ms_clear += x.ms_clear;
        s->launches_validate += x.launches_validate;
        s->launches_resolve += x.launches_resolve;
        s->launches_replay += x.launches_replay;
        s->launches_clear += x.launches_clear;
        s->ms_apply += x.ms_apply;
        s->launches_apply += x.launches_apply;
        s->flow_passes += x.flow_passes;
        s->flow_units += x.flow_units;
        s->flow_runs += x.flow_runs;
        s->flow_run_units += x.flow_run_units;
        s->flow_plan_ms += x.flow_plan_ms;
        s->flow_run_ms += x.flow_run_ms;
        s->bounds_passes += x.bounds_passes;
        s->bounds_units += x.bounds_units;
        s->bounds_rounds += x.bounds_rounds;
        s->bounds_skipped += x.bounds_skipped;
        s->bounds_abandoned += x.bounds_abandoned;
        s->bounds_swept += x.bounds_swept;
        s->sweep_ms += x.sweep_ms;
        s->sweep_loop_ms += x.sweep_loop_ms;
        s->sweep_wait_ms += x.sweep_wait_ms;
        s->sweep_u64_passes += x.sweep_u64_passes;
        s->flow_exec_ms += x.flow_exec_ms;
        for (int k = 0; k < 8; k++) s->flow_phase_ms[k] += x.flow_phase_ms[k];
        for (int k = 0; k < 3; k++) {
            s->span_ms[k] += x.span_ms[k];
            s->span_launches[k] += x.span_launches[k];
        }
        s->walk_segments += x.walk_segments;
        s->walk_heavy += x.walk_heavy;
        s->walk_heavy_positions += x.walk_heavy_positions;
        s->walk_heavy_windows += x.walk_heavy_windows;
        s->walk_heavy_stops += x.walk_heavy_stops;
        s->walk_heavy_blocks += x.walk_heavy_blocks;
        s->walk_heavy_blocked_ms += x.walk_heavy_blocked_ms;
        s->walk_longest = std::max(s->walk_longest, x.walk_longest);
        s->walk_crit_windows += x.walk_crit_windows;
        s->walk_crit_blocks += x.walk_crit_blocks;
        s->walk_crit_wait_ms += x.walk_crit_wait_ms;
        s->walk_crit_ms += x.walk_crit_ms;
    }
    s->log_used = (u64)std::ceil(fill * (double)s->log_capacity);
    return TBGPU_STATUS_OK;
}

// Host memory for every shard's DMA: registered once, portable (every device may read it).
static int node_api_register_host(TbNode* N, void* ptr, u64 bytes) {
    NCK(hipSetDevice(N->D[0].device));
    NCK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    if (N->n_host_reg < 64) N->host_reg[N->n_host_reg++] = {(const u8*)ptr, bytes};
    return TBGPU_STATUS_OK;
}

static int node_api_unregister_host(TbNode* N, void* ptr) {
    const int st = node_sync(N);
    if (st) return st;
    NCK(hipSetDevice(N->D[0].device));
    NCK(hipHostUnregister(ptr));
    for (u32 i = 0; i < N->n_host_reg; i++) {
        if (N->host_reg[i].p == (const u8*)ptr) {
            N->host_reg[i] = N->host_reg[--N->n_host_reg];
            break;
        }
    }
    return TBGPU_STATUS_OK;
}

// Accounts from elsewhere (a load from the forest, an upsert): each to its owner; every shard's limit
// bitmap learns the limit accounts among them.
static int node_api_accounts_in(TbNode* N, const void* records, u32 n, bool load) {
    if (const int st = node_imports_flush(N)) return st;  // accounts are inserted on their owners below
    std::vector<std::vector<u8>> recs(N->world);
    bool limits = false;
    for (u32 i = 0; i < n; i++) {
        const u8* r = (const u8*)records + (u64)i * 128;
        recs[node_home(r, N->world)].insert(recs[node_home(r, N->world)].end(), r, r + 128);
        limits |= (*(const u16*)(r + 118) & AF_LIMITS) != 0;
    }
    for (u32 o = 0; o < N->world; o++) {
        const u32 m = (u32)(recs[o].size() / 128);
        if (!m) continue;
        const int st = load ? tbgpu_load_accounts(N->D[o].E, recs[o].data(), m) : tbgpu_upsert_accounts(N->D[o].E, recs[o].data(), m);
        if (st) return st;
    }
    if (!limits) return TBGPU_STATUS_OK;
    for (u32 d = 0; d < N->world; d++) {  // through the shard's staging buffer, in slices
        NodeDev& D = N->D[d];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        for (u32 i0 = 0; i0 < n; i0 += E->pe_max) {
            const u32 m = std::min<u32>(n - i0, E->pe_max);
            NCK(hipMemcpyAsync(E->staging, (const u8*)records + (u64)i0 * 128, (u64)m * 128, hipMemcpyHostToDevice, E->stream));
            hipLaunchKernelGGL(tb_limbits_from_records, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->staging, m, D.limbits,
                               D.limmask);
            NCK(hipGetLastError());
        }
        NCK(hipStreamSynchronize(E->stream));
    }
    N->limit_any = true;
    return TBGPU_STATUS_OK;
}

// Transfers from elsewhere: each to its home.
static int node_api_transfers_in(TbNode* N, const void* records, const u8* state, u32 n, bool load) {
    std::vector<std::vector<u8>> recs(N->world), sts(N->world);
    for (u32 i = 0; i < n; i++) {
        const u8* r = (const u8*)records + (u64)i * 128;
        const u32 h = node_home(r, N->world);
        recs[h].insert(recs[h].end(), r, r + 128);
        sts[h].push_back(state[i]);
    }
    for (u32 h = 0; h < N->world; h++) {
        if (sts[h].empty()) continue;
        const u32 m = (u32)sts[h].size();
        const int st = load ? tbgpu_load_transfers(N->D[h].E, recs[h].data(), sts[h].data(), m)
                            : tbgpu_upsert_transfers(N->D[h].E, recs[h].data(), sts[h].data(), m);
        if (st) return st;
    }
    return TBGPU_STATUS_OK;
}


static u64 node_commit_ts(TbNode* N) { return N->commit_ts; }
static u32 node_world(TbNode* N) { return N->world; }
static tbgpu* node_engine(TbNode* N, u32 d) { return N->D[d].E; }

static int node_api_set_commit_timestamp(TbNode* N, u64 timestamp) {
    const int st = node_sync(N);
    if (st) return st;
    N->commit_ts = timestamp;
    return node_publish_commit_ts(N);
}

// Bounded residency on a node (include/tbgpu.h tbgpu_evict_transfers): every home shard evicts from
// its own log what the last write-back covered, keeping its share of `keep` (its log's fraction of
// the node's).  Refused as a whole, before any shard moves, while any shard has a log position the
// last write-back did not cover (the node's write-back covers every shard at once).
static int node_api_evict(TbNode* N, uint64_t keep, uint64_t* evicted) {
    *evicted = 0;
    if (N->wb_inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight");
    int st = node_sync(N);
    if (st) return st;
    u64 cap = 0;
    for (u32 d = 0; d < N->world; d++) {
        const tbgpu* E = N->D[d].E;
        if (E->wb.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight");
        if (E->ckpt_valid && E->ckpt_pos != E->log_next) {
            return fail(TBGPU_STATUS_INVALID, "shard %u: %llu log positions written since the last write-back", d,
                        (unsigned long long)(E->log_next - E->ckpt_pos));
        }
        cap += E->xlog_cap;
    }
    for (u32 d = 0; d < N->world; d++) {
        tbgpu* E = N->D[d].E;
        const u64 k = cap ? (u64)((unsigned __int128)keep * E->xlog_cap / cap) : 0;
        u64 ev = 0;
        if ((st = engine_evict(E, k, &ev))) return st;
        *evicted += ev;
    }
    return TBGPU_STATUS_OK;
}

// tbgpu_transfers_maybe_cold on a node: each id asks its home shard (the one that would hold it and
// whose filter holds it if it left).
static int node_api_maybe_cold(TbNode* N, const uint64_t* ids, uint32_t n, uint8_t* cold) {
    memset(cold, 0, n);
    int st = node_sync(N);
    if (st) return st;
    const u32 W = N->world;
    std::vector<u64> per[NODE_WORLD_MAX];
    std::vector<u32> where[NODE_WORLD_MAX];
    for (u32 i = 0; i < n; i++) {
        const u32 h = tb_home(ids[2 * i], ids[2 * i + 1], W);
        per[h].push_back(ids[2 * i]);
        per[h].push_back(ids[2 * i + 1]);
        where[h].push_back(i);
    }
    std::vector<u8> c;
    for (u32 h = 0; h < W; h++) {
        const u32 m = (u32)where[h].size();
        if (!m) continue;
        c.assign(m, 0);
        if ((st = engine_maybe_cold(N->D[h].E, per[h].data(), m, c.data()))) return st;
        for (u32 j = 0; j < m; j++) cold[where[h][j]] = c[j];
    }
    return TBGPU_STATUS_OK;
}

// tbgpu_checkpoint_delta_async / _wait on a node: the same contract (the buffers belong to the engine
// until the wait; no other write-back may start), with the merged delta produced at the call.  The
// overlap with the next bar's commits that a single device gets (its capture in stream order, the
// objects crossing PCIe beside the commits) is not built for a node: its objects are merged over the
// shards on the host (owners' balances, homes' records).
static int node_api_checkpoint_delta_async(TbNode* N, void* accounts_out, void* accounts_before_out, u64 accounts_cap,
                                           void* transfers_out, u64 transfers_cap, u64* posted_out, u64 posted_cap) {
    tbgpu_delta_counts c;
    const int st = node_api_checkpoint_delta(N, accounts_out, accounts_before_out, accounts_cap, transfers_out,
                                             transfers_cap, posted_out, posted_cap, &c);
    if (st) return st;
    N->wb_counts = c;
    N->wb_inflight = true;
    return TBGPU_STATUS_OK;
}

static int node_api_checkpoint_delta_wait(TbNode* N, tbgpu_delta_counts* counts) {
    if (!N->wb_inflight) return fail(TBGPU_STATUS_INVALID, "no asynchronous write-back in flight");
    N->wb_inflight = false;
    *counts = N->wb_counts;
    return TBGPU_STATUS_OK;
}
