// node.h — the multi-device engine behind include/tbgpu.h (tbgpu_config.device_count > 1).
//
// The reference commits on one thread of one replica (src/vsr/replica.zig:3654, serial stages
// :3045-3102), and SURVEY.md §8e asks for one 8-GPU node with accounts hash-partitioned and
// cross-shard legs exchanged over xGMI.  Here the replica's single caller keeps its single call:
// tbgpu_commit / _many / _pipelined on a node engine route every pass across N shards (one per
// device listed in the config) inside the library — the exchange is kernels reading their peers'
// HBM (k_node.h), so no host staging, no collective library and no Python sit on the data path.
//
// Partition (the protocol of tigerbeetle_amd/sharded.py): account records replicated
// on every shard (create_accounts commits every prepare on every shard), balances on owner(id)
// only, a transfer on home(id).  A create_transfers call is cut into passes: pass p takes up to
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
// dirty pass is sequenced (node_sequence_pass): every in-flight pass drains, the transfers and
// accounts the pass reads are fetched from their homes / owners into a scratch engine on the first
// device, the pass commits there in order (the reference's prefetch -> commit split,
// src/state_machine.zig:345-506), and what changed is written back to homes and owners.
#pragma once

#include <thread>

#include "k_node.h"

struct NodeDev {
    tbgpu* E = nullptr;
    int device = 0;
    hipStream_t rs = nullptr;   // route stream (plans); E->copy_stream: H2D; E->stream: the pass
    // Source side, by pass parity.
    u8* stage[2] = {};
    u8* send[2] = {};
    u32* slot[2] = {};
    u8* home[2] = {};
    u64* words[2] = {};
    u64* h_words[2] = {};        // pinned: the plan words back on the host
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
};

struct NodeBlock {
    u32 k0 = 0, k1 = 0;  // global prepares [k0, k1)
    u64 events = 0;
};

struct NodePass {
    u32 k0 = 0, k1 = 0;
    NodeBlock blk[NODE_WORLD_MAX];
    std::vector<u64> off[NODE_WORLD_MAX];  // block-relative event offsets of its prepares
    bool issued = false, consumed = false;
};

struct TbNode {
    u32 world = 0;
    NodeDev D[NODE_WORLD_MAX];
    u64 pe_src = 0;        // source events per pass per shard
    u32 pb_src = 0;        // source prepares per pass per shard
    u64 recv_cap = 0;      // events a home can receive in one pass (world * pe_src)
    u64 commit_ts = 0;
    tbgpu* scratch = nullptr;  // the sequencer's engine (device of shard 0), grown on demand
    tbgpu_config scratch_cfg{};
    u64 passes_clean = 0, passes_sequenced = 0;
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

static void node_free(TbNode* N) {
    if (!N) return;
    for (u32 d = 0; d < N->world; d++) {
        NodeDev& D = N->D[d];
        if (D.E) {
            (void)hipSetDevice(D.device);
            (void)hipDeviceSynchronize();
        }
        void* dev[] = {D.stage[0], D.stage[1], D.send[0], D.send[1], D.slot[0], D.slot[1], D.home[0], D.home[1],
                       D.words[0], D.words[1], D.meta[0], D.meta[1], D.block_counts, D.results, D.reply_bytes,
                       D.recv, D.codes, D.legs, D.leg_counts, D.hmeta_dev[0], D.hmeta_dev[1], D.hmeta_dev[2]};
        for (void* p : dev) if (p) (void)hipFree(p);
        void* host[] = {D.h_words[0], D.h_words[1], D.h_meta[0], D.h_meta[1], D.hmeta_host[0], D.hmeta_host[1],
                        D.hmeta_host[2], D.h_arena[0], D.h_arena[1], D.h_arena[2]};
        for (void* p : host) if (p) (void)hipHostFree(p);
        hipEvent_t evs[] = {D.ev_start[0], D.ev_start[1], D.ev_start[2], D.ev_done[0], D.ev_done[1], D.ev_done[2],
                            D.ev_planned[0], D.ev_planned[1], D.ev_copied, D.ev_gathered, D.ev_committed,
                            D.ev_applied, D.ev_replied};
        for (hipEvent_t e : evs) if (e) (void)hipEventDestroy(e);
        if (D.rs) (void)hipStreamDestroy(D.rs);
        if (D.E) tbgpu_deinit(D.E);
    }
    if (N->scratch) tbgpu_deinit(N->scratch);
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
    N->world = W;
    N->pe_src = config->pass_events_max;
    N->pb_src = config->pass_batches_max;
    N->recv_cap = (u64)W * N->pe_src;
    // Shard engines: the account table of the whole ledger (records are replicated), the transfer
    // log of the transfers homed there (1/N of the ledger, with room for hash imbalance), routed
    // passes of up to ~1.25x a source block (larger receipts are committed in several passes).
    tbgpu_config sc = *config;
    sc.device_count = 0;
    sc.transfers_max = std::min<u64>(1ULL << 31, config->transfers_max / W + config->transfers_max / (8 * W) + N->recv_cap + 4096);
    sc.pass_events_max = (u32)std::min<u64>(N->recv_cap, N->pe_src + N->pe_src / 4 + 8192);
    sc.pass_batches_max = (u32)std::min<u64>(FLOW_NB_MAX, (sc.pass_events_max + BATCH_EVENTS_MAX - 2) / (BATCH_EVENTS_MAX - 1) + 2);
    sc.pass_batches_max = std::max(sc.pass_batches_max, N->pb_src);
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
            NALLOC(hipMalloc(&D.stage[k], pe * 128));
            NALLOC(hipMalloc(&D.send[k], pe * 128));
            NALLOC(hipMalloc(&D.slot[k], pe * 4));
            NALLOC(hipMalloc(&D.home[k], pe));
            NALLOC(hipMalloc(&D.words[k], ROUTE_WORDS * 8));
            NALLOC(hipHostMalloc(&D.h_words[k], ROUTE_WORDS * 8, hipHostMallocDefault));
            NALLOC(hipMalloc(&D.meta[k], (2 * (u64)N->pb_src + 1) * 8));
            NALLOC(hipHostMalloc(&D.h_meta[k], (2 * (u64)N->pb_src + 1) * 8, hipHostMallocDefault));
            NALLOC(hipEventCreateWithFlags(&D.ev_planned[k], hipEventDisableTiming));
        }
        NALLOC(hipMalloc(&D.block_counts, 2 * nblocks * W * 4));
        NALLOC(hipMalloc(&D.results, pe * 8));
        NALLOC(hipMalloc(&D.reply_bytes, (u64)N->pb_src * 4));
        NALLOC(hipMalloc(&D.recv, N->recv_cap * 128));
        NALLOC(hipMalloc(&D.codes, N->recv_cap));
        NALLOC(hipMalloc(&D.legs, legs_cap_total * OWNER_LEG_WORDS * 8));
        NALLOC(hipMalloc(&D.leg_counts, (u64)W * 8));
        const u64 hm = 2 * ((N->recv_cap + BATCH_EVENTS_MAX - 2) / (BATCH_EVENTS_MAX - 1) + 2) + 1;
        for (int k = 0; k < 3; k++) {
            NALLOC(hipMalloc(&D.hmeta_dev[k], hm * 8));
            NALLOC(hipHostMalloc(&D.hmeta_host[k], hm * 8, hipHostMallocDefault));
            NALLOC(hipHostMalloc(&D.h_arena[k], node_arena_bytes(N), hipHostMallocMapped));
            if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&D.d_arena[k], D.h_arena[k], 0);
            NALLOC(hipEventCreate(&D.ev_start[k]));
            NALLOC(hipEventCreate(&D.ev_done[k]));
        }
        NALLOC(hipEventCreateWithFlags(&D.ev_copied, hipEventDisableTiming));
        NALLOC(hipEventCreateWithFlags(&D.ev_gathered, hipEventDisableTiming));
        NALLOC(hipEventCreateWithFlags(&D.ev_committed, hipEventDisableTiming));
        NALLOC(hipEventCreateWithFlags(&D.ev_applied, hipEventDisableTiming));
        NALLOC(hipEventCreateWithFlags(&D.ev_replied, hipEventDisableTiming));
        // The events of "the previous pass" exist before the first pass: record them once.
        NALLOC(hipEventRecord(D.ev_gathered, D.E->stream));
        NALLOC(hipEventRecord(D.ev_applied, D.E->stream));
        NALLOC(hipEventRecord(D.ev_replied, D.E->stream));
    }
#undef NALLOC
    if (e != hipSuccess) {
        node_free(N);
        return node_fail_dev("tbgpu_init (node buffers)", e);
    }
    N->scratch_cfg = sc;
    N->scratch_cfg.device = N->D[0].device;
    *out = N;
    return TBGPU_STATUS_OK;
}

// Drain every device and read back its globals (panic, commit_timestamp).
static int node_sync(TbNode* N) {
    int status = TBGPU_STATUS_OK;
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
        E->h_meta[0] = N->commit_ts;  // staging word for the async copy (the stream is drained)
        NCK(hipMemcpyAsync(&E->g->commit_timestamp, E->h_meta, 8, hipMemcpyHostToDevice, E->stream));
        NCK(hipStreamSynchronize(E->stream));
    }
    return TBGPU_STATUS_OK;
}

// -- create_accounts: every shard commits every prepare (records are replicated) ------------------

static int node_commit_replicated(TbNode* N, u8 op, u32 n, const u64* ts, const void* const* inputs, const u32* in_lens,
                                  void* const* outputs, u32* out_lens, u32 chunk) {
    std::vector<std::vector<u8>> outs((size_t)N->world - 1);
    std::vector<std::vector<void*>> optrs((size_t)N->world - 1);
    std::vector<std::vector<u32>> olens((size_t)N->world - 1, std::vector<u32>(n));
    for (u32 d = 1; d < N->world; d++) {
        u64 total = 0;
        for (u32 k = 0; k < n; k++) total += (u64)(in_lens[k] / 128) * 8;
        outs[d - 1].resize(std::max<u64>(total, 8));
        optrs[d - 1].resize(n);
        u64 o = 0;
        for (u32 k = 0; k < n; k++) {
            optrs[d - 1][k] = outs[d - 1].data() + o;
            o += (u64)(in_lens[k] / 128) * 8;
        }
    }
    std::vector<int> st(N->world, TBGPU_STATUS_OK);
    std::vector<std::string> err(N->world);
    std::vector<std::thread> th;
    for (u32 d = 0; d < N->world; d++) {
        th.emplace_back([&, d]() {
            tbgpu* E = N->D[d].E;
            if (hipSetDevice(N->D[d].device) != hipSuccess) {
                st[d] = TBGPU_STATUS_DEVICE;
                return;
            }
            st[d] = commit_pipelined(E, op, n, ts, inputs, in_lens, d == 0 ? outputs : optrs[d - 1].data(),
                                     d == 0 ? out_lens : olens[d - 1].data(), nullptr, chunk, nullptr);
            if (st[d]) err[d] = g_err;  // g_err is thread-local
        });
    }
    for (auto& t : th) t.join();
    for (u32 d = 0; d < N->world; d++) {
        if (st[d]) return fail(st[d], "%s", err[d].c_str());
    }
    for (u32 d = 1; d < N->world; d++) {  // replicas of the same deterministic commit
        for (u32 k = 0; k < n; k++) {
            if (olens[d - 1][k] != out_lens[k] || memcmp(optrs[d - 1][k], outputs[k], out_lens[k]) != 0) {
                return fail(TBGPU_STATUS_PANIC, "node: shard %u replied differently to replicated prepare %u", d, k);
            }
        }
    }
    for (u32 d = 0; d < N->world; d++) N->commit_ts = std::max(N->commit_ts, N->D[d].E->commit_ts);
    return TBGPU_STATUS_OK;
}

// -- create_transfers ----------------------------------------------------------------------------

// H2D of source d's block of pass p and its route plan (enqueued; ev_planned[p & 1] fires when the
// plan's words are in pinned host memory).
static int node_issue_plan(TbNode* N, NodePass& P, u32 p, const u64* ts, const void* const* inputs, const u32* lens) {
    const u32 par = p & 1;
    for (u32 d = 0; d < N->world; d++) {
        NodeDev& D = N->D[d];
        const NodeBlock& B = P.blk[d];
        const u32 nb = B.k1 - B.k0;
        if (nb == 0) continue;
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        u64* h_off = D.h_meta[par];
        u64* h_ts = h_off + nb + 1;
        for (u32 k = 0; k <= nb; k++) h_off[k] = P.off[d][k];
        for (u32 k = 0; k < nb; k++) h_ts[k] = ts[B.k0 + k];
        // Copy stream: the bodies (runs of address-contiguous prepares as one DMA).
        NCK(hipEventRecord(D.ev_start[p % 3], E->copy_stream));
        for (u32 k = B.k0; k < B.k1;) {
            u32 j = k + 1;
            const u8* base = (const u8*)inputs[k];
            u64 bytes = (u64)lens[k] * 128;
            while (j < B.k1 && (const u8*)inputs[j] == base + bytes) bytes += (u64)lens[j++] * 128;
            if (bytes) NCK(hipMemcpyAsync(D.stage[par] + P.off[d][k - B.k0] * 128, base, bytes, hipMemcpyHostToDevice,
                                          E->copy_stream));
            k = j;
        }
        NCK(hipEventRecord(D.ev_copied, E->copy_stream));
        // Route stream: wait for the buffers' previous users (pass p-2's gathers on every home and
        // this source's replies), then the plan.
        NCK(hipStreamWaitEvent(D.rs, D.ev_copied, 0));
        NCK(hipStreamWaitEvent(D.rs, D.ev_replied, 0));
        for (u32 h = 0; h < N->world; h++) {
            NCK(hipSetDevice(D.device));
            NCK(hipStreamWaitEvent(D.rs, N->D[h].ev_gathered, 0));
        }
        NCK(hipMemcpyAsync(D.meta[par], h_off, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, D.rs));
        NCK(hipMemsetAsync(D.words[par], 0, ROUTE_WORDS * 8, D.rs));
        RouteArgs A{};
        A.events = D.stage[par];
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
        if (B.events) {
            hipLaunchKernelGGL(tb_route_classify, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A);
            NCK(hipGetLastError());
            hipLaunchKernelGGL(tb_route_offsets, dim3(A.world), dim3(1024), 0, D.rs, A);
            NCK(hipGetLastError());
            hipLaunchKernelGGL(tb_route_scatter, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, D.rs, A, D.send[par], D.slot[par]);
            NCK(hipGetLastError());
        }
        NCK(hipMemcpyAsync(D.h_words[par], D.words[par], ROUTE_WORDS * 8, hipMemcpyDeviceToHost, D.rs));
        NCK(hipEventRecord(D.ev_planned[par], D.rs));
    }
    return TBGPU_STATUS_OK;
}

struct NodePlan {
    u64 C[NODE_WORLD_MAX][NODE_WORLD_MAX];  // events of source s for home h
    unsigned __int128 S = 0;                // saturating sum of every amount of the pass
    u32 dirty = 0;
    bool huge = false;
};

static int node_read_plan(TbNode* N, const NodePass& P, u32 p, NodePlan* out) {
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
        NCK(hipEventSynchronize(D.ev_planned[par]));
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

// Gather, routed commit with owner legs, legs to owners, replies to sources — every device, enqueued.
static int node_issue_commit(TbNode* N, NodePass& P, u32 p, const NodePlan& PL, u32 cert, u64 ts_max) {
    const u32 W = N->world, par = p & 1, tri = p % 3;
    u64 R[NODE_WORLD_MAX][NODE_WORLD_MAX];    // R[h][s]: where source s's run starts in home h's receipt
    u64 off[NODE_WORLD_MAX][NODE_WORLD_MAX];  // off[s][h]: where home h's run starts in source s's send buffer
    u64 nh[NODE_WORLD_MAX];
    for (u32 h = 0; h < W; h++) {
        u64 r = 0;
        for (u32 s = 0; s < W; s++) {
            R[h][s] = r;
            r += PL.C[s][h];
        }
        nh[h] = r;
    }
    for (u32 s = 0; s < W; s++) {
        u64 o = 0;
        for (u32 h = 0; h < W; h++) {
            off[s][h] = o;
            o += PL.C[s][h];
        }
    }
    for (u32 h = 0; h < W; h++) {
        if (nh[h] > N->recv_cap) return fail(TBGPU_STATUS_INVALID, "node: home %u receives %llu events > %llu", h,
                                             (unsigned long long)nh[h], (unsigned long long)N->recv_cap);
        if (N->D[h].E->log_next + nh[h] > N->D[h].E->xlog_cap) {
            return fail(TBGPU_STATUS_INVALID, "node: transfer log of shard %u full (%llu + %llu > %llu)", h,
                        (unsigned long long)N->D[h].E->log_next, (unsigned long long)nh[h],
                        (unsigned long long)N->D[h].E->xlog_cap);
        }
    }
    // 1. Homes: gather, then (after the previous pass's readers of codes / legs) the routed commit.
    for (u32 h = 0; h < W; h++) {
        NodeDev& D = N->D[h];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        if (nh[h]) {
            NodeGatherArgs G{};
            G.world = W;
            G.recv = D.recv;
            for (u32 s = 0; s < W; s++) {
                G.src[s] = N->D[s].send[par] + off[s][h] * 128;
                G.start[s] = R[h][s];
            }
            G.start[W] = nh[h];
            hipLaunchKernelGGL(tb_node_gather, dim3((unsigned)((nh[h] * 8 + 255) / 256)), dim3(256), 0, E->stream, G);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_gathered, E->stream));
        for (u32 o = 0; o < W; o++) {
            NCK(hipSetDevice(D.device));
            NCK(hipStreamWaitEvent(E->stream, N->D[o].ev_applied, 0));
            NCK(hipStreamWaitEvent(E->stream, N->D[o].ev_replied, 0));
        }
        NCK(hipSetDevice(D.device));
        NCK(hipMemsetAsync(D.leg_counts, 0, (u64)W * 8, E->stream));
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
            NCK(hipMemcpyAsync(D.hmeta_dev[tri], h_off, (2 * nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
            std::vector<u64> offs(h_off, h_off + nb + 1);
            OwnerLegArgs O{W, h, D.legs, 2 * nh[h], D.leg_counts};
            const int st = enqueue_call(E, OP_CREATE_TRANSFERS, (u32)nb, offs.data(), D.recv, E->results, E->reply_bytes,
                                        true, D.codes, cert, nullptr, D.hmeta_dev[tri], &O);
            if (st) return st;
        }
        NCK(hipEventRecord(D.ev_committed, E->stream));
    }
    // 2. Owners: the legs they own, from every home.
    for (u32 o = 0; o < W; o++) {
        NodeDev& D = N->D[o];
        tbgpu* E = D.E;
        NCK(hipSetDevice(D.device));
        NodeLegArgs L{};
        L.world = W;
        L.cert64 = cert == TBGPU_CERT_U64 ? 1u : 0u;
        u64 legs_max = 0;
        for (u32 h = 0; h < W; h++) {
            if (h != o) NCK(hipStreamWaitEvent(E->stream, N->D[h].ev_committed, 0));
            L.legs[h] = N->D[h].legs + (u64)o * 2 * nh[h] * OWNER_LEG_WORDS;
            L.counts[h] = N->D[h].leg_counts + o;
            legs_max += 2 * nh[h];
        }
        if (legs_max) {
            const u32 grid = (u32)std::min<u64>(4096, std::max<u64>(1, (legs_max / W + 255) / 256));
            hipLaunchKernelGGL(tb_node_apply_legs, dim3(grid), dim3(256), 0, E->stream, E->T, L);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_applied, E->stream));
    }
    // 3. Sources: replies from the codes their homes wrote, into the reply arena.
    for (u32 s = 0; s < W; s++) {
        NodeDev& D = N->D[s];
        tbgpu* E = D.E;
        const u32 nb = P.blk[s].k1 - P.blk[s].k0;
        NCK(hipSetDevice(D.device));
        if (nb) {
            NodeReplyArgs A{};
            for (u32 h = 0; h < W; h++) {
                A.codes[h] = N->D[h].codes;
                A.delta[h] = (i64)R[h][s] - (i64)off[s][h];
            }
            hipLaunchKernelGGL(tb_node_replies, dim3(nb), dim3(1024), 0, E->stream, D.meta[par], D.home[par], D.slot[par], A,
                               D.results, D.reply_bytes);
            NCK(hipGetLastError());
        }
        NCK(hipEventRecord(D.ev_replied, E->stream));
        if (nb) {
            hipLaunchKernelGGL(tb_reply_out, dim3(nb), dim3(64), 0, E->stream, D.meta[par], nb, D.reply_bytes, D.results,
                               E->g, D.d_arena[tri]);
            NCK(hipGetLastError());
            NCK(hipEventRecord(D.ev_done[tri], E->stream));
        }
    }
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
        if (!nb) continue;
        NCK(hipSetDevice(D.device));
        NCK(hipEventSynchronize(D.ev_done[tri]));
        if (!take || status) continue;
        const u64* head = (const u64*)D.h_arena[tri];
        const u32* rb = (const u32*)(D.h_arena[tri] + 16);
        const u8* res = D.h_arena[tri] + 16 + (u64)nb * 4;
        float ms = 0;
        if (latency_ms) NCK(hipEventElapsedTime(&ms, D.ev_start[tri], D.ev_done[tri]));
        for (u32 k = B.k0; k < B.k1; k++) {
            const u32 bytes = rb[k - B.k0];
            if (bytes) memcpy(outputs[k], res + 8 * P.off[s][k - B.k0], bytes);
            out_lens[k] = bytes;
            if (latency_ms) latency_ms[k] = ms;
        }
        N->commit_ts = std::max(N->commit_ts, head[1]);
        if (head[0]) status = fail(TBGPU_STATUS_PANIC, "device panic 0x%llx on shard %u (the reference would have trapped)",
                                   (unsigned long long)head[0], s);
    }
    P.consumed = true;
    return status;
}

static int node_upsert_accounts_keep_flow(tbgpu* E, const void* records, uint32_t n);

// A dirty pass, committed in order on the scratch engine after fetching what it reads, then
// written back (synchronous; every earlier pass has drained).
static int node_sequence_pass(TbNode* N, const NodePass& P, const u64* ts, const void* const* inputs, const u32* lens,
                              void* const* outputs, u32* out_lens) {
    typedef unsigned __int128 h128;
    const u32 W = N->world;
    auto key = [](const u8* p) { return *(const h128*)p; };
    const h128 MAXID = ~(h128)0;
    // 1. The transfers the pass reads: every event id, the pending id of post / void events.
    std::vector<h128> tids;
    for (u32 k = P.k0; k < P.k1; k++) {
        const u8* body = (const u8*)inputs[k];
        for (u32 i = 0; i < lens[k]; i++) {
            const u8* ev = body + (u64)i * 128;
            tids.push_back(key(ev));
            const u16 fl = *(const u16*)(ev + 118);
            if (fl & (TF_POST | TF_VOID)) tids.push_back(key(ev + 64));
        }
    }
    auto uniq = [&](std::vector<h128>& v) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        v.erase(std::remove_if(v.begin(), v.end(), [&](h128 x) { return x == 0 || x == MAXID; }), v.end());
    };
    uniq(tids);
    const u64 nt = tids.size();
    std::vector<u8> trec(nt * 128), tstate(nt);
    {
        std::vector<std::vector<u64>> ids(W);
        std::vector<std::vector<u64>> where(W);
        for (u64 i = 0; i < nt; i++) {
            const u32 h = node_home((const u8*)&tids[i], W);
            ids[h].push_back((u64)tids[i]);
            ids[h].push_back((u64)(tids[i] >> 64));
            where[h].push_back(i);
        }
        for (u32 h = 0; h < W; h++) {
            const u64 m = where[h].size();
            if (!m) continue;
            std::vector<u8> rec(m * 128), st(m);
            const int s = tbgpu_fetch_transfers(N->D[h].E, ids[h].data(), (u32)m, rec.data(), st.data());
            if (s) return s;
            for (u64 j = 0; j < m; j++) {
                memcpy(&trec[where[h][j] * 128], &rec[j * 128], 128);
                tstate[where[h][j]] = st[j];
            }
        }
    }
    // 2. The accounts: of every event, and of every pending transfer a post / void reads.
    std::vector<h128> aids;
    for (u32 k = P.k0; k < P.k1; k++) {
        const u8* body = (const u8*)inputs[k];
        for (u32 i = 0; i < lens[k]; i++) {
            aids.push_back(key(body + (u64)i * 128 + 16));
            aids.push_back(key(body + (u64)i * 128 + 32));
        }
    }
    for (u64 i = 0; i < nt; i++) {
        if (!tstate[i]) continue;
        aids.push_back(key(&trec[i * 128 + 16]));
        aids.push_back(key(&trec[i * 128 + 32]));
    }
    uniq(aids);
    const u64 na = aids.size();
    std::vector<u8> arec(na * 128), afound(na);
    {
        std::vector<std::vector<u64>> ids(W);
        std::vector<std::vector<u64>> where(W);
        for (u64 i = 0; i < na; i++) {
            const u32 o = node_home((const u8*)&aids[i], W);
            ids[o].push_back((u64)aids[i]);
            ids[o].push_back((u64)(aids[i] >> 64));
            where[o].push_back(i);
        }
        for (u32 o = 0; o < W; o++) {
            const u64 m = where[o].size();
            if (!m) continue;
            std::vector<u8> rec(m * 128), fd(m);
            const int s = tbgpu_fetch_accounts(N->D[o].E, ids[o].data(), (u32)m, rec.data(), fd.data());
            if (s) return s;
            for (u64 j = 0; j < m; j++) {
                memcpy(&arec[where[o][j] * 128], &rec[j * 128], 128);
                afound[where[o][j]] = fd[j];
            }
        }
    }
    // 3. The scratch engine, holding exactly what the pass reads.
    u64 events = 0;
    for (u32 k = P.k0; k < P.k1; k++) events += lens[k];
    const u64 need_a = std::max<u64>(1024, na + 1), need_t = std::max<u64>(1024, nt + events + 1);
    if (N->scratch && (N->scratch->cfg.accounts_max < need_a || N->scratch->cfg.transfers_max < need_t)) {
        tbgpu_deinit(N->scratch);
        N->scratch = nullptr;
    }
    if (!N->scratch) {
        tbgpu_config c = N->scratch_cfg;
        c.accounts_max = std::max<u64>(need_a, 1 << 16);
        c.transfers_max = std::max<u64>(need_t, 1 << 20);
        c.pass_events_max = (u32)std::max<u64>(N->pe_src, BATCH_EVENTS_MAX);
        c.pass_batches_max = std::max<u32>(1, std::min<u32>(N->pb_src, FLOW_NB_MAX));
        c.flags &= ~(u32)TBGPU_CONFIG_PROFILE;
        const int s = tbgpu_init(&c, &N->scratch);
        if (s) return s;
    }
    tbgpu* X = N->scratch;
    int s = tbgpu_reset(X);
    if (s) return s;
    if ((s = tbgpu_set_commit_timestamp(X, N->commit_ts))) return s;
    {
        std::vector<u8> found_recs;
        for (u64 i = 0; i < na; i++) {
            if (afound[i]) found_recs.insert(found_recs.end(), &arec[i * 128], &arec[i * 128] + 128);
        }
        if (!found_recs.empty() && (s = tbgpu_load_accounts(X, found_recs.data(), (u32)(found_recs.size() / 128)))) return s;
        std::vector<u8> present, pstate;
        for (u64 i = 0; i < nt; i++) {
            if (!tstate[i]) continue;
            present.insert(present.end(), &trec[i * 128], &trec[i * 128] + 128);
            pstate.push_back((u8)(tstate[i] - 1));
        }
        if (!pstate.empty() && (s = tbgpu_load_transfers(X, present.data(), pstate.data(), (u32)pstate.size()))) return s;
    }
    // 4. The pass, in order.
    const u32 nk = P.k1 - P.k0;
    std::vector<u32> in_lens(nk);
    for (u32 k = 0; k < nk; k++) in_lens[k] = lens[P.k0 + k] * 128;
    if ((s = commit_pipelined(X, OP_CREATE_TRANSFERS, nk, ts + P.k0, inputs + P.k0, in_lens.data(), outputs + P.k0,
                              out_lens + P.k0, nullptr, std::min<u32>(nk, X->pb_max), nullptr))) {
        return s;
    }
    // 5. Write back: new transfers and changed posted states to their homes, the touched accounts'
    //    balances to their owners.
    {
        std::vector<u64> ids(2 * nt);
        for (u64 i = 0; i < nt; i++) {
            ids[2 * i] = (u64)tids[i];
            ids[2 * i + 1] = (u64)(tids[i] >> 64);
        }
        std::vector<u8> after(nt * 128), ast(nt);
        if (nt && (s = tbgpu_fetch_transfers(X, ids.data(), (u32)nt, after.data(), ast.data()))) return s;
        std::vector<std::vector<u8>> recs(W), sts(W);
        for (u64 i = 0; i < nt; i++) {
            if (ast[i] == 0 || ast[i] == tstate[i]) continue;
            const u32 h = node_home(&after[i * 128], W);
            recs[h].insert(recs[h].end(), &after[i * 128], &after[i * 128] + 128);
            sts[h].push_back(ast[i]);
        }
        for (u32 h = 0; h < W; h++) {
            if (!sts[h].empty() && (s = tbgpu_upsert_transfers(N->D[h].E, recs[h].data(), sts[h].data(), (u32)sts[h].size()))) {
                return s;
            }
        }
        std::vector<u64> aid2;
        for (u64 i = 0; i < na; i++) {
            if (!afound[i]) continue;
            aid2.push_back((u64)aids[i]);
            aid2.push_back((u64)(aids[i] >> 64));
        }
        const u64 nf = aid2.size() / 2;
        std::vector<u8> aafter(nf * 128), afd(nf);
        if (nf && (s = tbgpu_fetch_accounts(X, aid2.data(), (u32)nf, aafter.data(), afd.data()))) return s;
        std::vector<std::vector<u8>> arecs(W);
        for (u64 i = 0; i < nf; i++) {
            const u32 o = node_home(&aafter[i * 128], W);
            arecs[o].insert(arecs[o].end(), &aafter[i * 128], &aafter[i * 128] + 128);
        }
        for (u32 o = 0; o < W; o++) {
            if (!arecs[o].empty() && (s = node_upsert_accounts_keep_flow(N->D[o].E, arecs[o].data(), (u32)(arecs[o].size() / 128)))) {
                return s;
            }
        }
    }
    N->commit_ts = std::max(N->commit_ts, X->commit_ts);
    N->passes_sequenced++;
    return TBGPU_STATUS_OK;
}

// The node's commit of n create_transfers prepares from host memory.
static int node_commit_transfers(TbNode* N, u32 n, const u64* ts, const void* const* inputs, const u32* lens,
                                 void* const* outputs, u32* out_lens, u32 chunk, double* latency_ms) {
    typedef unsigned __int128 h128;
    const u32 W = N->world;
    const u32 per = std::max<u32>(1, std::min<u32>(chunk ? chunk : N->pb_src, N->pb_src));
    // Passes: W blocks of up to `per` prepares and pe_src events each, in prepare order.
    std::vector<NodePass> passes;
    for (u32 k = 0; k < n;) {
        NodePass P;
        P.k0 = k;
        for (u32 d = 0; d < W; d++) {
            NodeBlock& B = P.blk[d];
            B.k0 = B.k1 = k;
            P.off[d].assign(1, 0);
            while (k < n && B.k1 - B.k0 < per && B.events + lens[k] <= N->pe_src) {
                B.events += lens[k];
                P.off[d].push_back(B.events);
                k++;
                B.k1 = k;
            }
        }
        if (k == P.k0) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
        P.k1 = k;
        passes.push_back(std::move(P));
    }
    int st = node_sync(N);
    if (st) return st;
    h128 bound = node_bound(N);
    int status = TBGPU_STATUS_OK;
    const u32 NP = (u32)passes.size();
    u32 next_consume = 0;
    auto consume_upto = [&](u32 end) {  // consume every issued pass < end
        for (; next_consume < end; next_consume++) {
            NodePass& P = passes[next_consume];
            if (P.issued && !P.consumed) {
                const int c = node_consume(N, P, next_consume, outputs, out_lens, latency_ms, status == TBGPU_STATUS_OK);
                if (status == TBGPU_STATUS_OK) status = c;
            }
        }
    };
    if ((status = node_issue_plan(N, passes[0], 0, ts, inputs, lens))) return status;
    for (u32 p = 0; p < NP && status == TBGPU_STATUS_OK; p++) {
        if (p >= 2) consume_upto(p - 1);  // pass p-2: its arena slot, start event and meta are reused next
        if (status) break;
        if (p + 1 < NP && (status = node_issue_plan(N, passes[p + 1], p + 1, ts, inputs, lens))) break;
        NodePlan PL;
        if ((status = node_read_plan(N, passes[p], p, &PL))) break;
        const h128 total = bound + PL.S < bound ? ~(h128)0 : bound + PL.S;
        if (PL.dirty || PL.huge || total == ~(h128)0) {
            consume_upto(p);
            if (status) break;
            if ((status = node_sync(N))) break;
            if ((status = node_sequence_pass(N, passes[p], ts, inputs, lens, outputs, out_lens))) break;
            if (latency_ms) for (u32 k = passes[p].k0; k < passes[p].k1; k++) latency_ms[k] = 0;
            passes[p].consumed = true;
            if ((status = node_sync(N))) break;
            bound = node_bound(N);
            continue;
        }
        const u32 cert = (total >> 64) == 0 ? TBGPU_CERT_U64 : TBGPU_CERT_U128;
        if ((status = node_issue_commit(N, passes[p], p, PL, cert, ts[passes[p].k1 - 1]))) break;
        bound = total;
        N->passes_clean++;
    }
    consume_upto(NP);
    const int s2 = node_sync(N);
    if (status == TBGPU_STATUS_OK) status = s2;
    const int s3 = node_publish_commit_ts(N);
    return status ? status : s3;
}

static int node_commit_pipelined(TbNode* N, u8 op, u32 n, const u64* ts, const void* const* inputs, const u32* input_lens,
                                 void* const* outputs, u32* out_lens, u32 chunk, double* latency_ms) {
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
        const int st = node_commit_replicated(N, op, n, ts, inputs, input_lens, outputs, out_lens, chunk);
        const int s2 = node_publish_commit_ts(N);
        return st ? st : s2;
    }
    return node_commit_transfers(N, n, ts, inputs, lens.data(), outputs, out_lens, chunk, latency_ms);
}

// -- lookups, exports, write-back, test setup ------------------------------------------------------

// Every account (identical on every shard but the balances) with the balances of its owner.
static int node_export_accounts(TbNode* N, std::vector<u8>& out) {
    std::vector<std::vector<u8>> per(N->world);
    for (u32 d = 0; d < N->world; d++) {
        if (hipSetDevice(N->D[d].device) != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "hipSetDevice");
        const int st = export_records<true>(N->D[d].E, per[d], nullptr);
        if (st) return st;
        if (per[d].size() != per[0].size()) return fail(TBGPU_STATUS_PANIC, "node: shards hold different accounts");
    }
    out = per[0];
    const u64 n = out.size() / 128;
    for (u64 i = 0; i < n; i++) {
        const u32 o = node_home(&out[i * 128], N->world);
        if (o) memcpy(&out[i * 128 + 16], &per[o][i * 128 + 16], 64);  // dp, dpost, cp, cpost
    }
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
    E->device = N->D[0].device;
    *out = E;
    return TBGPU_STATUS_OK;
}

static int node_api_reset(TbNode* N) {
    for (u32 d = 0; d < N->world; d++) {
        const int st = tbgpu_reset(N->D[d].E);
        if (st) return st;
    }
    N->commit_ts = 0;
    return TBGPU_STATUS_OK;
}

static int node_api_commit(TbNode* N, u8 op, u64 timestamp, const void* input, u32 input_len, void* output,
                           u32 output_cap, u32* out_len) {
    *out_len = 0;
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

// The setup action (state_machine.zig:1398-1407): the owner holds the balances, every other shard
// zeros for the account.
static int node_api_set_balances(TbNode* N, u64 id_lo, u64 id_hi, const u64 b[8]) {
    const u32 o = tb_home(id_lo, id_hi, N->world);
    const u64 zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (u32 d = 0; d < N->world; d++) {
        const int st = tbgpu_test_set_balances(N->D[d].E, id_lo, id_hi, d == o ? b : zero);
        if (st) return st;
    }
    return TBGPU_STATUS_OK;
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

// Groove write-back of the node, O(changes) like a single engine's (engine.hip delta_*): the new
// transfers of every shard's log, merged by timestamp; the posted entries their post / void records
// make (the pending transfer may live on another shard: its timestamp is fetched from its home); the
// accounts the new transfers moved — wherever those transfers live — plus the listed creates and
// direct writes, each looked up on its OWNER, whose copy holds its balances (a whole-table diff of
// a shard keeps only the accounts it owns).
static int node_api_checkpoint_delta(TbNode* N, void* accounts_out, void* accounts_before_out, u64 accounts_cap,
                                     void* transfers_out, u64 transfers_cap, u64* posted_out, u64 posted_cap,
                                     tbgpu_delta_counts* counts) {
    memset(counts, 0, sizeof(*counts));
    const u32 W = N->world;
    int st = node_sync(N);
    if (st) return st;
    std::vector<DeltaCtx> C(W);
    auto abort_all = [&](int status) {
        for (u32 d = 0; d < W; d++) delta_free(C[d]);
        return status;
    };
    std::vector<u64> ids_all, pv_all;
    u64 nt = 0;
    for (u32 d = 0; d < W; d++) {
        NCK(hipSetDevice(N->D[d].device));
        std::vector<u64> ids, pv;
        if ((st = delta_begin(N->D[d].E, C[d]))) return abort_all(st);
        if ((st = delta_log_ids(N->D[d].E, C[d], &ids, &pv))) return abort_all(st);
        ids_all.insert(ids_all.end(), ids.begin(), ids.end());
        pv_all.insert(pv_all.end(), pv.begin(), pv.end());
        ids_all.insert(ids_all.end(), N->D[d].E->ckpt_ids.begin(), N->D[d].E->ckpt_ids.end());
        nt += C[d].nt;
    }
    std::vector<std::vector<u64>> owned(W);
    for (size_t i = 0; i + 1 < ids_all.size(); i += 2) {
        const u32 o = tb_home(ids_all[i], ids_all[i + 1], W);
        owned[o].push_back(ids_all[i]);
        owned[o].push_back(ids_all[i + 1]);
    }
    std::vector<u64> na(W, 0);
    u64 na_total = 0;
    for (u32 o = 0; o < W; o++) {
        tbgpu* E = N->D[o].E;
        NCK(hipSetDevice(N->D[o].device));
        if ((st = delta_alloc_accounts(E, C[o], owned[o].size() / 2))) return abort_all(st);
        if ((st = delta_ids_host(E, C[o], owned[o]))) return abort_all(st);
        if ((st = delta_scan(E, C[o], W, o))) return abort_all(st);
        if ((st = delta_account_count(E, C[o], &na[o]))) return abort_all(st);
        na_total += na[o];
    }
    std::vector<std::pair<u64, u64>> posted;
    st = delta_posted_pairs(pv_all, posted, [&](const u64* ids, u32 n, u8* out, u8* state) {
        return node_fetch(N, false, ids, n, out, state);
    });
    if (st) return abort_all(st);
    counts->created_after = N->D[0].E->ckpt_ts;
    counts->accounts = na_total;
    counts->transfers = nt;
    counts->posted = posted.size();
    if (na_total > accounts_cap || nt > transfers_cap || posted.size() > posted_cap) {  // nothing advanced
        return abort_all(fail(TBGPU_STATUS_INVALID, "checkpoint delta: needs %llu accounts, %llu transfers, %llu posted",
                              (unsigned long long)na_total, (unsigned long long)nt, (unsigned long long)posted.size()));
    }
    for (size_t i = 0; i < posted.size(); i++) {
        posted_out[2 * i] = posted[i].first;
        posted_out[2 * i + 1] = posted[i].second;
    }
    // Transfers: each shard's in timestamp order, merged.
    std::vector<std::vector<u8>> runs(W);
    for (u32 d = 0; d < W; d++) {
        NCK(hipSetDevice(N->D[d].device));
        runs[d].resize(C[d].nt * 128);
        if ((st = delta_copy_transfers(N->D[d].E, C[d], runs[d].data()))) return abort_all(st);
        delta_sort_by_timestamp(runs[d].data(), C[d].nt);
    }
    {
        std::vector<size_t> pos(W, 0);
        auto ts_at = [&](u32 d) { return *(const u64*)&runs[d][pos[d] * 128 + 120]; };
        for (u64 k = 0; k < nt; k++) {
            u32 best = W;
            for (u32 d = 0; d < W; d++) {
                if (pos[d] < C[d].nt && (best == W || ts_at(d) < ts_at(best))) best = d;
            }
            memcpy((u8*)transfers_out + k * 128, &runs[best][pos[best] * 128], 128);
            pos[best]++;
        }
    }
    // Accounts: each owner's, one after the other.
    u64 at = 0;
    for (u32 o = 0; o < W; o++) {
        NCK(hipSetDevice(N->D[o].device));
        if ((st = delta_copy_accounts(N->D[o].E, C[o], na[o], (u8*)accounts_out + at * 128,
                                      accounts_before_out ? (u8*)accounts_before_out + at * 64 : nullptr))) {
            return abort_all(st);
        }
        at += na[o];
    }
    for (u32 d = 0; d < W; d++) {
        NCK(hipSetDevice(N->D[d].device));
        if ((st = delta_end(N->D[d].E, C[d]))) return abort_all(st);
    }
    return TBGPU_STATUS_OK;
}

static int node_api_get_stats(TbNode* N, tbgpu_stats* s) {
    memset(s, 0, sizeof(*s));
    for (u32 d = 0; d < N->world; d++) {
        tbgpu_stats x;
        const int st = tbgpu_get_stats(N->D[d].E, &x);
        if (st) return st;
        s->passes += x.passes;
        s->events += x.events;
        s->dependent_events += x.dependent_events;
        if (d == 0) s->accounts = x.accounts;  // replicated records
        s->transfers += x.transfers;
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
    return TBGPU_STATUS_OK;
}

// Host memory for every shard's DMA: registered once, portable (every device may read it).
static int node_api_register_host(TbNode* N, void* ptr, u64 bytes) {
    NCK(hipSetDevice(N->D[0].device));
    NCK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    return TBGPU_STATUS_OK;
}

static int node_api_unregister_host(TbNode* N, void* ptr) {
    const int st = node_sync(N);
    if (st) return st;
    NCK(hipSetDevice(N->D[0].device));
    NCK(hipHostUnregister(ptr));
    return TBGPU_STATUS_OK;
}

// Accounts from elsewhere (a load from the forest, an upsert): every shard gets the record, the
// owner its balances, the others zeros.
static int node_api_accounts_in(TbNode* N, const void* records, u32 n, bool load) {
    std::vector<u8> zeroed((const u8*)records, (const u8*)records + (u64)n * 128);
    for (u32 i = 0; i < n; i++) memset(&zeroed[(u64)i * 128 + 16], 0, 64);
    for (u32 d = 0; d < N->world; d++) {
        std::vector<u8> mine(zeroed);
        for (u32 i = 0; i < n; i++) {
            if (node_home((const u8*)records + (u64)i * 128, N->world) == d) {
                memcpy(&mine[(u64)i * 128 + 16], (const u8*)records + (u64)i * 128 + 16, 64);
            }
        }
        const int st = load ? tbgpu_load_accounts(N->D[d].E, mine.data(), n) : tbgpu_upsert_accounts(N->D[d].E, mine.data(), n);
        if (st) return st;
    }
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

static int node_upsert_accounts_keep_flow(tbgpu* E, const void* records, uint32_t n) {
    return upsert_accounts(E, records, n, false, true);
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
