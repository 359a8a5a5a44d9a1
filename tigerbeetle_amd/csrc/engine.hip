// engine.hip — host side of the MI355X commit engine: the C ABI of include/tbgpu.h.
//
// One engine = one HIP device + one stream + HBM tables allocated at init (static allocation, as
// the reference's grooves: src/lsm/groove.zig:486-555).  A commit call is split into device passes
// of up to pass_events_max events / pass_batches_max prepares; each pass is three kernels
// (validate, resolve, replay — see pass.h) enqueued without host synchronisation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>
#include <map>
#include <functional>
#include <mutex>

#include "../../include/tbgpu.h"
#include "../../include/tbgpu_bench.h"
#include "../../include/tbgpu_shard.h"
#include "k_apply.h"
#include "k_flow.h"
#include "k_aux.h"
#include "k_replay.h"
#include "k_route.h"
#include "k_node.h"
#include "k_workload.h"
#include "k_evict.h"
#include "checksum.h"

static thread_local std::string g_err;

// Every device / pinned allocation and HIP event the library makes goes through these (counted):
// tbgpu.h promises none after tbgpu_init on the commit path, and tests/test_gpu_alloc.py holds the
// library to it with tbgpu_debug_allocations().
static std::atomic<uint64_t> g_allocs{0};
template <typename T>
static hipError_t tbMalloc(T** p, size_t bytes) {
    g_allocs++;
    return hipMalloc((void**)p, bytes);
}
template <typename T>
static hipError_t tbHostMalloc(T** p, size_t bytes, unsigned flags) {
    g_allocs++;
    return hipHostMalloc((void**)p, bytes, flags);
}
static hipError_t tbEventCreate(hipEvent_t* e) {
    g_allocs++;
    return hipEventCreate(e);
}
static hipError_t tbEventCreateWithFlags(hipEvent_t* e, unsigned flags) {
    g_allocs++;
    return hipEventCreateWithFlags(e, flags);
}

static int fail(int status, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int status, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return status;
}

#define HIPCK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "%s: %s (%s:%d)", #x,               \
                                          hipGetErrorString(e_), __FILE__, __LINE__);              \
    } while (0)

static u64 pow2_at_least(u64 v) {
    u64 c = 1;
    while (c < v) c <<= 1;
    return c;
}

#define PIPE_SLOTS 3
#define KCLOCK_SLOTS 2048  // profiled passes between two collects (a full ring is collected early)

enum { K_VALIDATE = 0, K_RESOLVE = 1, K_REPLAY = 2, K_CLEAR = 3, K_PASS = 4, K_APPLY = 5, K_COUNT = 6 };
// prof_mask bit without an event pair: the launch spans on the device clock only (TBGPU_PROF_SPANS).
#define K_SPANS 6

struct ProfilePair {
    int kind;
    hipEvent_t a, b;
};

struct TbNode;  // node.h: the multi-device engine (tbgpu_config.device_count > 1)

// Groove write-back buffers (tbgpu_checkpoint_delta / _async), every one allocated at tbgpu_init.
#define WB_IDS_MAX (1ULL << 20)  // listed ids (creates, direct balance writes) between write-backs
enum { WB_ACCOUNTS = 0, WB_SLOTS = 1, WB_PV = 2, WB_RECORDS = 3, WB_STATUS = 4, WB_ORDER = 5, WB_COUNT_WORDS = 8 };
struct WbBufs {
    u64 cap_t = 0;    // log positions per slice
    u64 cap_ids = 0;  // listed ids per chunk
    u64 cap_a = 0;    // accounts emitted per slice / chunk
    u32* d_bc = nullptr;          // [cap_t / DELTA_THREADS] live records per workgroup
    u64* d_base = nullptr;        // their exclusive prefix
    u8* d_out = nullptr;          // [cap_t] records
    u64* d_ids = nullptr;         // [cap_t][4] debit / credit account ids of the records
    u64* d_pv = nullptr;          // [cap_t][3] post / void records: {pending id, voided}
    u64* d_pairs = nullptr;       // [cap_t][2] posted pairs {pending timestamp, voided}
    u64* d_hids = nullptr;        // [cap_ids][2] listed ids
    u8* d_acc = nullptr;          // [cap_a] emitted accounts
    AccountBal* d_before = nullptr;
    u32* d_slots = nullptr;       // [account_cap] every slot one write-back covers
    AccountBal* d_cap = nullptr;  // [cap_a] asynchronous write-back: the balances captured at the bar
    u64* d_cnt = nullptr;         // [WB_COUNT_WORDS] WB_* counters
    u64* h_cnt = nullptr;         // pinned mirror
    hipStream_t stream = nullptr; // the asynchronous copy-out (DMA engine)
    hipEvent_t gathered = nullptr, done = nullptr;
    hipEvent_t read_done = nullptr;  // on the engine stream after a commit's validate (its PCIe reads)
    hipEvent_t captured = nullptr;   // on the engine stream after the bar's capture (the rest follows beside)
    bool inflight = false;
    // The copy-out in flight: regions (records, accounts, before, pairs) from HBM to the caller's
    // registered buffers, sent a slice per commit (wb_pump) once the gather's counts are known.
    bool copying = false, counts_known = false;
    bool tail = false;            // the gather's work beside the commits is not enqueued yet (wb_tail)
    u64 tail_pos0 = 0, tail_pos1 = 0, tail_ts0 = 0;
    const u8* src[4] = {};
    u8* dst[4] = {};
    u64 len[4] = {}, at[4] = {};
    u64 slice = 0;
    // Commits between an asynchronous write-back's start and its wait: this one's so far, and the
    // previous one's — the slices of the next copy-out are spread over that many commits (a bar
    // written back one bar behind: ~64; a replica writing back every 4 ops: 4).
    u32 calls = 0, calls_prev = 0;
    // Bound-sized copy-out: the regions are sent at their bounds (every log position, two accounts
    // per position plus the listed ids), so the first commit after the write-back starts sending
    // without waiting for the gather's counts; the bytes past the counts are never read by the
    // caller.  Taken when the previous write-back's objects filled their bounds to within ~1/8
    // and it saw two commits or more (a replica writing back every few ops), never for a whole
    // bar (far fewer accounts than two a transfer) nor every op (measured slower: the copy-out then
    // beside every commit instead of at the wait).
    bool bound = false, bound_ok = false;
    bool posted_late = false;     // bound mode: the posted pairs cross at the wait, by their count
    u64 bound_len[2] = {};        // bound mode: the transfers and accounts the regions were sized for
    u64 n_async = 0, n_bound = 0;  // tbgpu_stats write_backs_async / _bound
    bool staged_reads = false;    // the commit this slice follows read a staged body (no PCIe reads)
    tbgpu_delta_counts counts{};
    u8* out_t = nullptr;          // the in-flight write-back's caller buffers (sorted by the wait)
    u64* out_p = nullptr;
    std::vector<u64> ids_inflight;
};

struct tbgpu {
    tbgpu_config cfg{};
    TbNode* node = nullptr;  // set: this handle is a node engine; every call goes to node.h
    int device = 0;
    hipStream_t stream = nullptr;

    Tables T{};
    Globals* g = nullptr;
    u64 account_cap = 0, xidx_cap = 0, xlog_cap = 0;
    u64 log_next = 0;  // next free transfer-log position (host-owned)
    // Evicted transfers (k_evict.h): the Bloom filter of their ids, its mask, how many so far.
    u64* bloom = nullptr;
    u64 bloom_mask = 0;
    u64 evicted_total = 0;
    bool inplace_call = false;  // the call being enqueued commits its events in place (tbgpu_log_window)

    // Pass scratch.
    u32 pe_max = 0, pb_max = 0;
    u16* eflags = nullptr;
    u32 *info = nullptr, *dr = nullptr, *cr = nullptr, *ps = nullptr, *rs = nullptr;
    u32 *dep_list = nullptr, *dep_count = nullptr;
    u64 *amt = nullptr, *kid = nullptr, *kpid = nullptr;
    u64* dedup = nullptr;
    u64 dedup_cap = 0;
    u64* sum_shards = nullptr;
    UndoEntry* undo = nullptr;
    u32 undo_cap = 0;
    // Balance legs (k_apply.h); legs_ok = false: resolve applies every leg with atomics.
    bool legs_ok = false;
    u32 leg_shift = 0, leg_buckets = 0;
    u32* resolve_slow = nullptr;  // [pb_max] tb_resolve_lean's verdict per prepare of a legs pass
    bool lean_ok = true;          // legs passes run tb_resolve_lean first (TBGPU_NO_LEAN=1: tb_resolve alone)
    bool wb_bound_ok = true;      // bound-sized copy-outs allowed (TBGPU_WB_BOUND=0: counts always)
    bool wb_stage = true;         // prefetch stages registered bodies during a copy-out (TBGPU_WB_STAGE=0: never)
    u32 flow_launch = 0;          // tbgpu_bench_flow_launch (tests): tb_flow launched with this many workgroups
    u64* leg_w = nullptr;
    u32* leg_off = nullptr;
    u32* leg_tot = nullptr;  // [leg_buckets] legs per bucket of the current pass
    // Parallel ordered fallback (k_flow.h): create_transfers passes run tb_flow instead of
    // tb_replay while no balance was set directly (the post/void assert argument, k_replay.h).
    bool flow_ok = false;
    bool balances_set = false;
    u64 flow_capacity = 0;     // tb_flow workgroups the device holds at once (occupancy x CUs)
    u32 flow_occ = 0;          // tb_flow workgroups per CU (its registers and LDS)
    bool dev_registered = false;
    FlowArgs F{};

    // Host-path staging.
    u8* staging = nullptr;
    u32* results = nullptr;
    u32* reply_bytes = nullptr;
    u64* meta = nullptr;   // device: [meta_cap + 1] offsets then [meta_cap] timestamps
    u64 meta_cap = 0;
    u64* h_meta = nullptr; // pinned mirror
    Globals* h_globals = nullptr;  // pinned: read back by engine_sync
    u32* h_rb = nullptr;           // pinned: reply bytes of one host call
    u8* h_results = nullptr;       // pinned: the results of a host call of <= h_results_events events
    u64 h_results_events = 0;
    struct HostRegion {
        const u8* ptr;
        u64 bytes;
        const u8* dev;  // its device mapping
    };
    std::vector<HostRegion> host_regions;  // tbgpu_register_host
    // Pipelined host commits (tbgpu_commit_pipelined): PIPE_SLOTS chunks in flight.  Slot s has its
    // own staging area, call metadata and pinned reply arena; chunk c+1's bodies cross PCIe on
    // copy_stream while chunk c commits on `stream`.
    hipStream_t copy_stream = nullptr;
    struct PipeSlot {
        u8* staging = nullptr;      // device: pe_max events (slot 0 aliases `staging`)
        u64* meta = nullptr;        // device: offsets then timestamps
        u64* h_meta = nullptr;      // pinned mirror
        u8* h_reply = nullptr;      // pinned, mapped: [2] head {panic, commit_ts}, [meta_cap] reply bytes, results
        u8* d_reply = nullptr;      // its device mapping
        hipEvent_t start = nullptr, copied = nullptr, done = nullptr;
    } pipe[PIPE_SLOTS];
    u64* lookup_ids = nullptr;
    u8* lookup_out = nullptr;
    u8* lookup_found = nullptr;
    u32 lookup_cap = 0;
    // tbgpu_prefetch: the body of the prepare about to be committed, staged in HBM by DMA.
    u8* pf_staging = nullptr;     // BATCH_EVENTS_MAX events
    hipEvent_t pf_done = nullptr; // on copy_stream: the staging copy landed
    const void* pf_input = nullptr;  // valid for the next entry point only, if it is tbgpu_commit
    const void* pf_claim = nullptr;  // tbgpu_commit -> commit_host: the staged body it may take
    u32 pf_len = 0;
    u8 pf_op = 0;
    u32* d_status = nullptr;
    // A device panic left state the reference never reaches (it traps there): every entry point that
    // changes state refuses until tbgpu_reset.
    bool poisoned = false;

    u32 epoch = 0;
    bool dedup_force = true;  // the next pass clears the whole dedup set (init, reset, epoch wrap)
    u64 dedup_prev = 0;       // dedup entries the previous pass could have written (its mask + 1)
    u64 commit_ts = 0;       // exact after every synchronous call
    u64 last_batch_ts = 0;   // upper bound for async calls
    bool pending = false;    // an async call was enqueued and not yet synced
    u32 reply_seq = 0;       // one-prepare commits: the done word tb_reply_out writes last


    bool profile = false;
    bool kclock_off = false;
    u64 api_calls = 0;        // entry points called on this handle (a node skips redundant drains by it)
    u64* h_pub = nullptr;     // pinned staging word of a node's commit-timestamp push to this shard
    u32 legs_min = LEGS_MIN_EVENTS;
    u64 wall_khz = 0;  // device wall clock (flow phase timing)
    WbBufs wb;
    // Groove write-back snapshot (tbgpu_checkpoint_delta).
    u64* ckpt_bal = nullptr;  // balances at the previous write-back: the two planes of T.bal (tb_device.h BalView)
    u32* ckpt_mark = nullptr;        // per slot: the write-back epoch that last covered it
    u32 ckpt_epoch = 0;
    u64 ckpt_pos = 0;                // log position of the first transfer not yet written back
    u64 ckpt_ts = 0;                 // commit timestamp at the previous write-back
    bool ckpt_valid = false;         // false: the snapshot is the empty state (zeroes)
    bool ckpt_scan = false;          // accounts created that ckpt_ids lacks: diff the whole table next
    std::vector<u64> ckpt_ids;       // ids (lo, hi) of create_accounts events / direct balance writes since
    u32 prof_mask = ~0u;  // kernels timed when profiling (1 << K_*; tbgpu_bench_profile_mask)
    u32 ablate = 0;  // TBGPU_TIMING_KNOBS builds only
    std::vector<hipEvent_t> event_pool;
    size_t event_next = 0;
    std::vector<ProfilePair> prof;
    double prof_ms[K_COUNT] = {};
    u64 prof_n[K_COUNT] = {};
    // Launch spans on the device clock (tbgpu_stats.span_ms): a ring of KCLOCK_WORDS words per pass.
    u64* kclock = nullptr;
    u64* h_kclock = nullptr;        // pinned: the ring read back by prof_collect
    u32 kclock_next = 0;            // next ring slot
    std::vector<std::pair<u32, u32>> kclock_used;  // (slot, kernels launched: bit k) since the last collect
    double span_ms[3] = {};
    u64 span_n[3] = {};
    u64 passes = 0, events = 0;
    std::vector<double> pass_ms;  // device duration of every profiled pass (batch latency)

    hipEvent_t markers[16] = {};

    // Multi-GPU routing scratch (tbgpu_route_init).
    u32 route_world = 0;
    u64 route_events_max = 0;
    u8* r_home = nullptr;
    u32* r_block_counts = nullptr;
    u64 r_block_cap = 0;
    u64* r_words = nullptr;
    u64* r_meta = nullptr;    // device [meta_cap + 1] offsets then [meta_cap] timestamps
    u64* h_rmeta = nullptr;   // pinned mirror
};

// The write-back snapshot as a balance view (its two planes, like T.bal).
static inline BalView ckpt_view(const tbgpu* E) {
    return BalView{E->ckpt_bal, E->ckpt_bal ? E->ckpt_bal + 4 * E->account_cap : nullptr};
}

static void ckpt_note_ids(tbgpu* E, const u8* records, u64 n);

// Every entry point but tbgpu_prefetch starts here.  A body staged by tbgpu_prefetch belongs to the
// commit that comes next (src/vsr/replica.zig:3324-3662: prefetch(op) -> commit(op), nothing in
// between): any other call first drops it, so a reused message buffer can never be committed from a
// stale staging copy.  `mutates`: refused on a poisoned engine (a device panic, tbgpu.h).
static int api_enter(tbgpu* E, bool mutates) {
    E->pf_input = nullptr;
    E->api_calls++;
    if (mutates && E->poisoned) {
        return fail(TBGPU_STATUS_PANIC, "engine stopped by an earlier device panic (tbgpu_reset or tbgpu_deinit it)");
    }
    return TBGPU_STATUS_OK;
}
#define API_ENTER(E, mutates)                        \
    do {                                             \
        if (const int st_ = api_enter((E), (mutates))) return st_; \
    } while (0)

// Pinned reply arena of one pipeline slot: head {panic, commit_ts}, reply bytes per prepare, then
// the results of every event of the chunk (8 B each, the worst case).
static u64 pipe_reply_bytes(const tbgpu* E) { return 16 + E->meta_cap * 4 + (u64)E->pe_max * 8; }

// HIP events of the profiling pairs: a pool created at init (TBGPU_CONFIG_PROFILE); a call that
// would need more between two collects leaves the extra launches untimed rather than allocate.
#define PROF_EVENTS 8192

static int prof_begin(tbgpu* E, ProfilePair* p, int kind) {
    p->kind = -1;
    if (!E->profile || !(E->prof_mask & (1u << kind))) return 0;
    if (E->event_next + 2 > E->event_pool.size()) return 0;
    p->kind = kind;
    p->a = E->event_pool[E->event_next++];
    p->b = E->event_pool[E->event_next++];
    HIPCK(hipEventRecord(p->a, E->stream));
    return 0;
}

static int prof_end(tbgpu* E, ProfilePair* p) {
    if (!E->profile || p->kind < 0) return 0;
    HIPCK(hipEventRecord(p->b, E->stream));
    E->prof.push_back(*p);
    return 0;
}

static int prof_collect(tbgpu* E) {
    if (!E->kclock_used.empty()) {  // the stream has drained: every stamped span is final
        HIPCK(hipMemcpy(E->h_kclock, E->kclock, (u64)E->kclock_next * KCLOCK_WORDS * 8, hipMemcpyDeviceToHost));
        for (const auto& u : E->kclock_used) {
            const u64* w = E->h_kclock + (u64)u.first * KCLOCK_WORDS;
            for (u32 k = 0; k < 3; k++) {
                const u64* kw = w + k * KCLOCK_STRIDE;
                u64 end = 0;
                for (u32 q = 1; q <= KCLOCK_ENDS; q++) end = std::max(end, kw[q * KCLOCK_LINE]);
                if (k == 0) end = w[KCLOCK_STRIDE];  // validate: until resolve's start (pass.h)
                if (!((u.second >> k) & 1) || end < kw[0] || !E->wall_khz) continue;
                E->span_ms[k] += (double)(end - kw[0]) / E->wall_khz;
                E->span_n[k] += 1;
            }
        }
        E->kclock_used.clear();
        E->kclock_next = 0;
    }
    for (const ProfilePair& p : E->prof) {
        float ms = 0;
        HIPCK(hipEventElapsedTime(&ms, p.a, p.b));
        E->prof_ms[p.kind] += ms;
        E->prof_n[p.kind] += 1;
        if (p.kind == K_PASS) E->pass_ms.push_back(ms);
    }
    E->prof.clear();
    E->event_next = 0;
    return 0;
}

// ------------------------------------------------------------------------------------------------

static int engine_clear(tbgpu* E) {
    HIPCK(hipMemsetAsync(E->T.acct_hot, 0, E->account_cap * sizeof(AccountHot), E->stream));
    HIPCK(hipMemsetAsync(E->T.bal.lo, 0, E->account_cap * sizeof(AccountBal), E->stream));  // both planes
    HIPCK(hipMemsetAsync(E->T.acct_cold, 0, E->account_cap * sizeof(AccountCold), E->stream));
    HIPCK(hipMemsetAsync(E->T.account_mark, 0, E->account_cap * sizeof(u32), E->stream));
    HIPCK(hipMemsetAsync(E->T.xidx, 0, E->xidx_cap * sizeof(u64), E->stream));
    HIPCK(hipMemsetAsync(E->T.xdup, 0, E->xidx_cap, E->stream));
    HIPCK(hipMemsetAsync(E->T.xposted, 0, E->xlog_cap, E->stream));
    HIPCK(hipMemsetAsync(E->bloom, 0, (E->bloom_mask + 1) / 8, E->stream));
    E->log_next = 0;
    E->evicted_total = 0;
    HIPCK(hipMemsetAsync(E->g, 0, sizeof(Globals), E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    E->epoch = 0;
    E->dedup_force = true;
    E->commit_ts = 0;
    E->last_batch_ts = 0;
    E->pending = false;
    E->balances_set = false;
    return TBGPU_STATUS_OK;
}

// tb_flow synchronises its workgroups with a software grid barrier, so every workgroup of a launch
// must be resident at once.  The launch is an ordinary one (a cooperative launch makes the HIP
// runtime keep a queue whose teardown at process exit faults inside libhsa-runtime when rocprofv3 is
// loaded: tools/gpu/exit_probe.py), so residency is guaranteed here: the engines of
// this process on one device split its capacity (occupancy x CUs) and each launches at most its
// share — the persistent workgroups of every concurrent tb_flow then fit together, and every other
// kernel they share the device with runs to completion without waiting on them.  Every barrier wait
// is also bounded in wall time (PANIC_FLOW_STALL).
static std::mutex g_dev_mu;
static std::map<int, u32> g_dev_engines;

static void dev_register(tbgpu* E, bool add) {
    std::lock_guard<std::mutex> lock(g_dev_mu);
    if (add && !E->dev_registered) {
        g_dev_engines[E->device]++;
        E->dev_registered = true;
    } else if (!add && E->dev_registered) {
        if (--g_dev_engines[E->device] == 0) g_dev_engines.erase(E->device);
        E->dev_registered = false;
    }
}

// The co-residency tb_flow relies on, checked once at init (tbgpu.h "Device exclusivity"): a grid of
// tb_flow's shape (workgroups, threads, LDS) whose workgroups each arrive at a counter and wait until
// every one has arrived, for at most `deadline` ticks of the device clock.  A workgroup that gave up
// sets *failed.  On a device this process has to itself every workgroup is resident at once and the
// probe takes microseconds.
__global__ __launch_bounds__(FLOW_THREADS) void tb_residency_probe(u32* counter, u32 total, u64 deadline, u32* failed) {
    extern __shared__ u32 s_probe_lds[];  // sized like tb_flow's LDS: the same residency per CU
    if (threadIdx.x != 0) return;
    s_probe_lds[0] = 0;
    atomicAdd(counter, 1u);
    const u64 t0 = wall_clock64();
    while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total) {
        if (wall_clock64() - t0 > deadline) {
            atomicOr(failed, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

static int residency_probe(tbgpu* E, u32 grid) {
    u32* d = nullptr;
    HIPCK(tbMalloc(&d, 8));
    hipFuncAttributes attr{};
    size_t lds = 0;
    if (hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&tb_flow)) == hipSuccess) lds = attr.sharedSizeBytes;
    // The probe uses almost no registers, so more of its workgroups than tb_flow's can share a CU.  The
    // property to prove is that the CUs tb_flow's grid needs (grid / tb_flow's occupancy) are free: so
    // the probe launches that many CUs' worth of ITS workgroups (grid x its occupancy / tb_flow's), all
    // of which must become resident together.
    lds = std::max<size_t>(lds, 4);
    int probe_occ = 0;
    if (E->flow_occ &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&probe_occ, reinterpret_cast<const void*>(&tb_residency_probe),
                                                     FLOW_THREADS, lds) == hipSuccess &&
        probe_occ > (int)E->flow_occ) {
        grid = (u32)(((u64)grid * (u64)probe_occ + E->flow_occ - 1) / E->flow_occ);
    }
    int st = TBGPU_STATUS_OK;
    u32 h[2] = {0, 0};
    hipError_t e = hipMemsetAsync(d, 0, 8, E->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(tb_residency_probe, dim3(grid), dim3(FLOW_THREADS), std::max<size_t>(lds, 4), E->stream, d, grid,
                           (u64)200 * E->wall_khz, d + 1);  // 200 ms
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, E->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(E->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "tbgpu_init: residency probe: %s", hipGetErrorString(e));
    if (h[1]) {
        st = fail(TBGPU_STATUS_DEVICE,
                  "tbgpu_init: device %d is not exclusive: %u workgroups of the ordered fallback's grid could not be "
                  "resident together (another process or kernel holds its CUs; tbgpu.h \"Device exclusivity\")",
                  E->device, grid);
    }
    return st;
}

static u32 flow_grid(tbgpu* E) {
    u32 engines = 1;
    {
        std::lock_guard<std::mutex> lock(g_dev_mu);
        auto it = g_dev_engines.find(E->device);
        if (it != g_dev_engines.end()) engines = std::max<u32>(1, it->second);
    }
    return (u32)std::max<u64>(1, std::min<u64>(E->F.grid, E->flow_capacity / engines));
}

// node.h entry points (defined at the end of this file).
static int node_api_init(const tbgpu_config* config, tbgpu_t** out);
static void node_free(TbNode* N);
static int node_api_reset(TbNode* N);
static int node_commit_pipelined(TbNode* N, u8 op, u32 n, const u64* ts, const void* const* inputs, const u32* input_lens,
                                 void* const* outputs, u32* out_lens, u32 chunk, double* latency_ms);
static int node_api_commit(TbNode* N, u8 op, u64 timestamp, const void* input, u32 input_len, void* output,
                           u32 output_cap, u32* out_len);
static int node_sync(TbNode* N);
static u64 node_commit_ts(TbNode* N);
static int node_api_set_balances(TbNode* N, u64 id_lo, u64 id_hi, const u64 b[8]);
static int node_api_export(TbNode* N, int what, void* out, u64 cap, u64* count);
static int node_api_evict(TbNode* N, uint64_t keep, uint64_t* evicted);
static int node_api_checkpoint_delta_async(TbNode* N, void* accounts_out, void* accounts_before_out, u64 accounts_cap,
                                           void* transfers_out, u64 transfers_cap, u64* posted_out, u64 posted_cap);
static int node_api_checkpoint_delta_wait(TbNode* N, tbgpu_delta_counts* counts);
static int node_api_maybe_cold(TbNode* N, const uint64_t* ids, uint32_t n, uint8_t* cold);
static int node_api_checkpoint_delta(TbNode* N, void* accounts_out, void* accounts_before_out, u64 accounts_cap,
                                     void* transfers_out, u64 transfers_cap, u64* posted_out, u64 posted_cap,
                                     tbgpu_delta_counts* counts);
static int node_api_get_stats(TbNode* N, tbgpu_stats* s);
static void node_reset_stats(TbNode* N);
static u32 node_world(TbNode* N);
static tbgpu* node_engine(TbNode* N, u32 d);
static int node_api_register_host(TbNode* N, void* ptr, u64 bytes);
static int node_api_unregister_host(TbNode* N, void* ptr);
static int node_fetch(TbNode* N, bool accounts, const u64* ids, u32 n, u8* out, u8* found);
static int node_api_accounts_in(TbNode* N, const void* records, u32 n, bool load);
static int node_api_transfers_in(TbNode* N, const void* records, const u8* state, u32 n, bool load);
static int node_api_set_commit_timestamp(TbNode* N, u64 timestamp);

extern "C" int tbgpu_init(const tbgpu_config* config, tbgpu_t** out) {
    if (config && config->device_count > 1) return node_api_init(config, out);
    *out = nullptr;
    if (!config || config->accounts_max == 0 || config->transfers_max == 0 || config->pass_events_max == 0 ||
        config->pass_batches_max == 0) {
        return fail(TBGPU_STATUS_INVALID, "tbgpu_init: invalid config");
    }
    if (config->accounts_max > (1ULL << 31) || config->transfers_max > (1ULL << 31)) {
        return fail(TBGPU_STATUS_INVALID, "tbgpu_init: table capacity above 2^31 objects per device");
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        return fail(TBGPU_STATUS_DEVICE, "tbgpu_init: no HIP device visible");
    }
    if (config->device < 0 || config->device >= ndev) {
        return fail(TBGPU_STATUS_INVALID, "tbgpu_init: device %d out of range (%d devices)", config->device, ndev);
    }
    tbgpu* E = new tbgpu();
    E->cfg = *config;
    E->device = config->device;
    E->profile = (config->flags & TBGPU_CONFIG_PROFILE) != 0;
#ifdef TBGPU_TIMING_KNOBS
    if (const char* ab = getenv("TBGPU_ABLATE")) E->ablate = (u32)strtoul(ab, nullptr, 0);  // timing experiments only
    E->kclock_off = getenv("TBGPU_NO_KCLOCK") != nullptr;  // timing experiments: no launch-span stamps
#endif
    int st = TBGPU_STATUS_OK;
#define INIT_CK(x)                                                                                 \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            st = fail(TBGPU_STATUS_DEVICE, "%s: %s", #x, hipGetErrorString(e_));                   \
            tbgpu_deinit(E);                                                                       \
            return st;                                                                             \
        }                                                                                          \
    } while (0)
    INIT_CK(hipSetDevice(E->device));
    INIT_CK(hipStreamCreateWithFlags(&E->stream, hipStreamNonBlocking));
    dev_register(E, true);

    // Account table slots per account (load factor <= 1/2).  4 slots shorten the probes (validate
    // -2..10 % at C2, box to box) but double the legs buckets (tb_apply_legs +40 %): a net loss.
    // TBGPU_ACCOUNT_SLOTS overrides (experiments).
    u64 load = 2;
#ifdef TBGPU_TIMING_KNOBS
    if (const char* s = getenv("TBGPU_ACCOUNT_SLOTS")) load = std::max<u64>(2, strtoull(s, nullptr, 0));
#endif
    E->account_cap = pow2_at_least(std::max<u64>(load * config->accounts_max, 1024));
    // The index is sized for 2x the log so tombstones of withdrawn speculative inserts leave room.
    E->xlog_cap = std::max<u64>(config->transfers_max, 1024);
    E->xidx_cap = pow2_at_least(std::max<u64>(2 * E->xlog_cap, 2048));
    E->pe_max = config->pass_events_max;
    E->pb_max = config->pass_batches_max;
    if (const char* v = getenv("TBGPU_NO_LEAN")) E->lean_ok = atoi(v) == 0;
    if (const char* v = getenv("TBGPU_WB_BOUND")) E->wb_bound_ok = atoi(v) != 0;
    if (const char* v = getenv("TBGPU_WB_STAGE")) E->wb_stage = atoi(v) != 0;
    E->dedup_cap = pow2_at_least(std::max<u64>(4ULL * E->pe_max, 64));
    E->undo_cap = 4 * (BATCH_EVENTS_MAX + 1);
    E->meta_cap = std::max<u64>(E->pb_max, 1 << 16);
    E->lookup_cap = 1 << 16;
    // Legs buckets: about LEG_BUCKETS_PREF buckets, at most LEG_SLOTS_MAX slots (LDS) each.
    {
        u32 shift = 0;
        while ((E->account_cap >> shift) > LEG_BUCKETS_PREF && (1u << shift) < LEG_SLOTS_MAX) shift++;
        E->leg_shift = shift;
        E->leg_buckets = (u32)(E->account_cap >> shift);
        E->legs_ok = E->leg_buckets <= LEG_BUCKETS_MAX;
    }

    size_t free_b = 0, total_b = 0;
    INIT_CK(hipMemGetInfo(&free_b, &total_b));
    const u64 need = E->account_cap * (sizeof(Account) + 4) + E->xlog_cap * (sizeof(Transfer) + 1) +
                     E->xidx_cap * (sizeof(u64) + 1) +
                     (u64)E->pe_max * (4 * 4 + 8 * 4 + 128 * PIPE_SLOTS + 8 + 4) + E->dedup_cap * 8;
    if (need > free_b) {
        st = fail(TBGPU_STATUS_INVALID, "tbgpu_init: needs %llu bytes of HBM, %llu free",
                  (unsigned long long)need, (unsigned long long)free_b);
        tbgpu_deinit(E);
        return st;
    }

    INIT_CK(tbMalloc(&E->T.acct_hot, E->account_cap * sizeof(AccountHot)));
    INIT_CK(tbMalloc(&E->T.bal.lo, E->account_cap * sizeof(AccountBal)));  // low plane, then high plane
    E->T.bal.hi = E->T.bal.lo + 4 * E->account_cap;
    INIT_CK(tbMalloc(&E->T.acct_cold, E->account_cap * sizeof(AccountCold)));
    INIT_CK(tbMalloc(&E->T.account_mark, E->account_cap * sizeof(u32)));
    INIT_CK(tbMalloc(&E->T.xidx, E->xidx_cap * sizeof(u64)));
    INIT_CK(tbMalloc(&E->T.xdup, E->xidx_cap));
    INIT_CK(tbMalloc(&E->T.xlog, E->xlog_cap * sizeof(Transfer)));
    INIT_CK(tbMalloc(&E->T.xposted, E->xlog_cap));
    INIT_CK(tbMalloc(&E->g, sizeof(Globals)));
    {
        // The evicted-id filter: 8 bits per log position (about 2 % false positives at one log's worth
        // of evicted ids with 3 hashes; more evictions raise it — extra forest lookups, never errors).
        const u64 bits = std::min<u64>(1ULL << 34, pow2_at_least(std::max<u64>(1ULL << 16, 8 * E->xlog_cap)));
        E->bloom_mask = bits - 1;
        INIT_CK(tbMalloc(&E->bloom, bits / 8));
    }
    {
        // tb_flow: 1024-thread workgroups, all resident (see flow_grid).
        hipDeviceProp_t prop;
        int occ = 0;
        if (hipGetDeviceProperties(&prop, E->device) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&tb_flow), FLOW_THREADS, 0) ==
                hipSuccess &&
            occ >= 1) {
            // A quarter of the CUs at most: co-residency of the grid then holds even with a few
            // engines (processes) sharing the device, each with a tb_flow in flight.
            E->F.grid = (u32)std::max(1, std::min(prop.multiProcessorCount / 4, 64));
#ifdef TBGPU_TIMING_KNOBS
            if (const char* gs = getenv("TBGPU_FLOW_GRID")) E->F.grid = std::max(1u, std::min(E->F.grid, (u32)atoi(gs)));
#endif
            // tb_flow's grid barrier needs every workgroup resident: the grid is at most occupancy x
            // CUs, shared among the engines of this process on the device (flow_grid).
            E->flow_capacity = (u64)occ * prop.multiProcessorCount;
            E->flow_occ = (u32)occ;
            E->F.grid = (u32)std::min<u64>(E->F.grid, E->flow_capacity);
            E->F.grid_alloc = E->F.grid;
            int khz = 0;
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, E->device) != hipSuccess) khz = 0;
            khz = std::max(khz, 100000);  // s_memrealtime: 100 MHz on gfx9 parts; never trust a lower figure
            E->F.stall_ticks = 60ULL * 1000ULL * (u64)khz;  // 60 s
            if (const char* ms = getenv("TBGPU_STALL_MS")) {  // diagnostics: a shorter bound on every wait
                E->F.stall_ticks = std::max<u64>(1, strtoull(ms, nullptr, 10)) * (u64)khz;
            }
            E->wall_khz = (u64)khz;
            if (getenv("TBGPU_DEBUG")) {  // diagnostics only: changes no behaviour
                fprintf(stderr, "tbgpu: flow grid %u, occupancy %d, wall clock %d kHz, stall ticks %llu\n", E->F.grid,
                        occ, khz, (unsigned long long)E->F.stall_ticks);
            }
            E->flow_ok = E->pb_max <= FLOW_NB_MAX && !(config->flags & TBGPU_CONFIG_SEQUENTIAL_FALLBACK);
#ifdef TBGPU_TIMING_KNOBS
            if (getenv("TBGPU_NO_FLOW")) E->flow_ok = false;
#endif
        }
    }
    E->T.account_mask = E->account_cap - 1;
    E->T.xidx_mask = E->xidx_cap - 1;
    E->T.xlog_cap = E->xlog_cap;
    E->T.g = E->g;

    const u64 pe = E->pe_max;
    INIT_CK(tbMalloc(&E->info, pe * 4));
    INIT_CK(tbMalloc(&E->eflags, pe * 2));
    INIT_CK(tbMalloc(&E->dr, pe * 4));
    INIT_CK(tbMalloc(&E->cr, pe * 4));
    INIT_CK(tbMalloc(&E->ps, pe * 4));
    INIT_CK(tbMalloc(&E->rs, pe * 4));
    INIT_CK(tbMalloc(&E->dep_list, pe * 4));
    INIT_CK(tbMalloc(&E->dep_count, (u64)E->pb_max * 4));
    INIT_CK(tbMalloc(&E->amt, pe * 16));
    INIT_CK(tbMalloc(&E->kid, pe * 8));
    INIT_CK(tbMalloc(&E->kpid, pe * 8));
    INIT_CK(tbMalloc(&E->dedup, E->dedup_cap * 8));
    INIT_CK(tbMalloc(&E->sum_shards, SUM_WORDS * 8));
    INIT_CK(tbMalloc(&E->undo, (u64)E->undo_cap * sizeof(UndoEntry)));
    if (E->legs_ok) {
        INIT_CK(tbMalloc(&E->resolve_slow, (u64)E->pb_max * 4));
        INIT_CK(tbMalloc(&E->leg_w, pe * 2 * 8));
        INIT_CK(tbMalloc(&E->leg_off, (u64)std::min<u32>(E->pb_max, LEG_PREPARES_MAX) * (E->leg_buckets + 1) * 4));
        INIT_CK(tbMalloc(&E->leg_tot, ((u64)E->leg_buckets + 1) * 4));
        INIT_CK(hipMemset(E->leg_tot, 0, ((u64)E->leg_buckets + 1) * 4));
    }
    if (E->flow_ok) {
        FlowArgs& F = E->F;
        INIT_CK(tbMalloc(&F.f_pe, pe * 4));
        INIT_CK(tbMalloc(&F.f_batch, pe * 4));
        INIT_CK(tbMalloc(&F.f_len, pe * 4));
        INIT_CK(tbMalloc(&F.need, pe * 4));
        INIT_CK(tbMalloc(&F.nsucc, pe * 4));
        INIT_CK(tbMalloc(&F.queue, pe * 4));
        INIT_CK(tbMalloc(&F.uflags, pe * 4));
        INIT_CK(tbMalloc(&F.nacct, pe * 4));
        INIT_CK(tbMalloc(&F.rpos, pe * 4));
        INIT_CK(tbMalloc(&F.succ, pe * 4 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.run, pe * sizeof(RunEntry) * FLOW_RMAX));
        for (int k = 0; k < 2; k++) {
            INIT_CK(tbMalloc(&F.keys[k], pe * 4 * FLOW_RMAX));
            INIT_CK(tbMalloc(&F.vals[k], pe * 4 * FLOW_RMAX));
        }
        INIT_CK(tbMalloc(&F.hist, (u64)F.grid * 256 * 4));
        INIT_CK(tbMalloc(&F.words, FW_WORDS * 4));
        INIT_CK(tbMalloc(&F.undo, pe * 4 * sizeof(UndoEntry)));
        INIT_CK(tbMalloc(&F.b_st, pe * 4));
        INIT_CK(tbMalloc(&F.b_vd, pe));
        INIT_CK(tbMalloc(&F.b_vc, pe));
        INIT_CK(tbMalloc(&F.b_amt, pe * 8 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.b_meta, pe * 4 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.b_blk, (u64)F.grid * 5 * 8));
        INIT_CK(tbMalloc(&F.b_qd, pe * 4));
        INIT_CK(tbMalloc(&F.b_qc, pe * 4));
        INIT_CK(tbMalloc(&F.b_head, pe * 4 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.b_xy, pe * 16 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.b_ex, pe * 16 * FLOW_RMAX));
        INIT_CK(tbMalloc(&F.b_rec, pe * sizeof(SweepRec)));
        INIT_CK(tbMalloc(&F.b_vw, pe * 4));
        F.walk = (config->flags & TBGPU_CONFIG_SWEEP_WINDOW) ? 0u : 1u;
        F.walk_merge = WALK_MERGE_DEFAULT;

        F.bounds_rounds_max = FLOW_BOUNDS_ROUNDS_MAX;
        F.sweep_min = (config->flags & TBGPU_CONFIG_SWEEP_OFF) ? 0u
                      : (config->flags & TBGPU_CONFIG_SWEEP_EARLY) ? 0xFFFFFFFFu
                                                                   : FLOW_SWEEP_MIN;
    }
    INIT_CK(tbMalloc(&E->staging, pe * 128));
    INIT_CK(tbMalloc(&E->results, pe * 8));
    INIT_CK(tbMalloc(&E->reply_bytes, E->meta_cap * 4));
    INIT_CK(tbMalloc(&E->meta, (2 * E->meta_cap + 1) * 8));
    INIT_CK(tbHostMalloc(&E->h_meta, (2 * E->meta_cap + 1) * 8, hipHostMallocDefault));
    INIT_CK(tbHostMalloc(&E->h_globals, sizeof(Globals), hipHostMallocDefault));
    INIT_CK(tbHostMalloc(&E->h_rb, E->meta_cap * 4, hipHostMallocDefault));
    E->h_results_events = std::min<u64>(E->pe_max, 1ULL << 16);
    INIT_CK(tbHostMalloc(&E->h_results, E->h_results_events * 8, hipHostMallocDefault));
    INIT_CK(hipStreamCreateWithFlags(&E->copy_stream, hipStreamNonBlocking));
    for (int k = 0; k < PIPE_SLOTS; k++) {
        tbgpu::PipeSlot& S = E->pipe[k];
        if (k == 0) S.staging = E->staging;
        else INIT_CK(tbMalloc(&S.staging, pe * 128));
        INIT_CK(tbMalloc(&S.meta, (2 * E->meta_cap + 1) * 8));
        INIT_CK(tbHostMalloc(&S.h_meta, (2 * E->meta_cap + 1) * 8, hipHostMallocDefault));
        INIT_CK(tbHostMalloc(&S.h_reply, pipe_reply_bytes(E) + 64, hipHostMallocMapped));  // + the done word
        memset(S.h_reply + pipe_reply_bytes(E), 0, 64);
        INIT_CK(hipHostGetDevicePointer((void**)&S.d_reply, S.h_reply, 0));
        INIT_CK(tbEventCreate(&S.start));
        INIT_CK(tbEventCreate(&S.copied));
        INIT_CK(tbEventCreate(&S.done));
    }
    INIT_CK(tbMalloc(&E->lookup_ids, (u64)E->lookup_cap * 16));
    INIT_CK(tbMalloc(&E->lookup_out, (u64)E->lookup_cap * 128));
    INIT_CK(tbMalloc(&E->lookup_found, E->lookup_cap));
    INIT_CK(tbMalloc(&E->d_status, 16));
    INIT_CK(tbMalloc(&E->pf_staging, (u64)BATCH_EVENTS_MAX * 128));
    INIT_CK(tbEventCreateWithFlags(&E->pf_done, hipEventDisableTiming));
    {  // groove write-back (tbgpu_checkpoint_delta*): snapshot, marks and one slice of buffers
        WbBufs& W = E->wb;
        W.cap_t = std::max<u64>(1, std::min<u64>(E->xlog_cap, std::max<u64>(pe, 64ULL * BATCH_EVENTS_MAX)));
        W.cap_ids = WB_IDS_MAX;
        W.cap_a = std::min<u64>(E->account_cap, std::max<u64>(2 * W.cap_t, W.cap_ids));
        const u64 nb = (W.cap_t + DELTA_THREADS - 1) / DELTA_THREADS;
        INIT_CK(tbMalloc(&E->ckpt_bal, E->account_cap * sizeof(AccountBal)));
        INIT_CK(tbMalloc(&E->ckpt_mark, E->account_cap * sizeof(u32)));
        INIT_CK(hipMemset(E->ckpt_mark, 0, E->account_cap * sizeof(u32)));
        INIT_CK(tbMalloc(&W.d_bc, nb * 4));
        INIT_CK(tbMalloc(&W.d_base, nb * 8));
        INIT_CK(tbMalloc(&W.d_out, W.cap_t * 128));
        INIT_CK(tbMalloc(&W.d_ids, W.cap_t * 32));
        INIT_CK(tbMalloc(&W.d_pv, W.cap_t * 24));
        INIT_CK(tbMalloc(&W.d_pairs, W.cap_t * 16));
        INIT_CK(tbMalloc(&W.d_hids, W.cap_ids * 16));
        INIT_CK(tbMalloc(&W.d_acc, W.cap_a * 128));
        INIT_CK(tbMalloc(&W.d_before, W.cap_a * sizeof(AccountBal)));
        INIT_CK(tbMalloc(&W.d_slots, E->account_cap * 4));
        INIT_CK(tbMalloc(&W.d_cap, W.cap_a * sizeof(AccountBal)));
        INIT_CK(tbMalloc(&W.d_cnt, WB_COUNT_WORDS * 8));
        INIT_CK(tbHostMalloc(&W.h_cnt, WB_COUNT_WORDS * 8, hipHostMallocDefault));
        {   // the copy-out and the work beside the commits: the lowest priority, so the commits' kernels
            // are dispatched first
            int least = 0, greatest = 0;
            INIT_CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            INIT_CK(hipStreamCreateWithPriority(&W.stream, hipStreamNonBlocking, least));
        }
        INIT_CK(tbEventCreateWithFlags(&W.gathered, hipEventDisableTiming));
        INIT_CK(tbEventCreateWithFlags(&W.done, hipEventDisableTiming));
        INIT_CK(tbEventCreateWithFlags(&W.read_done, hipEventDisableTiming));
        INIT_CK(tbEventCreateWithFlags(&W.captured, hipEventDisableTiming));
    }
    INIT_CK(tbHostMalloc(&E->h_pub, 8, hipHostMallocDefault));
    INIT_CK(tbMalloc(&E->kclock, (u64)KCLOCK_SLOTS * KCLOCK_WORDS * 8));
    INIT_CK(tbHostMalloc(&E->h_kclock, (u64)KCLOCK_SLOTS * KCLOCK_WORDS * 8, hipHostMallocDefault));
    for (int i = 0; i < 16; i++) INIT_CK(tbEventCreate(&E->markers[i]));
    if (E->profile) {
        E->event_pool.resize(PROF_EVENTS);
        for (auto& ev : E->event_pool) INIT_CK(tbEventCreate(&ev));
    }
#undef INIT_CK
    st = engine_clear(E);
    if (st == TBGPU_STATUS_OK && E->flow_ok) st = residency_probe(E, flow_grid(E));
    if (st) {
        tbgpu_deinit(E);
        return st;
    }
    *out = E;
    return TBGPU_STATUS_OK;
}

extern "C" void tbgpu_deinit(tbgpu_t* E) {
    if (E && E->node) {
        node_free(E->node);
        delete E;
        return;
    }
    if (!E) return;
    (void)hipSetDevice(E->device);
    dev_register(E, false);
    if (E->stream) (void)hipStreamSynchronize(E->stream);
    void* bufs[] = {E->ckpt_bal, E->ckpt_mark, E->T.acct_hot, E->T.bal.lo, E->T.acct_cold, E->T.account_mark, E->T.xidx, E->T.xdup, E->T.xlog,
                    E->T.xposted, E->g, E->bloom, E->info, E->eflags, E->dr,
                    E->cr, E->ps, E->rs, E->dep_list, E->dep_count, E->amt, E->kid, E->kpid, E->dedup,
                    E->sum_shards, E->undo, E->staging, E->results, E->reply_bytes, E->meta,
                    E->lookup_ids, E->lookup_out, E->lookup_found, E->d_status, E->pf_staging, E->kclock, E->r_home,
                    E->wb.d_bc, E->wb.d_base, E->wb.d_out, E->wb.d_ids, E->wb.d_pv, E->wb.d_pairs, E->wb.d_hids,
                    E->wb.d_acc, E->wb.d_before, E->wb.d_slots, E->wb.d_cap, E->wb.d_cnt,
                    E->r_block_counts, E->r_words, E->r_meta, E->resolve_slow, E->leg_w, E->leg_off, E->leg_tot,
                    E->F.f_pe, E->F.f_batch, E->F.f_len, E->F.need, E->F.nsucc, E->F.queue, E->F.uflags, E->F.nacct, E->F.rpos, E->F.succ,
                    E->F.run, E->F.keys[0], E->F.keys[1], E->F.vals[0], E->F.vals[1], E->F.hist, E->F.words, E->F.undo,
                    E->F.b_st, E->F.b_vd, E->F.b_vc, E->F.b_amt, E->F.b_meta, E->F.b_blk,
                    E->F.b_qd, E->F.b_qc, E->F.b_head, E->F.b_xy, E->F.b_ex, E->F.b_rec, E->F.b_vw};
    for (void* p : bufs) if (p) (void)hipFree(p);
    for (int k = 0; k < PIPE_SLOTS; k++) {
        tbgpu::PipeSlot& S = E->pipe[k];
        if (k > 0 && S.staging) (void)hipFree(S.staging);
        if (S.meta) (void)hipFree(S.meta);
        if (S.h_meta) (void)hipHostFree(S.h_meta);
        if (S.h_reply) (void)hipHostFree(S.h_reply);
        for (hipEvent_t e : {S.start, S.copied, S.done}) if (e) (void)hipEventDestroy(e);
    }
    if (E->copy_stream) (void)hipStreamDestroy(E->copy_stream);
    if (E->h_meta) (void)hipHostFree(E->h_meta);
    if (E->h_globals) (void)hipHostFree(E->h_globals);
    if (E->h_rb) (void)hipHostFree(E->h_rb);
    if (E->h_results) (void)hipHostFree(E->h_results);
    if (E->h_rmeta) (void)hipHostFree(E->h_rmeta);
    if (E->h_kclock) (void)hipHostFree(E->h_kclock);
    if (E->h_pub) (void)hipHostFree(E->h_pub);
    if (E->wb.h_cnt) (void)hipHostFree(E->wb.h_cnt);
    if (E->wb.stream) {
        (void)hipStreamSynchronize(E->wb.stream);
        (void)hipStreamDestroy(E->wb.stream);
    }
    if (E->wb.gathered) (void)hipEventDestroy(E->wb.gathered);
    if (E->wb.done) (void)hipEventDestroy(E->wb.done);
    if (E->wb.read_done) (void)hipEventDestroy(E->wb.read_done);
    if (E->wb.captured) (void)hipEventDestroy(E->wb.captured);
    for (hipEvent_t e : E->event_pool) (void)hipEventDestroy(e);
    if (E->pf_done) (void)hipEventDestroy(E->pf_done);
    for (int i = 0; i < 16; i++) if (E->markers[i]) (void)hipEventDestroy(E->markers[i]);
    if (E->stream) (void)hipStreamDestroy(E->stream);
    delete E;
}

extern "C" int tbgpu_reset(tbgpu_t* E) {
    API_ENTER(E, false);
    if (E->node) return node_api_reset(E->node);
    E->pf_input = E->pf_claim = nullptr;
    E->poisoned = false;
    HIPCK(hipSetDevice(E->device));
    if (E->wb.inflight) {  // its copy-out finishes; its results are dropped with the state
        HIPCK(hipStreamSynchronize(E->stream));  // its gather
        HIPCK(hipStreamSynchronize(E->wb.stream));
        E->wb.inflight = E->wb.copying = E->wb.counts_known = E->wb.tail = false;
    }
    E->ckpt_valid = false;
    E->ckpt_scan = false;
    std::vector<u64>().swap(E->ckpt_ids);
    return engine_clear(E);
}

// Read back commit_timestamp and the panic word after the stream drained.
static int engine_sync(tbgpu* E) {
    // One round trip: the globals come back on the stream, behind the call's kernels.
    HIPCK(hipMemcpyAsync(E->h_globals, E->g, sizeof(Globals), hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    const Globals g = *E->h_globals;
    E->commit_ts = g.commit_timestamp;
    E->pending = false;
    int st = prof_collect(E);
    if (st) return st;
    if (g.panic) {
        E->poisoned = true;
        return fail(TBGPU_STATUS_PANIC, "device panic 0x%llx (the reference would have trapped)", (unsigned long long)g.panic);
    }
    return TBGPU_STATUS_OK;
}

// Enqueue every pass of one call.  meta (device) already holds the call's offsets/timestamps.
// Routed mode (a shard of a multi-GPU pass): events carry their execute timestamps, codes = dense
// result codes instead of sparse replies, cert_ext = the router's certificate.
static int enqueue_call(tbgpu* E, u8 op, u32 nb, const u64* h_off, const u8* events_dev, u32* results_dev,
                        u32* reply_bytes_dev, bool routed = false, u8* codes = nullptr, u32 cert_ext = 0,
                        const u8* events_src = nullptr, const u64* d_meta = nullptr,
                        const OwnerLegArgs* owner = nullptr, const u64* inline_meta = nullptr,
                        const NodeImport* imp = nullptr, const u64* ev_ts = nullptr) {
    const u64* d_off = d_meta ? d_meta : E->meta;
    const u64* d_ts = d_off + (nb + 1);
    u32 b0 = 0;
    while (b0 < nb) {
        u32 b1 = b0;
        while (b1 < nb && b1 - b0 < E->pb_max && h_off[b1 + 1] - h_off[b0] <= E->pe_max) b1++;
        if (b1 == b0) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
        const u64 n = h_off[b1] - h_off[b0];
        E->epoch++;
        if (E->epoch == 0) {  // wrapped: clear stale balancing marks
            HIPCK(hipMemsetAsync(E->T.account_mark, 0, E->account_cap * sizeof(u32), E->stream));
            E->epoch = 1;
            E->dedup_force = true;
        }
        PassArgs P{};
        P.op = op;
        P.epoch = E->epoch;
        P.b0 = b0;
        P.b1 = b1;
        P.e0 = h_off[b0];
        P.n = (u32)n;
        P.batch_off = d_off;
        P.batch_ts = d_ts;
        P.events = events_dev;
        P.events_src = events_src;
        P.results = results_dev;
        P.reply_bytes = reply_bytes_dev;
        P.info = E->info;
        P.eflags = E->eflags;
        P.dr = E->dr;
        P.cr = E->cr;
        P.ps = E->ps;
        P.rs = E->rs;
        P.amt = E->amt;
        P.amt_hi = E->amt + E->pe_max;
        P.kid = E->kid;
        P.kpid = E->kpid;
        P.dep_list = E->dep_list;
        P.dep_count = E->dep_count;
        P.dedup = E->dedup;
        P.dedup_mask = std::min<u64>(pow2_at_least(std::max<u64>(4 * n, 64)), E->dedup_cap) - 1;
        P.sum_shards = E->sum_shards;
        P.pass_words = E->sum_shards;
        P.log_base = E->log_next;
        P.T = E->T;
        P.ablate = E->ablate;
        P.routed = routed ? 1 : 0;
        P.codes = codes;
        P.cert_ext = cert_ext;
        P.seq_pv = E->balances_set ? 1u : 0u;
        P.ev_ts = ev_ts;
        P.inplace = E->inplace_call ? 1u : 0u;
        // Legs pay a fixed ~30 us (one workgroup per bucket, LDS sums) that no-return atomics in
        // the resolve kernel (~20 G/s) only cost beyond ~LEGS_MIN_EVENTS events: the replica's
        // one-prepare commits take the atomics.
        P.legs = (op == OP_CREATE_TRANSFERS && E->legs_ok && b1 - b0 <= LEG_PREPARES_MAX && n >= E->legs_min &&
                  !(E->ablate & ABL_LEGS) && !owner) ? 1 : 0;
        P.apply_late = (op == OP_CREATE_TRANSFERS && !P.legs) ? 1 : 0;
        P.leg_shift = E->leg_shift;
        P.leg_buckets = E->leg_buckets;
        P.resolve_slow = P.legs && E->lean_ok ? E->resolve_slow : nullptr;
        P.leg_w = E->leg_w;
        P.leg_off = E->leg_off;
        P.leg_tot = E->leg_tot;
        // A node home's routed pass (owner legs) holds no chain, post / void, balancing or limit event:
        // its only dependent events are same-pass duplicate ids, which the one-workgroup replay
        // orders at a fraction of tb_flow's launch (a grid of whole-CU workgroups that must wait for
        // every CU it lands on to drain: ~45 us a pass on a node's shared device).
        const bool flow = op == OP_CREATE_TRANSFERS && E->flow_ok && !E->balances_set && !(E->ablate & ABL_FLOW) &&
                          b1 - b0 <= FLOW_NB_MAX && !owner;
        P.flow_words = E->flow_ok ? E->F.words : nullptr;
        P.late_in_flow = (flow && (P.apply_late || P.legs)) ? 1u : 0u;  // tb_flow applies the late events itself

        // Launch spans of this pass's kernels on the device clock (profiling only).
        P.kclock = nullptr;
        if (E->profile && !E->kclock_off && (E->prof_mask & ((1u << K_VALIDATE) | (1u << K_RESOLVE) | (1u << K_APPLY) | (1u << K_SPANS))) &&
            E->kclock_next < KCLOCK_SLOTS) {
            const u32 slot = E->kclock_next++;
            P.kclock = E->kclock + (u64)slot * KCLOCK_WORDS;
            E->kclock_used.push_back({slot, (n > 0 ? 1u : 0u) | 2u | (P.legs ? 4u : 0u)});
        }

        ProfilePair pass_pp;
        int st = prof_begin(E, &pass_pp, K_PASS);
        if (st) return st;
        ProfilePair pp;
        if ((st = prof_begin(E, &pp, K_CLEAR))) return st;
        // Grid sized to what may need zeroing: the previous pass's dedup extent (2 entries per
        // thread per step), or the whole set when forced.
        const u64 clear_n = E->dedup_force ? E->dedup_cap : E->dedup_prev;
        const u32 clear_grid = (u32)std::min<u64>(1024, std::max<u64>(1, clear_n / 2048));
        // inline_meta: a one-prepare call's metadata, written into E->meta by this first kernel.
        u64* meta_dst = inline_meta && b0 == 0 ? (u64*)d_off : nullptr;
        ImportGate gate{};
        if (imp && n > 0) gate = ImportGate{imp->count, imp->room, 0, imp->flag};
        hipLaunchKernelGGL(tb_pass_clear, dim3(clear_grid), dim3(256), 0, E->stream, E->dedup, E->dedup_cap, E->sum_shards,
                           E->g, E->epoch, E->dedup_force ? 1u : 0u, E->leg_tot, E->leg_buckets, meta_dst,
                           inline_meta ? inline_meta[0] : 0, inline_meta ? inline_meta[1] : 0, inline_meta ? inline_meta[2] : 0,
                           P.kclock, gate, imp && b0 == 0 ? imp->leg_counts : nullptr,
                           imp && b0 == 0 ? imp->legs_n : 0u);
        HIPCK(hipGetLastError());
        E->dedup_force = false;
        E->dedup_prev = P.dedup_mask + 1;
        if ((st = prof_end(E, &pp))) return st;

        if (imp && n > 0) {  // a node home: the foreign accounts this sub-pass names, from their owners
            const u32 ig = (u32)std::min<u64>(4096, (n + 255) / 256);
            // The imports of earlier passes stay, unless they passed the room (the gate in
            // tb_pass_clear above).
            hipLaunchKernelGGL(tb_node_import_flush, dim3((u32)std::min<u64>(1024, (E->account_cap + 255) / 256)), dim3(256), 0,
                               E->stream, E->T, E->account_cap, imp->N.world, imp->self, (const u32*)imp->flag);
            hipLaunchKernelGGL(tb_node_import, dim3(ig), dim3(256), 0, E->stream, E->T, imp->N, events_dev + P.e0 * 128, n,
                               imp->self, imp->count, imp->os_of);
            HIPCK(hipGetLastError());
        }
        if (n > 0) {
            if ((st = prof_begin(E, &pp, K_VALIDATE))) return st;
            const u32 grid = (u32)((n + VALIDATE_THREADS - 1) / VALIDATE_THREADS);
            if (op == OP_CREATE_TRANSFERS) {
                if (P.events_src) {
                    hipLaunchKernelGGL(tb_transfers_validate<true>, dim3(grid), dim3(VALIDATE_THREADS), 0, E->stream, P);
                } else {
                    hipLaunchKernelGGL(tb_transfers_validate<false>, dim3(grid), dim3(VALIDATE_THREADS), 0, E->stream, P);
                }
            } else {
                if (P.events_src) {
                    hipLaunchKernelGGL(tb_accounts_validate<true>, dim3(grid), dim3(VALIDATE_THREADS), 0, E->stream, P);
                } else {
                    hipLaunchKernelGGL(tb_accounts_validate<false>, dim3(grid), dim3(VALIDATE_THREADS), 0, E->stream, P);
                }
            }
            HIPCK(hipGetLastError());
            // A write-back's copy-out slice may follow this pass's PCIe reads (wb_pump).
            if (E->wb.copying) HIPCK(hipEventRecord(E->wb.read_done, E->stream));
            if ((st = prof_end(E, &pp))) return st;
        }
        if ((st = prof_begin(E, &pp, K_RESOLVE))) return st;
        if (op == OP_CREATE_TRANSFERS) {
            // A legs pass: the lean kernel first (the common case), tb_resolve for the prepares it left.
            if (P.resolve_slow) {
                hipLaunchKernelGGL(tb_resolve_lean, dim3(b1 - b0), dim3(RESOLVE_THREADS), 0, E->stream, P);
            }
            hipLaunchKernelGGL(tb_resolve<OP_CREATE_TRANSFERS>, dim3(b1 - b0), dim3(RESOLVE_THREADS), 0, E->stream, P);
        } else {
            hipLaunchKernelGGL(tb_resolve<OP_CREATE_ACCOUNTS>, dim3(b1 - b0), dim3(RESOLVE_THREADS), 0, E->stream, P);
        }
        HIPCK(hipGetLastError());
        if ((st = prof_end(E, &pp))) return st;
        if (P.legs || P.apply_late) {
            if ((st = prof_begin(E, &pp, K_APPLY))) return st;
            if (P.legs) {
                hipLaunchKernelGGL(tb_apply_legs, dim3(E->leg_buckets + APPLY_EXTRA), dim3(APPLY_THREADS),
                                   tb_apply_lds_bytes(E->leg_shift, b1 - b0), E->stream, P);
            }
            if (n > 0 && !owner && !P.late_in_flow) {  // owner-partitioned: the owners apply the legs instead
                const u32 grid = (u32)std::min<u64>((n + 255) / 256, P.legs ? 2048 : 1u << 20);
                hipLaunchKernelGGL(tb_apply_events, dim3(grid), dim3(256), 0, E->stream, P);
            }
            HIPCK(hipGetLastError());
            if ((st = prof_end(E, &pp))) return st;
        }
        if ((st = prof_begin(E, &pp, K_REPLAY))) return st;
        if (flow) {
            UndoEntry* seq_undo = E->undo;
            u32 seq_cap = E->undo_cap;
            FlowArgs F = E->F;
            F.grid = flow_grid(E);

            // A small pass (the replica's one-prepare commit) has at most n dependent events: a grid
            // of one workgroup per 512 of them holds every unit and launches faster.
            if (n <= 65536) F.grid = std::min<u32>(F.grid, std::max<u32>(4, (u32)((n + 511) / 512)));
            if (E->flow_launch) F.grid = E->flow_launch;  // tbgpu_bench_flow_launch (tests)
            hipLaunchKernelGGL(tb_flow, dim3(F.grid), dim3(FLOW_THREADS), 0, E->stream, P, F, seq_undo, seq_cap);
        } else if (op == OP_CREATE_TRANSFERS) {
            hipLaunchKernelGGL(tb_replay<OP_CREATE_TRANSFERS>, dim3(1), dim3(REPLAY_THREADS), 0, E->stream, P,
                               E->undo, E->undo_cap);
        } else {
            hipLaunchKernelGGL(tb_replay<OP_CREATE_ACCOUNTS>, dim3(1), dim3(REPLAY_THREADS), 0, E->stream, P,
                               E->undo, E->undo_cap);
        }
        HIPCK(hipGetLastError());
        if ((st = prof_end(E, &pp))) return st;
        if (owner && n > 0) {  // every committed transfer's legs, grouped by owner (k_route.h)
            hipLaunchKernelGGL(tb_owner_legs, dim3((u32)((n + 255) / 256)), dim3(256), 0, E->stream, P, *owner);
            HIPCK(hipGetLastError());
        }
        if (imp && imp->ev_legs) HIPCK(hipEventRecord((hipEvent_t)imp->ev_legs, E->stream));
        if ((st = prof_end(E, &pass_pp))) return st;
        E->passes++;
        E->events += n;
        if (op == OP_CREATE_TRANSFERS) E->log_next += n;
        b0 = b1;
    }
    return TBGPU_STATUS_OK;
}

// Host-side checks of the commit asserts (state_machine.zig:518-519, :645, :739, :780) and
// upload of the call metadata.
static int prepare_call(tbgpu* E, u8 op, u32 nb, const u64* timestamps, const u32* lens, u64 floor_ts,
                        u64* total_events, bool upload = true) {
    if (op != OP_CREATE_ACCOUNTS && op != OP_CREATE_TRANSFERS) {
        return fail(TBGPU_STATUS_INVALID, "operation %u is not a create operation", op);
    }
    if (nb == 0) return fail(TBGPU_STATUS_INVALID, "no batches");
    if (nb > E->meta_cap) return fail(TBGPU_STATUS_INVALID, "too many batches in one call (%u > %llu)", nb,
                                      (unsigned long long)E->meta_cap);
    if (E->pending) {  // the pinned metadata mirror may still be in flight
        int st = engine_sync(E);
        if (st) return st;
    }
    u64* h_off = E->h_meta;
    u64* h_ts = E->h_meta + (nb + 1);
    u64 prev = floor_ts;
    h_off[0] = 0;
    for (u32 k = 0; k < nb; k++) {
        const u64 ts = timestamps[k];
        const u32 L = lens[k];
        if (L > BATCH_EVENTS_MAX) return fail(TBGPU_STATUS_INVALID, "batch %u has %u events (max %u)", k, L, BATCH_EVENTS_MAX);
        if (!(ts > prev)) return fail(TBGPU_STATUS_PANIC, "timestamp %llu <= commit timestamp %llu",
                                      (unsigned long long)ts, (unsigned long long)prev);
        if (L > 0) {
            if (ts < L) return fail(TBGPU_STATUS_PANIC, "timestamp %llu < batch length %u", (unsigned long long)ts, L);
            if (!(ts - L + 1 > prev)) return fail(TBGPU_STATUS_PANIC, "first event timestamp <= commit timestamp");
        }
        prev = ts;
        h_off[k + 1] = h_off[k] + L;
        h_ts[k] = ts;
    }
    if (op == OP_CREATE_TRANSFERS && E->log_next + h_off[nb] > E->xlog_cap) {
        return fail(TBGPU_STATUS_INVALID, "transfer log full (%llu + %llu events > capacity %llu)",
                    (unsigned long long)E->log_next, (unsigned long long)h_off[nb], (unsigned long long)E->xlog_cap);
    }
    if (upload) HIPCK(hipMemcpyAsync(E->meta, E->h_meta, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
    E->last_batch_ts = prev;
    *total_events = h_off[nb];
    return TBGPU_STATUS_OK;
}

static int commit_lookup(tbgpu* E, bool accounts, const void* input, uint32_t input_len, void* output,
                         uint32_t output_cap, uint32_t* out_len) {
    if (input_len % 16 != 0) return fail(TBGPU_STATUS_INVALID, "lookup body not a multiple of 16");
    const u32 n = input_len / 16;
    if (n > E->lookup_cap) return fail(TBGPU_STATUS_INVALID, "too many ids");
    if (n == 0) return TBGPU_STATUS_OK;
    HIPCK(hipMemcpyAsync(E->lookup_ids, input, input_len, hipMemcpyHostToDevice, E->stream));
    if (accounts) {
        hipLaunchKernelGGL(tb_lookup<true>, dim3((n + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_ids, n,
                           E->lookup_out, E->lookup_found);
    } else {
        hipLaunchKernelGGL(tb_lookup<false>, dim3((n + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_ids, n,
                           E->lookup_out, E->lookup_found);
    }
    HIPCK(hipGetLastError());
    std::vector<u8> found(n);
    std::vector<u8> recs((u64)n * 128);
    HIPCK(hipMemcpyAsync(found.data(), E->lookup_found, n, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipMemcpyAsync(recs.data(), E->lookup_out, (u64)n * 128, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    const u32 slots = output_cap / 128;
    u32 m = 0;
    for (u32 i = 0; i < n; i++) {
        if (found[i] && m < slots) {
            memcpy((u8*)output + (u64)m * 128, recs.data() + (u64)i * 128, 128);
            m++;
        }
    }
    *out_len = m * 128;
    return TBGPU_STATUS_OK;
}

static int wb_pump(tbgpu* E, u64 budget, hipEvent_t after);  // the write-back's copy-out (below)

static int commit_host(tbgpu* E, u8 op, u32 n, const uint64_t* timestamps, const void* const* inputs,
                       const uint32_t* input_lens, void* const* outputs, uint32_t* out_lens, const uint32_t* out_caps) {
    const void* claim = E->pf_claim;  // the staged body tbgpu_commit handed over (or null), taken once
    E->pf_claim = nullptr;
    std::vector<u32> lens(n);
    for (u32 k = 0; k < n; k++) {
        if (input_lens[k] % 128 != 0) return fail(TBGPU_STATUS_INVALID, "create body not a multiple of 128");
        lens[k] = input_lens[k] / 128;
        if (out_caps && (u64)out_caps[k] < (u64)lens[k] * 8) return fail(TBGPU_STATUS_INVALID, "output too small");
    }
    if (op == OP_CREATE_ACCOUNTS) {  // the next write-back looks these ids up
        for (u32 k = 0; k < n; k++) ckpt_note_ids(E, (const u8*)inputs[k], lens[k]);
    }
    // Split into calls whose events fit the staging buffer.
    u32 k0 = 0;
    while (k0 < n) {
        u32 k1 = k0;
        u64 ev = 0;
        while (k1 < n && k1 - k0 < E->meta_cap && ev + lens[k1] <= E->pe_max) ev += lens[k1++];
        if (k1 == k0) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
        u64 total = 0;
        const bool one = k1 - k0 == 1;
        // One prepare (the replica's commit): its metadata rides on the first kernel's arguments
        // and its reply comes back through the mapped reply arena — no copy on either side.
        int st = prepare_call(E, op, k1 - k0, timestamps + k0, lens.data() + k0, E->commit_ts, &total, !one);
        if (st) return st;
        const u64 inline_meta[3] = {0, lens[k0], timestamps[k0]};
        // Its body: staged by tbgpu_prefetch (in HBM once the copy lands), or read through by kernel
        // 1 from registered memory (written through to staging), or copied here.
        const u8* src = nullptr;
        const u8* events = E->staging;
        if (one && lens[k0] && claim == inputs[k0] && E->pf_len == lens[k0] * 128 && E->pf_op == op) {
            if (hipEventQuery(E->pf_done) != hipSuccess) HIPCK(hipStreamWaitEvent(E->stream, E->pf_done, 0));
            events = E->pf_staging;
        } else if (one && lens[k0]) {
            const u8* in = (const u8*)inputs[k0];
            for (const auto& r : E->host_regions) {
                if (in >= r.ptr && in + (u64)lens[k0] * 128 <= r.ptr + r.bytes) src = r.dev + (in - r.ptr);
            }
        }
        claim = nullptr;
        u64 off = 0;
        for (u32 k = k0; k < k1 && !src && events == E->staging; k++) {
            if (lens[k]) HIPCK(hipMemcpyAsync(E->staging + off * 128, inputs[k], (u64)lens[k] * 128,
                                              hipMemcpyHostToDevice, E->stream));
            off += lens[k];
        }
        std::vector<u64> h_off(E->h_meta, E->h_meta + (k1 - k0) + 1);
        if ((st = enqueue_call(E, op, k1 - k0, h_off.data(), events, E->results, E->reply_bytes, false, nullptr, 0,
                               src, nullptr, nullptr, one ? inline_meta : nullptr))) {
            return st;
        }
        if (one) {
            tbgpu::PipeSlot& S = E->pipe[0];
            // The host spins on the arena's done word (system-scope store after the reply): the
            // stream's completion signal reaches a waiting host thread later.
            const u32 seq = ++E->reply_seq ? E->reply_seq : ++E->reply_seq;
            volatile u32* done = (volatile u32*)(S.h_reply + pipe_reply_bytes(E));
            hipLaunchKernelGGL(tb_reply_out, dim3(1), dim3(64), 0, E->stream, E->meta, 1u, E->reply_bytes, E->results, E->g,
                               S.d_reply, (u32*)(S.d_reply + pipe_reply_bytes(E)), seq);
            HIPCK(hipGetLastError());
            if (E->wb.inflight) E->wb.calls++;
            E->wb.staged_reads = events == E->pf_staging;
            st = wb_pump(E, 0, E->wb.read_done);  // one slice of a write-back in flight
            E->wb.staged_reads = false;
            if (st) return st;
            if (!E->profile) {
                const auto t0 = std::chrono::steady_clock::now();
                for (u32 spin = 0; *done != seq; spin++) {
                    // A kernel that faulted never writes it: after 2 s, wait for the stream (which
                    // reports the fault) instead.
                    if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
                }
                std::atomic_thread_fence(std::memory_order_acquire);
            }
            if (E->profile || *done != seq) HIPCK(hipStreamSynchronize(E->stream));
            E->pending = false;
            if ((st = prof_collect(E))) return st;
            const u64* head = (const u64*)S.h_reply;
            const u32 bytes = *(const u32*)(S.h_reply + 16);
            E->commit_ts = head[1];
            if (head[0]) {
                E->poisoned = true;
                return fail(TBGPU_STATUS_PANIC, "device panic 0x%llx (the reference would have trapped)",
                            (unsigned long long)head[0]);
            }
            if (bytes) memcpy(outputs[k0], S.h_reply + 16 + 4, bytes);
            out_lens[k0] = bytes;
            k0 = k1;
            continue;
        }
        // Reply sizes and (for calls of up to h_results_events events) the result slots come back on
        // the stream with the globals: one round trip.
        const u32* rb = E->h_rb;
        HIPCK(hipMemcpyAsync(E->h_rb, E->reply_bytes, (u64)(k1 - k0) * 4, hipMemcpyDeviceToHost, E->stream));
        const bool whole = total <= E->h_results_events;
        if (whole && total) {
            HIPCK(hipMemcpyAsync(E->h_results, E->results, total * 8, hipMemcpyDeviceToHost, E->stream));
        }
        if ((st = engine_sync(E))) return st;
        for (u32 k = k0; k < k1; k++) {
            const u32 bytes = rb[k - k0];
            if (bytes && whole) memcpy(outputs[k], E->h_results + 8 * h_off[k - k0], bytes);
            else if (bytes) HIPCK(hipMemcpy(outputs[k], E->results + 2 * h_off[k - k0], bytes, hipMemcpyDeviceToHost));
            out_lens[k] = bytes;
        }
        k0 = k1;
    }
    return TBGPU_STATUS_OK;
}

// Pipelined commit of n prepares from host memory (the replica's prefetch → commit overlap,
// src/state_machine.zig:345-506 / src/vsr/replica.zig:3324-3665, with the objects HBM-resident):
// prepares are grouped into chunks of up to `chunk_batches` prepares (and pe_max events); chunk
// c+1's bodies cross PCIe on copy_stream while chunk c commits on the engine stream, and chunk c's
// replies land in its slot's pinned arena (tb_reply_out) as soon as it is committed.  The host
// reads chunk c's replies before it reuses the slot for chunk c + PIPE_SLOTS.  Results are those
// of n sequential commits.  latency_ms[k] (optional): device-clock time from the start of prepare
// k's chunk crossing PCIe to its reply landing in host memory.
static int commit_pipelined(tbgpu* E, u8 op, u32 n, const uint64_t* timestamps, const void* const* inputs,
                            const uint32_t* input_lens, void* const* outputs, uint32_t* out_lens,
                            const uint32_t* out_caps, u32 chunk_batches, double* latency_ms) {
    if (op != OP_CREATE_ACCOUNTS && op != OP_CREATE_TRANSFERS) {
        return fail(TBGPU_STATUS_INVALID, "operation %u is not a create operation", op);
    }
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    std::vector<u32> lens(n);
    u64 prev = E->commit_ts, total = 0;
    for (u32 k = 0; k < n; k++) {  // the commit asserts of every prepare, before anything runs
        if (input_lens[k] % 128 != 0) return fail(TBGPU_STATUS_INVALID, "create body not a multiple of 128");
        const u32 L = input_lens[k] / 128;
        if (L > BATCH_EVENTS_MAX) return fail(TBGPU_STATUS_INVALID, "batch %u has %u events (max %u)", k, L, BATCH_EVENTS_MAX);
        if (out_caps && (u64)out_caps[k] < (u64)L * 8) return fail(TBGPU_STATUS_INVALID, "output too small");
        const u64 ts = timestamps[k];
        if (!(ts > prev)) return fail(TBGPU_STATUS_PANIC, "timestamp %llu <= commit timestamp %llu",
                                      (unsigned long long)ts, (unsigned long long)prev);
        if (L > 0) {
            if (ts < L) return fail(TBGPU_STATUS_PANIC, "timestamp %llu < batch length %u", (unsigned long long)ts, L);
            if (!(ts - L + 1 > prev)) return fail(TBGPU_STATUS_PANIC, "first event timestamp <= commit timestamp");
        }
        prev = ts;
        lens[k] = L;
        total += L;
        out_lens[k] = 0;
    }
    if (op == OP_CREATE_TRANSFERS && E->log_next + total > E->xlog_cap) {
        return fail(TBGPU_STATUS_INVALID, "transfer log full (%llu + %llu events > capacity %llu)",
                    (unsigned long long)E->log_next, (unsigned long long)total, (unsigned long long)E->xlog_cap);
    }
    if (op == OP_CREATE_ACCOUNTS) {  // the next write-back looks these ids up
        for (u32 k = 0; k < n; k++) ckpt_note_ids(E, (const u8*)inputs[k], lens[k]);
    }
    const u32 per_chunk = std::max<u32>(1, std::min<u32>(chunk_batches ? chunk_batches : E->pb_max, E->pb_max));
    struct Chunk {
        u32 k0, k1;
    };
    std::vector<Chunk> chunks;
    for (u32 k0 = 0; k0 < n;) {
        u32 k1 = k0;
        u64 ev = 0;
        while (k1 < n && k1 - k0 < per_chunk && k1 - k0 < E->meta_cap && ev + lens[k1] <= E->pe_max) ev += lens[k1++];
        if (k1 == k0) return fail(TBGPU_STATUS_INVALID, "batch larger than pass_events_max");
        chunks.push_back({k0, k1});
        k0 = k1;
    }
    int status = TBGPU_STATUS_OK;
    // Read chunk c's replies out of its slot (its done event has fired or is waited for here).
    // After a failed chunk the later ones (already enqueued) are only waited for: the reference
    // would have stopped at the panic, so their replies and timestamps are not taken.
    auto consume = [&](size_t c, bool take) -> int {
        tbgpu::PipeSlot& S = E->pipe[c % PIPE_SLOTS];
        HIPCK(hipEventSynchronize(S.done));
        if (!take) return TBGPU_STATUS_OK;
        const Chunk& C = chunks[c];
        const u32 nb = C.k1 - C.k0;
        const u64* head = (const u64*)S.h_reply;
        const u32* rb = (const u32*)(S.h_reply + 16);
        const u8* res = S.h_reply + 16 + (u64)nb * 4;
        float ms = 0;
        if (latency_ms) HIPCK(hipEventElapsedTime(&ms, S.start, S.done));
        for (u32 k = C.k0; k < C.k1; k++) {
            const u32 bytes = rb[k - C.k0];
            if (bytes) memcpy(outputs[k], res + 8 * S.h_meta[k - C.k0], bytes);
            out_lens[k] = bytes;
            if (latency_ms) latency_ms[k] = ms;
        }
        E->commit_ts = std::max(E->commit_ts, head[1]);
        if (head[0]) {
            E->poisoned = true;
            return fail(TBGPU_STATUS_PANIC, "device panic 0x%llx (the reference would have trapped)",
                        (unsigned long long)head[0]);
        }
        return TBGPU_STATUS_OK;
    };
    size_t issued = 0, consumed = 0;
    for (; issued < chunks.size() && status == TBGPU_STATUS_OK; issued++) {
        const size_t c = issued;
        if (c >= PIPE_SLOTS) {
            status = consume(consumed++, true);
            if (status) break;
        }
        tbgpu::PipeSlot& S = E->pipe[c % PIPE_SLOTS];
        const Chunk& C = chunks[c];
        const u32 nb = C.k1 - C.k0;
        u64* h_off = S.h_meta;
        u64* h_ts = S.h_meta + (nb + 1);
        h_off[0] = 0;
        for (u32 k = C.k0; k < C.k1; k++) {
            h_off[k - C.k0 + 1] = h_off[k - C.k0] + lens[k];
            h_ts[k - C.k0] = timestamps[k];
        }
        // Copy stream: the bodies only (runs of address-contiguous prepares as one DMA), back to back;
        // the chunk's small metadata goes on the engine stream, which has time to spare.
        HIPCK(hipEventRecord(S.start, E->copy_stream));
        for (u32 k = C.k0; k < C.k1;) {
            u32 j = k + 1;
            const u8* base = (const u8*)inputs[k];
            u64 bytes = (u64)lens[k] * 128;
            while (j < C.k1 && (const u8*)inputs[j] == base + bytes) bytes += (u64)lens[j++] * 128;
            if (bytes) HIPCK(hipMemcpyAsync(S.staging + h_off[k - C.k0] * 128, base, bytes, hipMemcpyHostToDevice,
                                            E->copy_stream));
            k = j;
        }
        HIPCK(hipEventRecord(S.copied, E->copy_stream));
        // Engine stream: the chunk's passes, then its replies into the pinned arena.
        HIPCK(hipMemcpyAsync(S.meta, S.h_meta, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
        HIPCK(hipStreamWaitEvent(E->stream, S.copied, 0));
        E->last_batch_ts = timestamps[C.k1 - 1];
        status = enqueue_call(E, op, nb, h_off, S.staging, E->results, E->reply_bytes, false, nullptr, 0, nullptr, S.meta);
        if (status) break;
        hipLaunchKernelGGL(tb_reply_out, dim3(nb), dim3(64), 0, E->stream, S.meta, nb, E->reply_bytes, E->results, E->g,
                           S.d_reply);
        HIPCK(hipGetLastError());
        HIPCK(hipEventRecord(S.done, E->stream));
    }
    // Drain what is in flight (also after a failure: every enqueued chunk has finished before the
    // call returns, as after any synchronous call).
    while (consumed < issued) {
        const int st = consume(consumed++, status == TBGPU_STATUS_OK);
        if (status == TBGPU_STATUS_OK) status = st;
    }
    const u64 taken_ts = E->commit_ts;  // as of the last chunk whose replies were taken
    HIPCK(hipStreamSynchronize(E->copy_stream));
    const int st = engine_sync(E);
    if (status) E->commit_ts = taken_ts;  // chunks queued behind a failure ran, but count for nothing
    return status ? status : st;
}

extern "C" int tbgpu_commit_pipelined(tbgpu_t* E, uint8_t operation, uint32_t n, const uint64_t* timestamps,
                                      const void* const* inputs, const uint32_t* input_lens, void* const* outputs,
                                      uint32_t* out_lens, uint32_t chunk_batches, double* latency_ms) {
    API_ENTER(E, true);
    if (E->node) return n ? node_commit_pipelined(E->node, operation, n, timestamps, inputs, input_lens, outputs, out_lens,
                                                  chunk_batches, latency_ms) : TBGPU_STATUS_OK;
    HIPCK(hipSetDevice(E->device));
    if (n == 0) return TBGPU_STATUS_OK;
    return commit_pipelined(E, operation, n, timestamps, inputs, input_lens, outputs, out_lens, nullptr, chunk_batches,
                            latency_ms);
}

extern "C" int tbgpu_commit(tbgpu_t* E, uint8_t operation, uint64_t timestamp, const void* input,
                            uint32_t input_len, void* output, uint32_t output_cap, uint32_t* out_len) {
    *out_len = 0;
    // The body tbgpu_prefetch staged (if any) may be taken by this commit only: hand it to
    // commit_host and drop it from the engine whatever happens next.
    const void* staged = E->pf_input;
    API_ENTER(E, true);  // before the node hand-off too: a node keys its drain skipping on the count
    if (E->node) return node_api_commit(E->node, operation, timestamp, input, input_len, output, output_cap, out_len);
    HIPCK(hipSetDevice(E->device));
    if (operation < OP_CREATE_ACCOUNTS || operation > OP_LOOKUP_TRANSFERS) {
        return fail(TBGPU_STATUS_INVALID, "unknown operation %u", operation);
    }
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    if (!(timestamp > E->commit_ts)) {  // state_machine.zig:519
        return fail(TBGPU_STATUS_PANIC, "timestamp %llu <= commit timestamp %llu", (unsigned long long)timestamp,
                    (unsigned long long)E->commit_ts);
    }
    if (operation == OP_LOOKUP_ACCOUNTS || operation == OP_LOOKUP_TRANSFERS) {
        return commit_lookup(E, operation == OP_LOOKUP_ACCOUNTS, input, input_len, output, output_cap, out_len);
    }
    if (input_len == 0) {  // empty batch: nothing to execute (execute loops zero times)
        return TBGPU_STATUS_OK;
    }
    const void* ins[1] = {input};
    void* outs[1] = {output};
    E->pf_claim = staged;
    return commit_host(E, operation, 1, &timestamp, ins, &input_len, outs, out_len, &output_cap);
}

// StateMachine.prefetch (src/state_machine.zig:345-506): every object is HBM-resident, so what is
// left to stage is the prepare body itself — a pageable create body starts its copy to HBM now, on
// the copy stream, and the commit of the same body only waits for it.  A registered body (the
// message pool) is not staged: the commit reads it through (below).  Anything else needs nothing.
static bool wb_copy_in_flight(tbgpu* E);  // (below)

extern "C" int tbgpu_prefetch(tbgpu_t* E, uint8_t operation, const void* input, uint32_t input_len) {
    if (E->node) return TBGPU_STATUS_OK;
    HIPCK(hipSetDevice(E->device));
    E->pf_input = nullptr;
    if ((operation != OP_CREATE_ACCOUNTS && operation != OP_CREATE_TRANSFERS) || input_len == 0 ||
        input_len % 128 != 0 || input_len / 128 > BATCH_EVENTS_MAX) {
        return TBGPU_STATUS_OK;
    }
    bool registered = false;
    for (const auto& r : E->host_regions) {
        if ((const u8*)input >= r.ptr && (const u8*)input + input_len <= r.ptr + r.bytes) registered = true;
    }
    // A registered body is read by the commit's first kernel straight over PCIe (and written through
    // to HBM): faster than a DMA ahead of it, which the replica's serial prefetch -> commit leaves
    // nothing to overlap with (round 5: 95 M/s staged against 123 M/s read through,
    // `replica_path`).  So only a pageable body is staged here: its copy, which the commit would
    // otherwise make itself, happens at prefetch.
    // Except while a write-back's copy-out is in flight: then the body crosses by DMA (the link carries
    // both directions at ~50 GB/s each, tools/microbench_h2d `duplex`), the commit reads HBM, and the
    // copy-out needs not wait for the commit's PCIe reads (wb_pump).
    // (Not for a write-back every op: the body's DMA then only lengthens each serial prepare.)
    // (A bound-sized copy-out is issued whole at its write-back: staged while it crosses.  A counts-
    // sized one, a slice per commit: while slices are still to be sent — measured: staging every
    // body of a bar while its copy-out crosses cost one bar behind 97 -> 86 M/s.)
    const bool stage = E->wb.bound ? wb_copy_in_flight(E) : E->wb.copying;
    if (registered && !(E->wb_stage && E->wb.calls_prev >= 2 && stage)) return TBGPU_STATUS_OK;
    // The staging slot's previous reader (the last commit) has finished: commits are synchronous.
    HIPCK(hipMemcpyAsync(E->pf_staging, input, input_len, hipMemcpyHostToDevice, E->copy_stream));
    HIPCK(hipEventRecord(E->pf_done, E->copy_stream));
    E->pf_input = input;
    E->pf_len = input_len;
    E->pf_op = operation;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_commit_many(tbgpu_t* E, uint8_t operation, uint32_t n, const uint64_t* timestamps,
                                 const void* const* inputs, const uint32_t* input_lens, void* const* outputs,
                                 uint32_t* out_lens) {
    API_ENTER(E, true);
    if (E->node) {
        for (u32 k = 0; k < n; k++) out_lens[k] = 0;
        return n ? node_commit_pipelined(E->node, operation, n, timestamps, inputs, input_lens, outputs, out_lens, 0, nullptr)
                 : TBGPU_STATUS_OK;
    }
    HIPCK(hipSetDevice(E->device));
    for (u32 k = 0; k < n; k++) out_lens[k] = 0;
    if (n == 0) return TBGPU_STATUS_OK;
    if (n == 1) return commit_host(E, operation, n, timestamps, inputs, input_lens, outputs, out_lens, nullptr);
    return commit_pipelined(E, operation, n, timestamps, inputs, input_lens, outputs, out_lens, nullptr, 0, nullptr);
}

extern "C" int tbgpu_commit_device_async(tbgpu_t* E, uint8_t operation, uint32_t n_batches,
                                         const uint64_t* timestamps, const uint32_t* batch_lens,
                                         const void* events_dev, void* results_dev, uint32_t* reply_bytes_dev) {
    API_ENTER(E, true);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "device-resident commits need a single-device engine");
    HIPCK(hipSetDevice(E->device));
    const u64 floor_ts = std::max(E->commit_ts, E->pending ? E->last_batch_ts : 0);
    u64 total = 0;
    int st = prepare_call(E, operation, n_batches, timestamps, batch_lens, floor_ts, &total);
    if (st) return st;
    std::vector<u64> h_off(E->h_meta, E->h_meta + n_batches + 1);
    if (operation == OP_CREATE_ACCOUNTS) E->ckpt_scan = true;  // ids in device memory: diff the table next
    // Prepares placed in the log window (tbgpu_log_window) are committed in place.
    E->inplace_call = operation == OP_CREATE_TRANSFERS && (const u8*)events_dev == (const u8*)(E->T.xlog + E->log_next);
    st = enqueue_call(E, operation, n_batches, h_off.data(), (const u8*)events_dev, (u32*)results_dev, reply_bytes_dev);
    E->inplace_call = false;
    if (st) return st;
    E->pending = true;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_log_window(tbgpu_t* E, uint64_t events, void** window) {
    API_ENTER(E, false);
    *window = nullptr;
    if (E->node) return fail(TBGPU_STATUS_INVALID, "the log window needs a single-device engine");
    if (E->log_next + events > E->xlog_cap) {
        return fail(TBGPU_STATUS_INVALID, "transfer log full: %llu of %llu positions used, %llu asked",
                    (unsigned long long)E->log_next, (unsigned long long)E->xlog_cap, (unsigned long long)events);
    }
    *window = E->T.xlog + E->log_next;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_sync(tbgpu_t* E) {
    API_ENTER(E, false);
    if (E->node) return node_sync(E->node);
    HIPCK(hipSetDevice(E->device));
    return engine_sync(E);
}

extern "C" uint64_t tbgpu_commit_timestamp(tbgpu_t* E) {
    if (E->node) return node_commit_ts(E->node);
    if (E->pending) engine_sync(E);
    return E->commit_ts;
}

extern "C" int tbgpu_test_set_balances(tbgpu_t* E, uint64_t id_lo, uint64_t id_hi, const uint64_t b[8]) {
    API_ENTER(E, true);
    if (E->node) return node_api_set_balances(E->node, id_lo, id_hi, b);
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    E->balances_set = true;  // the flow path's post/void argument needs consistent pending balances
    {
        u8 rec[128] = {};
        memcpy(rec, &id_lo, 8);
        memcpy(rec + 8, &id_hi, 8);
        ckpt_note_ids(E, rec, 1);
    }
    hipLaunchKernelGGL(tb_set_balances, dim3(1), dim3(1), 0, E->stream, E->T, id_lo, id_hi, b[0], b[1], b[2], b[3],
                       b[4], b[5], b[6], b[7], E->d_status);
    HIPCK(hipGetLastError());
    u32 status = 0;
    HIPCK(hipMemcpyAsync(&status, E->d_status, 4, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    if (status) return fail(TBGPU_STATUS_PANIC, "setup of a missing account");
    return TBGPU_STATUS_OK;
}

static bool id_less(const u8* a, const u8* b) {
    const u64* x = (const u64*)a;
    const u64* y = (const u64*)b;
    return x[1] != y[1] ? x[1] < y[1] : x[0] < y[0];
}

// Export live records in chunks (bounded temporaries), then sort by id.
template <bool ACCOUNTS>
static int export_records(tbgpu* E, std::vector<u8>& recs, std::vector<u64>* posted) {
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    const u64 cap = ACCOUNTS ? E->account_cap : E->xidx_cap;
    const u64 chunk = std::min<u64>(cap, 1ULL << 20);
    u8* d_out = nullptr;
    u64* d_cnt = nullptr;
    u64* d_posted = nullptr;
    HIPCK(tbMalloc(&d_out, chunk * 128));
    HIPCK(tbMalloc(&d_cnt, 16));
    HIPCK(tbMalloc(&d_posted, chunk * 16));
    int st = TBGPU_STATUS_OK;
    for (u64 s = 0; s < cap && st == TBGPU_STATUS_OK; s += chunk) {
        const u64 n = std::min<u64>(chunk, cap - s);
        hipError_t e = hipMemsetAsync(d_cnt, 0, 16, E->stream);
        if (e == hipSuccess) {
            if (ACCOUNTS) {
                hipLaunchKernelGGL(tb_export_accounts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, E->stream, E->T,
                                   s, s + n, d_out, d_cnt);
            } else {
                hipLaunchKernelGGL(tb_export_transfers, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, E->stream, E->T,
                                   s, n, d_out, d_cnt, d_posted, d_cnt + 1);
            }
            e = hipGetLastError();
        }
        u64 cnt[2] = {0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(cnt, d_cnt, 16, hipMemcpyDeviceToHost, E->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(E->stream);
        if (e == hipSuccess && cnt[0]) {
            const size_t at = recs.size();
            recs.resize(at + cnt[0] * 128);
            e = hipMemcpy(recs.data() + at, d_out, cnt[0] * 128, hipMemcpyDeviceToHost);
        }
        if (e == hipSuccess && posted && cnt[1]) {
            const size_t at = posted->size();
            posted->resize(at + cnt[1] * 2);
            e = hipMemcpy(posted->data() + at, d_posted, cnt[1] * 16, hipMemcpyDeviceToHost);
        }
        if (e != hipSuccess) st = fail(TBGPU_STATUS_DEVICE, "export: %s", hipGetErrorString(e));
    }
    (void)hipFree(d_out);
    (void)hipFree(d_cnt);
    (void)hipFree(d_posted);
    if (st) return st;
    const u64 n = recs.size() / 128;
    std::vector<u64> idx(n);
    for (u64 i = 0; i < n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](u64 a, u64 b) { return id_less(&recs[a * 128], &recs[b * 128]); });
    std::vector<u8> sorted(recs.size());
    for (u64 i = 0; i < n; i++) memcpy(&sorted[i * 128], &recs[idx[i] * 128], 128);
    recs.swap(sorted);
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_export_accounts(tbgpu_t* E, void* out, uint64_t cap, uint64_t* count) {
    API_ENTER(E, false);
    if (E->node) return node_api_export(E->node, 0, out, cap, count);
    HIPCK(hipSetDevice(E->device));
    std::vector<u8> recs;
    int st = export_records<true>(E, recs, nullptr);
    if (st) return st;
    const u64 n = std::min<u64>(recs.size() / 128, cap);
    memcpy(out, recs.data(), n * 128);
    *count = n;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_export_transfers(tbgpu_t* E, void* out, uint64_t cap, uint64_t* count) {
    API_ENTER(E, false);
    if (E->node) return node_api_export(E->node, 1, out, cap, count);
    HIPCK(hipSetDevice(E->device));
    std::vector<u8> recs;
    int st = export_records<false>(E, recs, nullptr);
    if (st) return st;
    const u64 n = std::min<u64>(recs.size() / 128, cap);
    memcpy(out, recs.data(), n * 128);
    *count = n;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_export_posted(tbgpu_t* E, uint64_t* out_pairs, uint64_t cap, uint64_t* count) {
    API_ENTER(E, false);
    if (E->node) return node_api_export(E->node, 2, out_pairs, cap, count);
    HIPCK(hipSetDevice(E->device));
    std::vector<u8> recs;
    std::vector<u64> posted;
    int st = export_records<false>(E, recs, &posted);
    if (st) return st;
    const u64 n = posted.size() / 2;
    std::vector<std::pair<u64, u64>> pairs(n);
    for (u64 i = 0; i < n; i++) pairs[i] = {posted[2 * i], posted[2 * i + 1]};
    std::sort(pairs.begin(), pairs.end());
    const u64 m = std::min<u64>(n, cap);
    for (u64 i = 0; i < m; i++) {
        out_pairs[2 * i] = pairs[i].first;
        out_pairs[2 * i + 1] = pairs[i].second;
    }
    *count = m;
    return TBGPU_STATUS_OK;
}

// Groove write-back: everything a durable replica's checkpoint / compact must insert or upsert into
// its forest since the previous call (or since init / reset) — state_machine.zig:542-582 with the
// groove semantics of src/lsm/groove.zig:902-963.  Accounts by id, transfers and posted pairs by
// timestamp.
//
// The cost is O(changes), not O(tables) (the reference's groove put / upsert per changed object):
//   * transfers: the log positions written since the previous write-back, each checked live by one
//     index probe (tb_delta_log_*), compacted in log (= timestamp) order on the device;
//   * posted-groove entries: one per new post / void record (the pending transfer's timestamp,
//     posted or voided: state_machine.zig:988-990), looked up on the device (tb_delta_posted);
//   * accounts: the debit and credit accounts of the new transfers, plus the ids of create_accounts
//     events and of direct balance writes the engine listed since — each looked up once and emitted
//     if created since or re-balanced (tb_delta_ids).  Only create_accounts committed from device
//     memory (or more listed ids than WB_IDS_MAX) makes the next write-back diff the whole account
//     table instead (tb_delta_accounts).
// Every device buffer is allocated at tbgpu_init (WbBufs): a write-back walks the log in slices of
// the buffers' size.  The caller's buffers are checked up front against what the write-back can
// emit at most (every log position since, twice as many accounts plus the listed ids), so a write-
// back that runs always fits and a refused one changes nothing.
//
// The snapshot exists and describes the previous write-back (the empty state if none).
static int ckpt_snapshot_ready(tbgpu* E) {
    if (!E->ckpt_valid) {  // the previous write-back is the empty state
        HIPCK(hipMemsetAsync(E->ckpt_bal, 0, E->account_cap * sizeof(AccountBal), E->stream));
        E->ckpt_pos = 0;
        E->ckpt_ts = 0;
        E->ckpt_valid = true;
    }
    return TBGPU_STATUS_OK;
}

// Listed since the previous write-back (host side): ids of create_accounts events and of direct
// balance writes.  Past WB_IDS_MAX the list gives way to one whole-table diff.
static void ckpt_note_ids(tbgpu* E, const u8* records, u64 n) {
    if (E->ckpt_scan) return;
    if (E->ckpt_ids.size() / 2 + n > WB_IDS_MAX) {
        E->ckpt_scan = true;
        std::vector<u64>().swap(E->ckpt_ids);
        return;
    }
    for (u64 i = 0; i < n; i++) {
        E->ckpt_ids.push_back(*(const u64*)(records + i * 128));
        E->ckpt_ids.push_back(*(const u64*)(records + i * 128 + 8));
    }
}

// This write-back's epoch: every slot it covers is marked once (tb_delta_ids); wrapped, the marks
// are cleared so no stale one can equal it.
static int wb_next_epoch(tbgpu* E) {
    if (++E->ckpt_epoch == 0) {
        HIPCK(hipMemsetAsync(E->ckpt_mark, 0, E->account_cap * sizeof(u32), E->stream));
        E->ckpt_epoch = 1;
    }
    return TBGPU_STATUS_OK;
}

// What a write-back of this engine can emit at most: transfers and posted entries <= the log
// positions written since; accounts <= two per new transfer plus the listed ids (or, after an
// unlisted create, every live account).
struct WbBounds {
    u64 transfers, posted, accounts;
};
static WbBounds wb_bounds(tbgpu* E, u64 live_accounts) {
    const u64 range = E->log_next - (E->ckpt_valid ? E->ckpt_pos : 0);
    WbBounds b;
    b.transfers = b.posted = range;
    b.accounts = E->ckpt_scan ? live_accounts : std::min<u64>(E->account_cap, 2 * range + E->ckpt_ids.size() / 2);
    return b;
}

// Slice [a, b) of the log range: gather its new transfers (records, their account ids, their post /
// void records and posted pairs) into the write-back buffers and look their accounts up.  Enqueued
// only; the slice's counts land in d_cnt (records, post / void records, accounts emitted).
// zero_counts = false: the caller zeroed them in stream order already (the asynchronous write-back).
static int wb_gather_slice(tbgpu* E, u64 a, u64 b, bool want_records, bool posted = true, hipStream_t stream = nullptr,
                           bool zero_counts = true) {
    WbBufs& W = E->wb;
    if (!stream) stream = E->stream;
    const u64 n = b - a, nblocks = (n + DELTA_THREADS - 1) / DELTA_THREADS;
    if (zero_counts) {
        HIPCK(hipMemsetAsync(W.d_cnt + WB_ACCOUNTS, 0, 8, stream));
        HIPCK(hipMemsetAsync(W.d_cnt + WB_PV, 0, 16, stream));  // WB_PV, WB_RECORDS
    }
    if (!n) return TBGPU_STATUS_OK;
    hipLaunchKernelGGL(tb_delta_log_count, dim3((unsigned)nblocks), dim3(DELTA_THREADS), 0, stream, E->T, a, n, E->ckpt_ts,
                       W.d_bc);
    hipLaunchKernelGGL(tb_delta_scan_blocks, dim3(1), dim3(1024), 0, stream, W.d_bc, nblocks, W.d_base,
                       W.d_cnt + WB_RECORDS);
    hipLaunchKernelGGL(tb_delta_log_scatter, dim3((unsigned)nblocks), dim3(DELTA_THREADS), 0, stream, E->T, a, n,
                       E->ckpt_ts, W.d_base, want_records ? W.d_out : (u8*)nullptr, W.d_ids, W.d_pv, W.d_cnt + WB_PV);
    if (posted) {  // a node's pending transfer may live on another shard: the node looks it up
        hipLaunchKernelGGL(tb_delta_posted, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, E->T, W.d_pv,
                           W.d_cnt + WB_PV, W.d_pairs, W.d_cnt + WB_STATUS);
    }
    HIPCK(hipGetLastError());
    return TBGPU_STATUS_OK;
}

// The account delta of ids on the device (2 x *n_dev of them when n_dev is given, else n).
static int wb_ids(tbgpu* E, const u64* d_ids, u64 n, const u64* n_dev) {
    if (E->ckpt_scan || !n) return TBGPU_STATUS_OK;
    WbBufs& W = E->wb;
    hipLaunchKernelGGL(tb_delta_ids, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, E->stream, E->T, ckpt_view(E), E->ckpt_ts,
                       d_ids, n, E->ckpt_mark, E->ckpt_epoch, W.d_acc, W.d_before, W.d_cnt + WB_ACCOUNTS, W.d_slots,
                       W.d_cnt + WB_SLOTS, n_dev);
    HIPCK(hipGetLastError());
    return TBGPU_STATUS_OK;
}

static int wb_read_counts(tbgpu* E) {
    HIPCK(hipMemcpyAsync(E->wb.h_cnt, E->wb.d_cnt, WB_COUNT_WORDS * 8, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    if (E->wb.h_cnt[WB_STATUS]) return fail(TBGPU_STATUS_PANIC, "checkpoint delta: a posted pending transfer is missing");
    return TBGPU_STATUS_OK;
}

// The emitted accounts of the current slice / chunk into the caller's buffers at *na.
static int wb_take_accounts(tbgpu* E, u8* out, u8* before_out, u64* na) {
    const u64 k = E->wb.h_cnt[WB_ACCOUNTS];
    if (k) {
        HIPCK(hipMemcpyAsync(out + *na * 128, E->wb.d_acc, k * 128, hipMemcpyDeviceToHost, E->stream));
        if (before_out) {
            HIPCK(hipMemcpyAsync(before_out + *na * sizeof(AccountBal), E->wb.d_before, k * sizeof(AccountBal),
                                 hipMemcpyDeviceToHost, E->stream));
        }
        HIPCK(hipStreamSynchronize(E->stream));
    }
    *na += k;
    HIPCK(hipMemsetAsync(E->wb.d_cnt + WB_ACCOUNTS, 0, 8, E->stream));
    return TBGPU_STATUS_OK;
}

// Listed ids (host) in chunks of the ids buffer, each chunk's accounts taken as it completes.
static int wb_listed_ids(tbgpu* E, const std::vector<u64>& ids, u8* out, u8* before_out, u64* na) {
    const u64 n = ids.size() / 2;
    for (u64 c = 0; c < n && !E->ckpt_scan; c += E->wb.cap_ids) {
        const u64 m = std::min<u64>(E->wb.cap_ids, n - c);
        HIPCK(hipMemcpyAsync(E->wb.d_hids, ids.data() + 2 * c, m * 16, hipMemcpyHostToDevice, E->stream));
        int st = wb_ids(E, E->wb.d_hids, m, nullptr);
        if (!st) st = wb_read_counts(E);  // also: the host list may change once this returns
        if (!st) st = wb_take_accounts(E, out, before_out, na);
        if (st) return st;
    }
    return TBGPU_STATUS_OK;
}

// The whole-table diff, in slot ranges of the accounts buffer; on a node shard (world > 1) only the
// accounts it owns.
static int wb_scan(tbgpu* E, u32 world, u32 self, u8* out, u8* before_out, u64* na) {
    if (!E->ckpt_scan) return TBGPU_STATUS_OK;
    for (u64 s0 = 0; s0 < E->account_cap; s0 += E->wb.cap_a) {
        const u64 s1 = std::min<u64>(E->account_cap, s0 + E->wb.cap_a);
        hipLaunchKernelGGL(tb_delta_accounts, dim3((unsigned)((s1 - s0 + 255) / 256)), dim3(256), 0, E->stream, E->T,
                           ckpt_view(E), E->ckpt_ts, s0, s1, E->wb.d_acc, E->wb.cap_a, E->wb.d_cnt + WB_ACCOUNTS,
                           E->wb.d_before, world, self);
        HIPCK(hipGetLastError());
        int st = wb_read_counts(E);
        if (!st) st = wb_take_accounts(E, out, before_out, na);
        if (st) return st;
    }
    return TBGPU_STATUS_OK;
}

// The write-back happened: the snapshot takes the covered balances (enqueued), the log and commit
// positions move, the lists empty.
static int wb_advance(tbgpu* E) {
    if (E->ckpt_scan) {
        HIPCK(hipMemcpyAsync(E->ckpt_bal, E->T.bal.lo, E->account_cap * sizeof(AccountBal), hipMemcpyDeviceToDevice,
                             E->stream));
    } else {
        const u32 grid = (u32)std::max<u64>(1, std::min<u64>(2048, (E->account_cap + 255) / 256));
        hipLaunchKernelGGL(tb_delta_advance, dim3(grid), dim3(256), 0, E->stream, E->T, ckpt_view(E), E->wb.d_slots,
                           E->wb.d_cnt + WB_SLOTS);
        HIPCK(hipGetLastError());
    }
    E->ckpt_pos = E->log_next;
    E->ckpt_ts = E->commit_ts;
    E->ckpt_scan = false;
    std::vector<u64>().swap(E->ckpt_ids);
    return TBGPU_STATUS_OK;
}

// Log order is timestamp order for everything a commit appends; records appended by an upsert or a
// load (a node's sequencer write-back, a restart's warm-up) may sit out of order: sort those runs.
static void delta_sort_by_timestamp(u8* recs, u64 n) {
    auto ts = [&](u64 i) { return *(const u64*)(recs + i * 128 + 120); };
    bool sorted = true;
    for (u64 i = 1; i < n && sorted; i++) sorted = ts(i - 1) < ts(i);
    if (sorted) return;
    std::vector<std::pair<u64, u64>> key(n);
    for (u64 i = 0; i < n; i++) key[i] = {ts(i), i};
    std::sort(key.begin(), key.end());
    std::vector<u8> tmp(recs, recs + n * 128);
    for (u64 i = 0; i < n; i++) memcpy(recs + i * 128, &tmp[key[i].second * 128], 128);
}

static void delta_sort_pairs(u64* pairs, u64 n) {
    std::sort((std::pair<u64, u64>*)pairs, (std::pair<u64, u64>*)pairs + n);
}

// The asynchronous write-back in flight (if any) has landed: its counts, sorted outputs.
static int wb_wait(tbgpu* E, tbgpu_delta_counts* counts) {
    WbBufs& W = E->wb;
    if (!W.inflight) return fail(TBGPU_STATUS_INVALID, "no asynchronous write-back in flight");
    if (W.copying) {  // what the commits since did not send yet
        const int st = wb_pump(E, ~0ULL, nullptr);
        if (st) return st;
    }
    W.inflight = false;
    if (W.calls) W.calls_prev = W.calls;  // (one waited for at once, a bar's last op, says nothing)
    HIPCK(hipEventSynchronize(W.done));
    *counts = W.counts;
    counts->transfers = W.h_cnt[WB_RECORDS];
    counts->posted = W.h_cnt[WB_PV];
    counts->accounts = W.h_cnt[WB_ACCOUNTS];
    if (W.posted_late && counts->posted) {
        HIPCK(hipMemcpyAsync(W.dst[3], W.src[3], counts->posted * 16, hipMemcpyDeviceToHost, W.stream));
        HIPCK(hipStreamSynchronize(W.stream));
    }
    W.posted_late = false;
    if (W.dst[1]) {  // an asynchronous copy-out ran: did its objects fill their bounds (within 1/8)?
        const u64 actual = counts->transfers * 128 + counts->accounts * (128 + sizeof(AccountBal));
        const u64 bound = W.bound_len[0] * 128 + W.bound_len[1] * (128 + sizeof(AccountBal));
        W.bound_ok = actual * 8 >= bound * 7;
    }
    if (W.h_cnt[WB_STATUS]) {
        E->poisoned = true;
        return fail(TBGPU_STATUS_PANIC, "checkpoint delta: a posted pending transfer is missing");
    }
    // Only when tb_delta_order saw them out of order (the synchronous path's outputs are sorted).
    if (W.out_t && (W.h_cnt[WB_ORDER] & 1)) delta_sort_by_timestamp(W.out_t, counts->transfers);
    if (W.out_p && (W.h_cnt[WB_ORDER] & 2)) delta_sort_pairs(W.out_p, counts->posted);
    return TBGPU_STATUS_OK;
}

static void wb_set_slice(tbgpu* E, u64 total);  // the copy-out's slice (below)
static int wb_tail(tbgpu* E, hipEvent_t after, bool counts);  // the gather beside the commits (below)

static int wb_checkpoint_sync(tbgpu* E, u8* accounts_out, u8* before_out, u64 accounts_cap, u8* transfers_out,
                              u64 transfers_cap, u64* posted_out, u64 posted_cap, tbgpu_delta_counts* counts) {
    memset(counts, 0, sizeof(*counts));
    int st = ckpt_snapshot_ready(E);
    if (st) return st;
    const WbBounds bd = wb_bounds(E, E->h_globals->account_count);
    counts->created_after = E->ckpt_ts;
    if (bd.accounts > accounts_cap || bd.transfers > transfers_cap || bd.posted > posted_cap) {  // nothing moved
        counts->accounts = bd.accounts;
        counts->transfers = bd.transfers;
        counts->posted = bd.posted;
        return fail(TBGPU_STATUS_INVALID, "checkpoint delta: buffers must hold %llu accounts, %llu transfers, %llu posted",
                    (unsigned long long)bd.accounts, (unsigned long long)bd.transfers, (unsigned long long)bd.posted);
    }
    if ((st = wb_next_epoch(E))) return st;
    HIPCK(hipMemsetAsync(E->wb.d_cnt, 0, WB_COUNT_WORDS * 8, E->stream));
    u64 nt = 0, npv = 0, na = 0;
    u32 slices = 0;
    for (u64 a = E->ckpt_pos; a < E->log_next; a += E->wb.cap_t, slices++) {
        const u64 b = std::min<u64>(E->log_next, a + E->wb.cap_t);
        if ((st = wb_gather_slice(E, a, b, true))) return st;
        if ((st = wb_ids(E, E->wb.d_ids, 2 * (b - a), E->wb.d_cnt + WB_RECORDS))) return st;
        hipLaunchKernelGGL(tb_delta_order, dim3(256), dim3(256), 0, E->stream, E->wb.d_out, E->wb.d_cnt + WB_RECORDS,
                           E->wb.d_pairs, E->wb.d_cnt + WB_PV, E->wb.d_cnt + WB_ORDER);
        HIPCK(hipGetLastError());
        if ((st = wb_read_counts(E))) return st;
        const u64* c = E->wb.h_cnt;
        if (c[WB_RECORDS]) HIPCK(hipMemcpyAsync(transfers_out + nt * 128, E->wb.d_out, c[WB_RECORDS] * 128,
                                                hipMemcpyDeviceToHost, E->stream));
        if (c[WB_PV]) HIPCK(hipMemcpyAsync(posted_out + 2 * npv, E->wb.d_pairs, c[WB_PV] * 16, hipMemcpyDeviceToHost,
                                           E->stream));
        nt += c[WB_RECORDS];
        npv += c[WB_PV];
        if ((st = wb_take_accounts(E, accounts_out, before_out, &na))) return st;  // syncs the copies above too
    }
    if ((st = wb_listed_ids(E, E->ckpt_ids, accounts_out, before_out, &na))) return st;
    if ((st = wb_scan(E, 0, 0, accounts_out, before_out, &na))) return st;
    if ((st = wb_advance(E))) return st;
    HIPCK(hipStreamSynchronize(E->stream));
    // Sorted on the device's word (tb_delta_order: within each slice; across slices the host looks).
    const u64 order = E->wb.h_cnt[WB_ORDER];
    if ((order & 1) || slices > 1) delta_sort_by_timestamp(transfers_out, nt);
    if ((order & 2) || slices > 1) delta_sort_pairs(posted_out, npv);
    counts->accounts = na;
    counts->transfers = nt;
    counts->posted = npv;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_checkpoint_delta(tbgpu_t* E, void* accounts_out, void* accounts_before_out, uint64_t accounts_cap,
                                      void* transfers_out, uint64_t transfers_cap, uint64_t* posted_out,
                                      uint64_t posted_cap, tbgpu_delta_counts* counts) {
    API_ENTER(E, true);
    if (E->node) return node_api_checkpoint_delta(E->node, accounts_out, accounts_before_out, accounts_cap, transfers_out,
                                                  transfers_cap, posted_out, posted_cap, counts);
    HIPCK(hipSetDevice(E->device));
    if (E->wb.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight (tbgpu_checkpoint_delta_wait)");
    int st = engine_sync(E);  // the globals (live accounts) and every enqueued commit
    if (st) return st;
    return wb_checkpoint_sync(E, (u8*)accounts_out, (u8*)accounts_before_out, accounts_cap, (u8*)transfers_out,
                              transfers_cap, posted_out, posted_cap, counts);
}

// The durable replica's compact without the wait (tbgpu.h): the bar's delta is gathered on the
// engine stream in stream order (so the next commits follow it), the snapshot advances there, and
// the objects cross PCIe on the write-back stream beside the next commits, straight into the
// caller's registered buffers (tb_delta_out).  When a precondition does not hold, the write-back runs
// synchronously instead and tbgpu_checkpoint_delta_wait returns at once.
extern "C" int tbgpu_checkpoint_delta_async(tbgpu_t* E, void* accounts_out, void* accounts_before_out,
                                            uint64_t accounts_cap, void* transfers_out, uint64_t transfers_cap,
                                            uint64_t* posted_out, uint64_t posted_cap) {
    API_ENTER(E, true);
    if (E->node) return node_api_checkpoint_delta_async(E->node, accounts_out, accounts_before_out, accounts_cap,
                                                        transfers_out, transfers_cap, posted_out, posted_cap);
    HIPCK(hipSetDevice(E->device));
    WbBufs& W = E->wb;
    if (W.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight (tbgpu_checkpoint_delta_wait)");
    if (E->pending) {
        const int st = engine_sync(E);
        if (st) return st;
    }
    int st = ckpt_snapshot_ready(E);
    if (st) return st;
    const u64 range = E->log_next - E->ckpt_pos;
    const WbBounds bd = wb_bounds(E, ~0ULL);
    // The caller's buffers, device-mapped (registered memory).
    auto mapped = [&](const void* p, u64 bytes) -> u8* {
        for (const auto& r : E->host_regions) {
            if ((const u8*)p >= r.ptr && (const u8*)p + bytes <= r.ptr + r.bytes) return (u8*)r.dev + ((const u8*)p - r.ptr);
        }
        return nullptr;
    };
    u8* m_acc = mapped(accounts_out, bd.accounts * 128);
    u8* m_before = accounts_before_out ? mapped(accounts_before_out, bd.accounts * sizeof(AccountBal)) : nullptr;
    u8* m_t = mapped(transfers_out, bd.transfers * 128);
    u8* m_p = mapped(posted_out, bd.posted * 16);
    const bool fits = !E->ckpt_scan && range <= W.cap_t && E->ckpt_ids.size() / 2 <= W.cap_ids &&
                      bd.accounts <= W.cap_a && bd.accounts <= accounts_cap && bd.transfers <= transfers_cap &&
                      bd.posted <= posted_cap && m_acc && m_t && m_p && (m_before || !accounts_before_out);
    W.out_t = (u8*)transfers_out;
    W.out_p = posted_out;
    if (!fits) {  // the synchronous write-back, its result kept for the wait
        st = engine_sync(E);
        if (!st) st = wb_checkpoint_sync(E, (u8*)accounts_out, (u8*)accounts_before_out, accounts_cap, (u8*)transfers_out,
                                         transfers_cap, posted_out, posted_cap, &W.counts);
        if (st) return st;
        W.h_cnt[WB_RECORDS] = W.counts.transfers;
        W.h_cnt[WB_PV] = W.counts.posted;
        W.h_cnt[WB_ACCOUNTS] = W.counts.accounts;
        W.h_cnt[WB_STATUS] = 0;
        W.out_t = nullptr;  // already sorted
        W.out_p = nullptr;
        for (u32 r = 0; r < 4; r++) W.dst[r] = nullptr;  // nothing is copied into the caller's buffers later
        HIPCK(hipEventRecord(W.done, E->stream));
        W.inflight = true;
        return TBGPU_STATUS_OK;
    }
    memset(&W.counts, 0, sizeof(W.counts));
    W.counts.created_after = E->ckpt_ts;
    W.calls = 0;
    if ((st = wb_next_epoch(E))) return st;
    HIPCK(hipMemsetAsync(W.d_cnt, 0, WB_COUNT_WORDS * 8, E->stream));
    // In stream order (the next commits follow): each account the bar's log range names, its slot and
    // its balances as of the bar (tb_delta_capture_log).
    if (range) {
        hipLaunchKernelGGL(tb_delta_capture_log, dim3((unsigned)((range + 255) / 256)), dim3(256), 0, E->stream, E->T,
                           E->ckpt_pos, range, E->ckpt_mark, E->ckpt_epoch, W.d_slots, W.d_cap, W.d_cnt + WB_SLOTS);
    }
    const u64 nl = E->ckpt_ids.size() / 2;
    if (nl) {  // the listed ids cross in the same stream order (their host copy lives until then)
        W.ids_inflight.swap(E->ckpt_ids);
        HIPCK(hipMemcpyAsync(W.d_hids, W.ids_inflight.data(), nl * 16, hipMemcpyHostToDevice, E->stream));
        hipLaunchKernelGGL(tb_delta_capture, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, E->stream, E->T, W.d_hids, nl,
                           E->ckpt_mark, E->ckpt_epoch, W.d_slots, W.d_cap, W.d_cnt + WB_SLOTS, nullptr);
    }
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(W.captured, E->stream));
    // The rest runs on the write-back stream beside the commits, enqueued by the next commit (wb_tail)
    // so that it overlaps that commit's later kernels rather than the first one after the bar.
    W.tail = true;
    W.tail_pos0 = E->ckpt_pos;
    W.tail_pos1 = E->log_next;
    W.tail_ts0 = E->ckpt_ts;
    E->ckpt_pos = E->log_next;  // wb_advance's host part (the snapshot advances on the write-back stream)
    E->ckpt_ts = E->commit_ts;
    E->ckpt_scan = false;
    E->ckpt_ids.clear();  // (holds the previous write-back's list after the swap above)
    W.src[0] = W.d_out;
    W.dst[0] = (u8*)transfers_out;
    W.src[1] = W.d_acc;
    W.dst[1] = (u8*)accounts_out;
    W.src[2] = accounts_before_out ? (const u8*)W.d_before : nullptr;
    W.dst[2] = (u8*)accounts_before_out;
    W.src[3] = (const u8*)W.d_pairs;
    W.dst[3] = (u8*)posted_out;
    W.copying = true;
    W.counts_known = false;
    W.bound_len[0] = bd.transfers;
    W.bound_len[1] = bd.accounts;
    W.bound = E->wb_bound_ok && W.bound_ok && W.calls_prev >= 2;
    W.posted_late = false;
    W.n_async++;
    if (W.bound) {
        W.n_bound++;  // the sizes are known now: wb_pump sends from the first commit on
        W.len[0] = bd.transfers * 128;
        W.len[1] = bd.accounts * 128;
        W.len[2] = W.src[2] ? bd.accounts * sizeof(AccountBal) : 0;
        W.len[3] = 0;  // posted pairs (usually none) cross at the wait, by their count
        W.posted_late = true;
        for (u32 r = 0; r < 4; r++) W.at[r] = 0;
        wb_set_slice(E, W.len[0] + W.len[1] + W.len[2]);
        W.counts_known = true;
        // The gather and the whole copy-out are enqueued by the next commit, right after its own
        // kernels (the host issues them while the device runs that commit): the sizes need no
        // counts, nothing waits for the commit's reads — a replica writing back every few ops stages
        // its bodies while the copy-out crosses (tbgpu_prefetch) — and the counts cross last.
    }
    W.inflight = true;
    return TBGPU_STATUS_OK;
}

// A write-back's copy-out still issuing or still crossing the link.
static bool wb_copy_in_flight(tbgpu* E) {
    const WbBufs& W = E->wb;
    return W.inflight && (W.copying || hipEventQuery(W.done) == hipErrorNotReady);
}

// The copy-out of an asynchronous write-back, a slice at a time (up to `budget` bytes; ~0: all of
// it), by the DMA engine on the write-back stream — after `after` (when given) on the engine stream.
// A device-initiated read from host memory may not pass the posted writes queued before it on the
// link, so a copy-out streaming 100+ MB beside a one-prepare commit held that commit's body read for
// milliseconds, and a copy kernel's host writes also crowded the L2 every other kernel shares.  So
// each commit sends one slice after its validate has read the body (the slice then overlaps its
// resolve, apply, flow and reply and the host's turn), sized to spread the bar's objects over about
// WB_SLICE_CALLS commits.  The sizes come from the gather's counts, known once it completed.
#define WB_SLICE_CALLS 56
// The slice: the copy-out spread over the commits the previous write-back saw before its wait, less
// the one that enqueues the gather and (counts mode) the one that learns its sizes — a chunked
// write-back every few ops would otherwise leave most of its bytes to a synchronous copy at the wait.
static void wb_set_slice(tbgpu* E, u64 total) {
    WbBufs& W = E->wb;
    const u32 skip = W.bound ? 1 : 2;
    const u32 spread = W.calls_prev ? std::max<u32>(1, std::min<u32>(WB_SLICE_CALLS, W.calls_prev > skip ? W.calls_prev - skip : 1))
                                     : WB_SLICE_CALLS;
    W.slice = std::max<u64>(512 << 10, (total / spread + 65535) & ~65535ULL);
}
// The asynchronous write-back's work beside the commits, after the in-order capture (and `after`):
// the records of the log range (immutable now), the emission, the snapshot's advance, the order
// check, the counts back to the host (counts = false: the caller copies them after the objects —
// a bound-sized copy-out needs them only at the wait).
static int wb_tail(tbgpu* E, hipEvent_t after, bool counts) {
    WbBufs& W = E->wb;
    W.tail = false;
    HIPCK(hipStreamWaitEvent(W.stream, W.captured, 0));
    if (after) HIPCK(hipStreamWaitEvent(W.stream, after, 0));
    const u64 ts = E->ckpt_ts;  // wb_gather_slice reads the previous write-back's timestamp
    E->ckpt_ts = W.tail_ts0;
    const int st = wb_gather_slice(E, W.tail_pos0, W.tail_pos1, true, true, W.stream, false);  // (zeroed at the call)
    E->ckpt_ts = ts;
    if (st) return st;
    hipLaunchKernelGGL(tb_delta_emit, dim3(1024), dim3(256), 0, W.stream, E->T, ckpt_view(E), W.tail_ts0, W.d_slots, W.d_cap,
                       W.d_cnt + WB_SLOTS, W.d_acc, W.d_before, W.d_cnt + WB_ACCOUNTS);
    hipLaunchKernelGGL(tb_delta_advance_from, dim3(1024), dim3(256), 0, W.stream, ckpt_view(E), W.d_slots, W.d_cap,
                       W.d_cnt + WB_SLOTS);
    hipLaunchKernelGGL(tb_delta_order, dim3(256), dim3(256), 0, W.stream, W.d_out, W.d_cnt + WB_RECORDS, W.d_pairs,
                       W.d_cnt + WB_PV, W.d_cnt + WB_ORDER);
    HIPCK(hipGetLastError());
    if (counts) {
        HIPCK(hipMemcpyAsync(W.h_cnt, W.d_cnt, WB_COUNT_WORDS * 8, hipMemcpyDeviceToHost, W.stream));
        HIPCK(hipEventRecord(W.gathered, W.stream));
    }
    return TBGPU_STATUS_OK;
}

static int wb_pump(tbgpu* E, u64 budget, hipEvent_t after) {
    WbBufs& W = E->wb;
    if (!W.copying) return TBGPU_STATUS_OK;
    if (W.tail) {  // (bound-sized: nothing waits for the commit's reads, the counts go last)
        const int st = wb_tail(E, W.bound ? nullptr : after, !W.bound);
        if (st || (budget != ~0ULL && !W.counts_known)) return st;  // its counts come back by the next commit
    }
    if (!W.counts_known) {
        if (budget != ~0ULL && hipEventQuery(W.gathered) != hipSuccess) return TBGPU_STATUS_OK;  // next call
        HIPCK(hipEventSynchronize(W.gathered));
        const u64 na = W.h_cnt[WB_ACCOUNTS];
        W.len[0] = W.h_cnt[WB_RECORDS] * 128;
        W.len[1] = na * 128;
        W.len[2] = W.src[2] ? na * sizeof(AccountBal) : 0;
        W.len[3] = W.h_cnt[WB_PV] * 16;
        u64 total = 0;
        for (u32 r = 0; r < 4; r++) {
            W.at[r] = 0;
            total += W.len[r];
        }
        wb_set_slice(E, total);
        W.counts_known = true;
    }
    // A commit that read no host memory (its body staged in HBM) leaves the link's upstream side to
    // the copy-out: everything goes now.  Otherwise one slice, after the commit's reads.
    if (budget != ~0ULL) budget = W.staged_reads || W.bound ? ~0ULL : W.slice;
    if (after && !W.staged_reads && !W.bound) HIPCK(hipStreamWaitEvent(W.stream, after, 0));
    for (u32 r = 0; r < 4 && budget; r++) {
        const u64 n = std::min<u64>(budget, W.len[r] - W.at[r]);
        if (!n) continue;
        HIPCK(hipMemcpyAsync(W.dst[r] + W.at[r], W.src[r] + W.at[r], n, hipMemcpyDeviceToHost, W.stream));
        W.at[r] += n;
        budget -= n;
    }
    bool left = false;
    for (u32 r = 0; r < 4; r++) left |= W.at[r] < W.len[r];
    if (!left) {
        if (W.bound) HIPCK(hipMemcpyAsync(W.h_cnt, W.d_cnt, WB_COUNT_WORDS * 8, hipMemcpyDeviceToHost, W.stream));  // for the wait
        HIPCK(hipEventRecord(W.done, W.stream));
        W.copying = false;
    }
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_checkpoint_delta_wait(tbgpu_t* E, tbgpu_delta_counts* counts) {
    API_ENTER(E, false);
    memset(counts, 0, sizeof(*counts));
    if (E->node) return node_api_checkpoint_delta_wait(E->node, counts);
    HIPCK(hipSetDevice(E->device));
    return wb_wait(E, counts);
}

extern "C" int tbgpu_get_stats(tbgpu_t* E, tbgpu_stats* s) {
    API_ENTER(E, false);
    if (E->node) return node_api_get_stats(E->node, s);
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    Globals g;
    HIPCK(hipMemcpy(&g, E->g, sizeof(Globals), hipMemcpyDeviceToHost));
    memset(s, 0, sizeof(*s));
    s->passes = E->passes;
    s->account_table_bytes = E->account_cap * (sizeof(AccountHot) + sizeof(AccountBal) + sizeof(AccountCold) + 4);
    s->transfers_evicted = E->evicted_total;
    s->log_used = E->log_next;
    s->log_capacity = E->xlog_cap;
    s->write_backs_async = E->wb.n_async;
    s->write_backs_bound = E->wb.n_bound;
    s->events = E->events;
    s->dependent_events = g.dependent_all;
    s->accounts = g.account_count;
    s->transfers = g.transfer_count;
    s->ms_validate = E->prof_ms[K_VALIDATE];
    s->ms_resolve = E->prof_ms[K_RESOLVE];
    s->ms_replay = E->prof_ms[K_REPLAY];
    s->ms_clear = E->prof_ms[K_CLEAR];
    s->launches_validate = E->prof_n[K_VALIDATE];
    s->launches_resolve = E->prof_n[K_RESOLVE];
    s->launches_replay = E->prof_n[K_REPLAY];
    s->launches_clear = E->prof_n[K_CLEAR];
    s->ms_apply = E->prof_ms[K_APPLY];
    s->launches_apply = E->prof_n[K_APPLY];
    for (u32 k = 0; k < 3; k++) {
        s->span_ms[k] = E->span_ms[k];
        s->span_launches[k] = E->span_n[k];
    }
    s->flow_passes = g.flow_passes;
    s->flow_units = g.flow_units;
    s->flow_runs = g.flow_runs;
    s->flow_run_units = g.flow_run_units;
    s->flow_plan_ms = E->wall_khz ? (double)g.flow_plan_ticks / E->wall_khz : 0.0;
    s->flow_run_ms = E->wall_khz ? (double)g.flow_run_ticks / E->wall_khz : 0.0;
    s->bounds_passes = g.bounds_passes;
    s->bounds_units = g.bounds_units;
    s->bounds_rounds = g.bounds_rounds;
    s->bounds_skipped = g.bounds_skipped;
    s->bounds_abandoned = g.bounds_abandoned;
    s->bounds_swept = g.bounds_swept;
    s->sweep_ms = E->wall_khz ? (double)g.sweep_ticks[0] / E->wall_khz : 0.0;
    s->sweep_loop_ms = E->wall_khz ? (double)g.sweep_ticks[1] / E->wall_khz : 0.0;
    s->sweep_wait_ms = E->wall_khz ? (double)g.sweep_ticks[2] / E->wall_khz : 0.0;
    s->sweep_u64_passes = g.sweep_u64_passes;
    s->flow_exec_ms = E->wall_khz ? (double)g.flow_exec_ticks / E->wall_khz : 0.0;
    for (int k = 0; k < 8; k++) s->flow_phase_ms[k] = E->wall_khz ? (double)g.flow_phase_ticks[k] / E->wall_khz : 0.0;
    s->walk_segments = g.walk[0];
    s->walk_heavy = g.walk[1];
    s->walk_heavy_positions = g.walk[2];
    s->walk_heavy_windows = g.walk[3];
    s->walk_heavy_stops = g.walk[4];
    s->walk_heavy_blocks = g.walk[5];
    s->walk_heavy_blocked_ms = E->wall_khz ? (double)g.walk[6] / E->wall_khz : 0.0;
    s->walk_longest = g.walk[7];
    s->walk_crit_windows = g.walk[8];
    s->walk_crit_blocks = g.walk[9];
    s->walk_crit_wait_ms = E->wall_khz ? (double)g.walk[10] / E->wall_khz : 0.0;
    s->walk_crit_ms = E->wall_khz ? (double)g.walk[11] / E->wall_khz : 0.0;
    for (int k = 0; k < 4; k++) s->walk_dbg[k] = g.walk_dbg[k];
    return TBGPU_STATUS_OK;
}

extern "C" void tbgpu_reset_stats(tbgpu_t* E) {
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) tbgpu_reset_stats(node_engine(E->node, d));
        node_reset_stats(E->node);
        return;
    }
    for (int k = 0; k < K_COUNT; k++) {
        E->prof_ms[k] = 0;
        E->prof_n[k] = 0;
    }
    for (int k = 0; k < 3; k++) {
        E->span_ms[k] = 0;
        E->span_n[k] = 0;
    }
    E->passes = 0;
    E->events = 0;
    E->pass_ms.clear();
}

extern "C" const char* tbgpu_last_error(void) { return g_err.c_str(); }

extern "C" uint64_t tbgpu_debug_allocations(void) { return g_allocs.load(); }

// vsr.checksum (src/vsr/checksum.zig:50): host only, no device or engine needed.
extern "C" void tbgpu_checksum(const void* data, uint64_t len, uint8_t out[16]) {
    tbck::checksum((const u8*)data, len, out);
}

// ------------------------------------------------------------------------------------------------
// tbgpu_bench.h
// ------------------------------------------------------------------------------------------------

static WorkloadParams workload_params(const tbgpu_workload* w, u64 first) {
    WorkloadParams W{};
    W.seed = w->seed;
    W.account_count = w->account_count;
    W.first_index = first;
    W.kind = w->kind;
    W.limit_permille = w->limit_permille;
    W.zipf_s = w->zipf_s > 0 ? w->zipf_s : 1.2;
    // Rank permutation r -> (a r + b) mod n with gcd(a, n) = 1.
    const u64 n = std::max<u64>(w->account_count, 1);
    u64 a = (0x9E3779B97F4A7C15ULL ^ w->seed) % n;
    if (a == 0) a = 1;
    while (std::gcd(a, n) != 1) a = a + 1 == n ? 1 : a + 1;
    W.perm_a = a;
    W.perm_b = tb_splitmix(w->seed ^ 0x5bd1e995ULL) % n;
    W.hot_limited = w->account_count >= 2 ? w->hot_limited : 0;
    return W;
}

extern "C" int tbgpu_bench_generate_accounts(tbgpu_t* E, void* out_dev, uint64_t first, uint64_t count,
                                             const tbgpu_workload* w) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    if (count == 0) return TBGPU_STATUS_OK;
    hipLaunchKernelGGL(tb_gen_accounts, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, E->stream,
                       (u8*)out_dev, first, count, workload_params(w, first));
    HIPCK(hipGetLastError());
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_generate_transfers(tbgpu_t* E, void* out_dev, uint64_t first, uint64_t count,
                                              const tbgpu_workload* w) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    if (count == 0) return TBGPU_STATUS_OK;
    if (w->account_count < 2) return fail(TBGPU_STATUS_INVALID, "need at least two accounts");
    hipLaunchKernelGGL(tb_gen_transfers, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, E->stream,
                       (u8*)out_dev, count, workload_params(w, first));
    HIPCK(hipGetLastError());
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_node_shard(tbgpu_t* E, uint32_t shard, tbgpu_t** out) {
    API_ENTER(E, false);
    *out = nullptr;
    if (!E->node || shard >= node_world(E->node)) return fail(TBGPU_STATUS_INVALID, "not a node shard");
    *out = node_engine(E->node, shard);
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_walk_merge_max(tbgpu_t* E, uint32_t segments) {
    API_ENTER(E, false);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) tbgpu_bench_walk_merge_max(node_engine(E->node, d), segments);
        return TBGPU_STATUS_OK;
    }
    E->F.walk_merge = std::min<u32>(segments, WALK_MERGE_MAX);
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_flow_launch(tbgpu_t* E, uint32_t workgroups) {
    API_ENTER(E, false);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) tbgpu_bench_flow_launch(node_engine(E->node, d), workgroups);
        return TBGPU_STATUS_OK;
    }
    E->flow_launch = workgroups;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_legs_min_events(tbgpu_t* E, uint32_t events) {
    API_ENTER(E, false);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) tbgpu_bench_legs_min_events(node_engine(E->node, d), events);
        return TBGPU_STATUS_OK;
    }
    E->legs_min = events;
    return TBGPU_STATUS_OK;
}

template <u32 M>
static float access_mix_ms(tbgpu_t* E, const MixArgs& A, int reps) {
    const dim3 grid((unsigned)((A.n + 255) / 256));
    float total = 0;
    for (int r = 0; r <= reps; r++) {  // the first launch warms up
        if (hipMemsetAsync(A.index, 0, (A.index_mask + 1) * 8, E->stream) != hipSuccess) return -1;  // empty slots
        if (hipEventRecord(E->markers[14], E->stream) != hipSuccess) return -1;
        hipLaunchKernelGGL(tb_access_mix<M>, grid, dim3(256), 0, E->stream, A);
        if (hipEventRecord(E->markers[15], E->stream) != hipSuccess) return -1;
        if (hipEventSynchronize(E->markers[15]) != hipSuccess) return -1;
        float ms = 0;
        if (hipEventElapsedTime(&ms, E->markers[14], E->markers[15]) != hipSuccess) return -1;
        if (r > 0) total += ms;
    }
    return total / reps;
}

extern "C" int tbgpu_bench_access_mix(tbgpu_t* E, uint64_t transfers, double out_ms[7]) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    HIPCK(hipStreamSynchronize(E->stream));
    MixArgs A = {};
    A.n = transfers;
    const u64 rows = E->account_cap;
    A.row_mask = rows - 1;
    A.index_mask = E->xidx_cap - 1;
    void *ev = nullptr, *rec = nullptr, *s4 = nullptr, *s2 = nullptr, *s8 = nullptr, *rw = nullptr, *ix = nullptr,
         *sink = nullptr;
    int st = TBGPU_STATUS_OK;
    if (tbMalloc(&ev, transfers * 128) != hipSuccess || tbMalloc(&rec, transfers * 128) != hipSuccess ||
        tbMalloc(&s4, transfers * 16) != hipSuccess || tbMalloc(&s2, transfers * 2) != hipSuccess ||
        tbMalloc(&s8, transfers * 24) != hipSuccess || tbMalloc(&rw, rows * 32) != hipSuccess ||
        tbMalloc(&ix, E->xidx_cap * 8) != hipSuccess || tbMalloc(&sink, 8) != hipSuccess ||
        hipMemsetAsync(ev, 1, transfers * 128, E->stream) != hipSuccess ||
        hipMemsetAsync(rw, 2, rows * 32, E->stream) != hipSuccess) {
        st = fail(TBGPU_STATUS_DEVICE, "access mix: allocation failed");
    } else {
        A.events = (const uint4*)ev;
        A.records = (uint4*)rec;
        A.s4 = (u32*)s4;
        A.s2 = (unsigned short*)s2;
        A.s8 = (u64*)s8;
        A.rows = (const uint4*)rw;
        A.index = (u64*)ix;
        A.sink = (u64*)sink;
        const int reps = 5;
        const float t[7] = {access_mix_ms<MIX_STREAM>(E, A, reps), access_mix_ms<MIX_PROBE>(E, A, reps),
                            access_mix_ms<MIX_CAS>(E, A, reps), access_mix_ms<MIX_STREAM | MIX_PROBE>(E, A, reps),
                            access_mix_ms<MIX_STREAM | MIX_CAS>(E, A, reps), access_mix_ms<MIX_PROBE | MIX_CAS>(E, A, reps),
                            access_mix_ms<MIX_STREAM | MIX_PROBE | MIX_CAS>(E, A, reps)};
        for (int k = 0; k < 7; k++) {
            out_ms[k] = t[k];
            if (t[k] < 0) st = fail(TBGPU_STATUS_DEVICE, "access mix: launch failed");
        }
    }
    void* bufs[] = {ev, rec, s4, s2, s8, rw, ix, sink};
    for (void* p : bufs) if (p) (void)hipFree(p);
    return st;
}

extern "C" int tbgpu_bench_profile_mask(tbgpu_t* E, uint32_t mask) {
    API_ENTER(E, false);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) tbgpu_bench_profile_mask(node_engine(E->node, d), mask);
        return TBGPU_STATUS_OK;
    }
    E->prof_mask = mask;
    return TBGPU_STATUS_OK;
}

static int ledger_summary(tbgpu* E, u32 world, u32 self, u64 out[10]) {
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    u64* d = nullptr;
    HIPCK(tbMalloc(&d, 80));
    hipError_t e = hipMemsetAsync(d, 0, 80, E->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(tb_ledger_summary, dim3((unsigned)((E->account_cap + 255) / 256)), dim3(256), 0, E->stream, E->T,
                           E->account_cap, world, self, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, 80, hipMemcpyDeviceToHost, E->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(E->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "ledger summary: %s", hipGetErrorString(e));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_ledger_summary(tbgpu_t* E, tbgpu_ledger_summary* out) {
    API_ENTER(E, false);
    memset(out, 0, sizeof(*out));
    const u32 W = E->node ? node_world(E->node) : 1;
    for (u32 d = 0; d < W; d++) {
        u64 v[10];
        const int st = ledger_summary(E->node ? node_engine(E->node, d) : E, E->node ? W : 0, d, v);
        if (st) return st;
        for (int f = 0; f < 4; f++) {  // u128 adds (wrapping, as the reference's balances never wrap)
            const u64 lo = out->sums[2 * f] + v[2 * f];
            out->sums[2 * f + 1] += v[2 * f + 1] + (lo < out->sums[2 * f] ? 1 : 0);
            out->sums[2 * f] = lo;
        }
        out->accounts += v[8];  // on a node, each account on its owner only
        out->stray += v[9];
    }
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_device_alloc(tbgpu_t* E, uint64_t bytes, void** out) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    HIPCK(tbMalloc(out, bytes));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_device_free(tbgpu_t* E, void* ptr) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    HIPCK(hipFree(ptr));
    return TBGPU_STATUS_OK;
}

// The replica's message pool is allocated once at init (static allocation); registering it lets
// the prepare bodies go to HBM by DMA straight from the message, with no staging copy.
extern "C" int tbgpu_register_host(tbgpu_t* E, void* ptr, uint64_t bytes) {
    API_ENTER(E, false);
    if (E->node) return node_api_register_host(E->node, ptr, bytes);
    HIPCK(hipSetDevice(E->device));
    HIPCK(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
    void* dev = nullptr;
    HIPCK(hipHostGetDevicePointer(&dev, ptr, 0));
    E->host_regions.push_back({(const u8*)ptr, bytes, (const u8*)dev});
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_unregister_host(tbgpu_t* E, void* ptr) {
    API_ENTER(E, false);
    if (E->node) return node_api_unregister_host(E->node, ptr);
    HIPCK(hipSetDevice(E->device));
    // A region an asynchronous write-back is still copying into belongs to the engine until
    // tbgpu_checkpoint_delta_wait (tbgpu.h): refuse it rather than unpin pages under the DMA.
    if (E->wb.inflight) {
        for (const auto& r : E->host_regions) {
            if (r.ptr != (const u8*)ptr) continue;
            for (u32 k = 0; k < 4; k++) {
                if (E->wb.dst[k] && E->wb.dst[k] >= r.ptr && E->wb.dst[k] < r.ptr + r.bytes) {
                    return fail(TBGPU_STATUS_INVALID, "unregister: an asynchronous write-back is copying into this "
                                                      "region (tbgpu_checkpoint_delta_wait first)");
                }
            }
        }
    }
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    HIPCK(hipStreamSynchronize(E->stream));
    HIPCK(hipStreamSynchronize(E->wb.stream));  // no copy-out slice still in flight
    for (size_t i = 0; i < E->host_regions.size(); i++) {
        if (E->host_regions[i].ptr == (const u8*)ptr) {
            E->host_regions.erase(E->host_regions.begin() + i);
            break;
        }
    }
    HIPCK(hipHostUnregister(ptr));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_copy_to_host(tbgpu_t* E, void* dst, const void* src_dev, uint64_t bytes) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    HIPCK(hipStreamSynchronize(E->stream));
    HIPCK(hipMemcpy(dst, src_dev, bytes, hipMemcpyDeviceToHost));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_copy_to_device(tbgpu_t* E, void* dst_dev, const void* src, uint64_t bytes) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    HIPCK(hipSetDevice(E->device));
    HIPCK(hipStreamSynchronize(E->stream));
    HIPCK(hipMemcpy(dst_dev, src, bytes, hipMemcpyHostToDevice));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_reset_transfers(tbgpu_t* E) {
    API_ENTER(E, true);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) {
            const int st = tbgpu_bench_reset_transfers(node_engine(E->node, d));
            if (st) return st;
        }
        return TBGPU_STATUS_OK;
    }
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    HIPCK(hipMemsetAsync(E->T.xidx, 0, E->xidx_cap * sizeof(u64), E->stream));
    HIPCK(hipMemsetAsync(E->T.xdup, 0, E->xidx_cap, E->stream));
    HIPCK(hipMemsetAsync(E->T.xposted, 0, E->xlog_cap, E->stream));
    hipLaunchKernelGGL(tb_zero_balances, dim3((unsigned)((E->account_cap + 255) / 256)), dim3(256), 0, E->stream, E->T,
                       E->account_cap);
    E->log_next = 0;
    E->ckpt_valid = false;
    E->ckpt_scan = true;  // the accounts stay, created before the (empty) snapshot
    HIPCK(hipGetLastError());
    HIPCK(hipStreamSynchronize(E->stream));
    return TBGPU_STATUS_OK;
}

// Bench: take the current state as written back (the snapshot, the log and commit positions), so
// the next tbgpu_checkpoint_delta covers only what is committed after this call.
extern "C" int tbgpu_bench_checkpoint_mark(tbgpu_t* E) {
    API_ENTER(E, true);
    if (E->node) {
        for (u32 d = 0; d < node_world(E->node); d++) {
            const int st = tbgpu_bench_checkpoint_mark(node_engine(E->node, d));
            if (st) return st;
        }
        return TBGPU_STATUS_OK;
    }
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    if (E->wb.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight");
    int st = ckpt_snapshot_ready(E);
    if (st) return st;
    E->ckpt_scan = true;  // the whole table is taken as written back
    if ((st = wb_advance(E))) return st;
    HIPCK(hipStreamSynchronize(E->stream));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_bench_pass_latencies(tbgpu_t* E, double* out_ms, uint64_t cap, uint64_t* count) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    const u64 n = std::min<u64>(cap, E->pass_ms.size());
    for (u64 i = 0; i < n; i++) out_ms[i] = E->pass_ms[i];
    *count = n;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_marker(tbgpu_t* E, uint32_t slot) {
    API_ENTER(E, false);
    if (E->node) E = node_engine(E->node, 0);
    if (slot >= 16) return fail(TBGPU_STATUS_INVALID, "marker slot");
    HIPCK(hipEventRecord(E->markers[slot], E->stream));
    return TBGPU_STATUS_OK;
}

extern "C" double tbgpu_marker_elapsed_ms(tbgpu_t* E, uint32_t a, uint32_t b) {
    if (E->node) E = node_engine(E->node, 0);
    float ms = -1;
    if (a >= 16 || b >= 16) return -1;
    if (hipEventSynchronize(E->markers[b]) != hipSuccess) return -1;
    if (hipEventElapsedTime(&ms, E->markers[a], E->markers[b]) != hipSuccess) return -1;
    return ms;
}

// ------------------------------------------------------------------------------------------------
// tbgpu_shard.h
// ------------------------------------------------------------------------------------------------

extern "C" uint32_t tbgpu_home(uint64_t id_lo, uint64_t id_hi, uint32_t world) { return tb_home(id_lo, id_hi, world); }

extern "C" void tbgpu_homes(const uint64_t* ids, uint64_t n, uint32_t world, uint32_t* out) {
    for (u64 i = 0; i < n; i++) out[i] = tb_home(ids[2 * i], ids[2 * i + 1], world);
}

extern "C" int tbgpu_route_init(tbgpu_t* E, uint32_t world, uint64_t events_max) {
    API_ENTER(E, false);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (world == 0 || world > ROUTE_WORLD_MAX) return fail(TBGPU_STATUS_INVALID, "world %u out of range", world);
    if (E->r_home) return fail(TBGPU_STATUS_INVALID, "tbgpu_route_init called twice");
    if (events_max == 0 || events_max >= (1ULL << 32)) return fail(TBGPU_STATUS_INVALID, "route events_max out of range");
    E->route_world = world;
    E->route_events_max = events_max;
    const u64 nblocks = (events_max + ROUTE_THREADS - 1) / ROUTE_THREADS;
    HIPCK(tbMalloc(&E->r_home, events_max));
    HIPCK(tbMalloc(&E->r_block_counts, 2 * nblocks * world * 4));  // counts, then bases
    E->r_block_cap = nblocks * world;
    HIPCK(tbMalloc(&E->r_words, ROUTE_WORDS * 8));
    HIPCK(tbMalloc(&E->r_meta, (2 * E->meta_cap + 1) * 8));
    HIPCK(tbHostMalloc(&E->h_rmeta, (2 * E->meta_cap + 1) * 8, hipHostMallocDefault));
    return TBGPU_STATUS_OK;
}

// Upload a local batch structure (offsets, timestamps) to r_meta; returns total events.
static int route_meta(tbgpu* E, u32 nb, const u64* timestamps, const u32* lens, u64* total) {
    if (nb > E->meta_cap) return fail(TBGPU_STATUS_INVALID, "too many batches (%u)", nb);
    HIPCK(hipStreamSynchronize(E->stream));  // the pinned mirror may still be in flight
    u64* off = E->h_rmeta;
    u64* ts = E->h_rmeta + nb + 1;
    off[0] = 0;
    for (u32 k = 0; k < nb; k++) {
        if (lens[k] > BATCH_EVENTS_MAX) return fail(TBGPU_STATUS_INVALID, "batch %u has %u events", k, lens[k]);
        off[k + 1] = off[k] + lens[k];
        ts[k] = timestamps ? timestamps[k] : 0;
        if (timestamps && lens[k] && timestamps[k] < lens[k]) return fail(TBGPU_STATUS_PANIC, "timestamp < batch length");
    }
    HIPCK(hipMemcpyAsync(E->r_meta, E->h_rmeta, (2 * (u64)nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
    *total = off[nb];
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_route_homes(tbgpu_t* E, const uint64_t* ids_dev, uint64_t n, uint32_t world, uint8_t* out_dev) {
    API_ENTER(E, false);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (world == 0 || world > ROUTE_WORLD_MAX) return fail(TBGPU_STATUS_INVALID, "world %u out of range", world);
    if (n == 0) return TBGPU_STATUS_OK;
    hipLaunchKernelGGL(tb_route_homes, dim3((u32)((n + 255) / 256)), dim3(256), 0, E->stream, ids_dev, n, world, out_dev);
    HIPCK(hipGetLastError());
    HIPCK(hipStreamSynchronize(E->stream));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_route_dependents(tbgpu_t* E, uint32_t nb, const uint32_t* lens, const void* events_dev,
                                      const uint64_t* marked_ids, uint32_t n_marked, uint8_t* dep_dev) {
    API_ENTER(E, false);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (!E->r_home) return fail(TBGPU_STATUS_INVALID, "tbgpu_route_init was not called");
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    u64 n = 0;
    int st = route_meta(E, nb, nullptr, lens, &n);
    if (st) return st;
    if (n == 0) return TBGPU_STATUS_OK;
    u64* d_marked = nullptr;
    if (n_marked) {
        HIPCK(tbMalloc(&d_marked, (u64)n_marked * 16));
        HIPCK(hipMemcpyAsync(d_marked, marked_ids, (u64)n_marked * 16, hipMemcpyHostToDevice, E->stream));
    }
    RouteArgs A{};
    A.events = (const u8*)events_dev;
    A.n = (u32)n;
    A.nb = nb;
    A.batch_off = E->r_meta;
    A.T = E->T;
    hipLaunchKernelGGL(tb_route_dependents, dim3((u32)((n + ROUTE_THREADS - 1) / ROUTE_THREADS)), dim3(ROUTE_THREADS), 0,
                       E->stream, A, d_marked, n_marked, dep_dev);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(E->stream);
    if (d_marked) (void)hipFree(d_marked);
    if (e != hipSuccess) return fail(TBGPU_STATUS_DEVICE, "route dependents: %s", hipGetErrorString(e));
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_route_plan_build(tbgpu_t* E, uint32_t nb, const uint64_t* timestamps, const uint32_t* lens,
                                      const void* events_dev, const uint8_t* skip_dev, void* send_events_dev,
                                      uint32_t* slot_dev, tbgpu_route_plan* plan) {
    API_ENTER(E, false);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (!E->r_home) return fail(TBGPU_STATUS_INVALID, "tbgpu_route_init was not called");
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    u64 n = 0;
    int st = route_meta(E, nb, timestamps, lens, &n);
    if (st) return st;
    if (n > E->route_events_max) return fail(TBGPU_STATUS_INVALID, "pass has %llu events > route capacity %llu",
                                             (unsigned long long)n, (unsigned long long)E->route_events_max);
    memset(plan, 0, sizeof(*plan));
    HIPCK(hipMemsetAsync(E->r_words, 0, ROUTE_WORDS * 8, E->stream));
    RouteArgs A{};
    A.events = (const u8*)events_dev;
    A.n = (u32)n;
    A.nb = nb;
    A.batch_off = E->r_meta;
    A.batch_ts = E->r_meta + nb + 1;
    A.world = E->route_world;
    A.nblocks = (u32)((n + ROUTE_THREADS - 1) / ROUTE_THREADS);
    A.home = E->r_home;
    A.block_counts = E->r_block_counts;
    A.block_base = E->r_block_counts + E->r_block_cap;
    A.words = E->r_words;
    A.T = E->T;
    A.skip = skip_dev;
    if (n > 0) {
        hipLaunchKernelGGL(tb_route_classify, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, E->stream, A);
        HIPCK(hipGetLastError());
        hipLaunchKernelGGL(tb_route_offsets, dim3(A.world), dim3(1024), 0, E->stream, A);
        HIPCK(hipGetLastError());
        hipLaunchKernelGGL(tb_route_scatter, dim3(A.nblocks), dim3(ROUTE_THREADS), 0, E->stream, A, (u8*)send_events_dev,
                           (u32*)slot_dev);
        HIPCK(hipGetLastError());
    }
    std::vector<u64> words(ROUTE_WORDS);
    HIPCK(hipMemcpyAsync(words.data(), E->r_words, ROUTE_WORDS * 8, hipMemcpyDeviceToHost, E->stream));
    Globals g;
    HIPCK(hipMemcpyAsync(&g, E->g, sizeof(Globals), hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    unsigned __int128 S = 0;
    bool huge = words[RW_HUGE] != 0;
    for (int i = 0; i < SUM_SHARDS && !huge; i++) {
        const unsigned __int128 v = ((unsigned __int128)words[2 * i + 1] << 64) | words[2 * i];
        const unsigned __int128 r = S + v;
        if (r < S) huge = true;
        S = r;
    }
    if (huge) S = ~(unsigned __int128)0;
    plan->sum_lo = (u64)S;
    plan->sum_hi = (u64)(S >> 64);
    plan->bound_lo = g.bound_lo;
    plan->bound_hi = g.bound_hi;
    plan->dirty = (u32)words[RW_DIRTY];
    for (u32 h = 0; h < E->route_world; h++) plan->send_counts[h] = words[RW_COUNTS + h];
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_commit_routed_async(tbgpu_t* E, uint64_t n, const void* events_dev, uint64_t ts_max,
                                         uint32_t cert, uint8_t* codes_dev) {
    API_ENTER(E, true);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (cert != TBGPU_CERT_U128 && cert != TBGPU_CERT_U64) return fail(TBGPU_STATUS_INVALID, "routed commit needs a certificate");
    if (n == 0) return TBGPU_STATUS_OK;
    if (E->pending) {  // the pinned metadata mirror may still be in flight
        int st = engine_sync(E);
        if (st) return st;
    }
    // Pseudo-prepares of up to 8190 events: the events are independent (no chains), so the split
    // only sizes the resolve workgroups.
    const u64 per = BATCH_EVENTS_MAX - 1;
    const u64 nb = (n + per - 1) / per;
    if (nb > E->meta_cap) return fail(TBGPU_STATUS_INVALID, "routed call too large");
    if (E->log_next + n > E->xlog_cap) {
        return fail(TBGPU_STATUS_INVALID, "transfer log full (%llu + %llu events > capacity %llu)",
                    (unsigned long long)E->log_next, (unsigned long long)n, (unsigned long long)E->xlog_cap);
    }
    u64* h_off = E->h_meta;
    u64* h_ts = E->h_meta + nb + 1;
    h_off[0] = 0;
    for (u64 k = 0; k < nb; k++) {
        h_off[k + 1] = std::min<u64>(n, h_off[k] + per);
        h_ts[k] = ts_max;
    }
    HIPCK(hipMemcpyAsync(E->meta, E->h_meta, (2 * nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
    std::vector<u64> off(h_off, h_off + nb + 1);
    int st = enqueue_call(E, OP_CREATE_TRANSFERS, (u32)nb, off.data(), (const u8*)events_dev, E->results,
                          E->reply_bytes, true, codes_dev, cert);
    if (st) return st;
    E->last_batch_ts = std::max(E->last_batch_ts, ts_max);
    E->pending = true;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_commit_routed_owner_async(tbgpu_t* E, uint64_t n, const void* events_dev, uint64_t ts_max,
                                               uint32_t cert, uint8_t* codes_dev, uint32_t world, uint32_t self,
                                               void* legs_dev, uint64_t legs_cap, uint64_t* leg_counts_dev) {
    API_ENTER(E, true);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (cert != TBGPU_CERT_U128 && cert != TBGPU_CERT_U64) return fail(TBGPU_STATUS_INVALID, "routed commit needs a certificate");
    if (world == 0 || world > ROUTE_WORLD_MAX || self >= world) return fail(TBGPU_STATUS_INVALID, "owner world / rank");
    if (legs_cap < 2 * n) return fail(TBGPU_STATUS_INVALID, "owner leg regions need 2 legs per event");
    HIPCK(hipMemsetAsync(leg_counts_dev, 0, (u64)world * 8, E->stream));
    if (n == 0) return TBGPU_STATUS_OK;
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    const u64 per = BATCH_EVENTS_MAX - 1;
    const u64 nb = (n + per - 1) / per;
    if (nb > E->meta_cap) return fail(TBGPU_STATUS_INVALID, "routed call too large");
    if (E->log_next + n > E->xlog_cap) {
        return fail(TBGPU_STATUS_INVALID, "transfer log full (%llu + %llu events > capacity %llu)",
                    (unsigned long long)E->log_next, (unsigned long long)n, (unsigned long long)E->xlog_cap);
    }
    u64* h_off = E->h_meta;
    u64* h_ts = E->h_meta + nb + 1;
    h_off[0] = 0;
    for (u64 k = 0; k < nb; k++) {
        h_off[k + 1] = std::min<u64>(n, h_off[k] + per);
        h_ts[k] = ts_max;
    }
    HIPCK(hipMemcpyAsync(E->meta, E->h_meta, (2 * nb + 1) * 8, hipMemcpyHostToDevice, E->stream));
    std::vector<u64> off(h_off, h_off + nb + 1);
    OwnerLegArgs O{world, self, (u64*)legs_dev, legs_cap, leg_counts_dev, nullptr, OWNER_LEG_WORDS};
    int st = enqueue_call(E, OP_CREATE_TRANSFERS, (u32)nb, off.data(), (const u8*)events_dev, E->results,
                          E->reply_bytes, true, codes_dev, cert, nullptr, nullptr, &O);
    if (st) return st;
    E->last_batch_ts = std::max(E->last_batch_ts, ts_max);
    E->pending = true;
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_apply_owner_legs_async(tbgpu_t* E, const void* legs_dev, uint64_t n, uint32_t cert) {
    API_ENTER(E, true);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (cert != TBGPU_CERT_U128 && cert != TBGPU_CERT_U64) return fail(TBGPU_STATUS_INVALID, "owner legs need a certificate");
    if (n == 0) return TBGPU_STATUS_OK;
    HIPCK(hipMemsetAsync(E->d_status, 0, 4, E->stream));
    hipLaunchKernelGGL(tb_apply_owner_legs, dim3((u32)((n + 255) / 256)), dim3(256), 0, E->stream, E->T,
                       (const u64*)legs_dev, n, cert == TBGPU_CERT_U64 ? 1u : 0u, E->d_status);
    HIPCK(hipGetLastError());
    u32 status = 0;
    HIPCK(hipMemcpyAsync(&status, E->d_status, 4, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    if (status) return fail(TBGPU_STATUS_PANIC, "owner leg for an account this rank does not hold");
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_route_replies_async(tbgpu_t* E, uint32_t nb, const uint32_t* lens, const uint32_t* slot_dev,
                                         const uint8_t* codes_dev, void* results_dev, uint32_t* reply_bytes_dev) {
    API_ENTER(E, false);
    if (E->node) return fail(TBGPU_STATUS_INVALID, "tbgpu_shard.h primitives take a single-device engine");
    HIPCK(hipSetDevice(E->device));
    if (!E->r_meta) return fail(TBGPU_STATUS_INVALID, "tbgpu_route_init was not called");
    if (nb == 0) return TBGPU_STATUS_OK;
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    u64 n = 0;
    int st = route_meta(E, nb, nullptr, lens, &n);
    if (st) return st;
    hipLaunchKernelGGL(tb_route_replies, dim3(nb), dim3(1024), 0, E->stream, E->r_meta, slot_dev, codes_dev,
                       (u32*)results_dev, reply_bytes_dev);
    HIPCK(hipGetLastError());
    E->pending = true;
    return TBGPU_STATUS_OK;
}

// Host <-> device staging through the lookup buffers, in chunks of lookup_cap.
extern "C" int tbgpu_fetch_accounts(tbgpu_t* E, const uint64_t* ids, uint32_t n, void* out, uint8_t* found) {
    API_ENTER(E, false);
    if (E->node) return node_fetch(E->node, true, ids, n, (u8*)out, found);
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    for (u32 c = 0; c < n; c += E->lookup_cap) {
        const u32 m = std::min<u32>(E->lookup_cap, n - c);
        HIPCK(hipMemcpyAsync(E->lookup_ids, ids + 2 * (u64)c, (u64)m * 16, hipMemcpyHostToDevice, E->stream));
        HIPCK(hipMemsetAsync(E->lookup_out, 0, (u64)m * 128, E->stream));
        hipLaunchKernelGGL(tb_lookup<true>, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_ids, m,
                           E->lookup_out, E->lookup_found);
        HIPCK(hipGetLastError());
        HIPCK(hipMemcpyAsync((u8*)out + (u64)c * 128, E->lookup_out, (u64)m * 128, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipMemcpyAsync(found + c, E->lookup_found, m, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipStreamSynchronize(E->stream));
    }
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_fetch_transfers(tbgpu_t* E, const uint64_t* ids, uint32_t n, void* out, uint8_t* state) {
    API_ENTER(E, false);
    if (E->node) return node_fetch(E->node, false, ids, n, (u8*)out, state);
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    for (u32 c = 0; c < n; c += E->lookup_cap) {
        const u32 m = std::min<u32>(E->lookup_cap, n - c);
        HIPCK(hipMemcpyAsync(E->lookup_ids, ids + 2 * (u64)c, (u64)m * 16, hipMemcpyHostToDevice, E->stream));
        HIPCK(hipMemsetAsync(E->lookup_out, 0, (u64)m * 128, E->stream));
        hipLaunchKernelGGL(tb_fetch_transfers, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_ids, m,
                           E->lookup_out, E->lookup_found);
        HIPCK(hipGetLastError());
        HIPCK(hipMemcpyAsync((u8*)out + (u64)c * 128, E->lookup_out, (u64)m * 128, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipMemcpyAsync(state + c, E->lookup_found, m, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipStreamSynchronize(E->stream));
    }
    return TBGPU_STATUS_OK;
}

// A load (if_absent) brings objects from the forest: they are already written back, so the
// write-back snapshot takes their state too, and the "created since" timestamp covers them.
static int load_snapshot(tbgpu* E, const void* records, uint32_t n) {
    int st = ckpt_snapshot_ready(E);
    if (st) return st;
    for (u32 i = 0; i < n; i++) E->ckpt_ts = std::max(E->ckpt_ts, *(const u64*)((const u8*)records + (u64)i * 128 + 120));
    return TBGPU_STATUS_OK;
}

static int upsert_accounts(tbgpu* E, const void* records, uint32_t n, bool if_absent, bool keep_flow = false) {
    HIPCK(hipSetDevice(E->device));
    if (if_absent) {
        if (E->pending) {
            int st = engine_sync(E);
            if (st) return st;
        }
        int st = load_snapshot(E, records, n);
        if (st) return st;
    }
    // Balances set from elsewhere: the sequential replay stays exact.  A load of absent accounts
    // from a consistent forest snapshot keeps the flow path's invariants (pending balances cover
    // the outstanding pending transfers).
    // keep_flow: balances a sequential commit from a consistent state produced (the node's
    // sequencer write-back), so the invariants hold as well.
    if (!if_absent && !keep_flow) E->balances_set = true;
    if (!if_absent) ckpt_note_ids(E, (const u8*)records, n);
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    // Keep `bound` >= dp+dpost, cp+cpost of every account (saturating).
    Globals g;
    HIPCK(hipMemcpy(&g, E->g, sizeof(Globals), hipMemcpyDeviceToHost));
    typedef unsigned __int128 h128;
    const h128 MAX = ~(h128)0;
    h128 bound = ((h128)g.bound_hi << 64) | g.bound_lo;
    for (u32 i = 0; i < n; i++) {
        const u64* w = (const u64*)((const u8*)records + (u64)i * 128);
        const h128 dp = ((h128)w[3] << 64) | w[2], dpo = ((h128)w[5] << 64) | w[4];
        const h128 cp = ((h128)w[7] << 64) | w[6], cpo = ((h128)w[9] << 64) | w[8];
        const h128 d = dp + dpo < dp ? MAX : dp + dpo;
        const h128 c = cp + cpo < cp ? MAX : cp + cpo;
        bound = std::max(bound, std::max(d, c));
    }
    u32 status = 0;
    HIPCK(hipMemsetAsync(E->d_status, 0, 4, E->stream));
    for (u32 c = 0; c < n; c += E->lookup_cap) {
        const u32 m = std::min<u32>(E->lookup_cap, n - c);
        HIPCK(hipMemcpyAsync(E->lookup_out, (const u8*)records + (u64)c * 128, (u64)m * 128, hipMemcpyHostToDevice,
                             E->stream));
        hipLaunchKernelGGL(tb_upsert_accounts, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_out, m,
                           E->d_status, if_absent ? 1u : 0u, if_absent ? ckpt_view(E) : BalView{nullptr, nullptr});
        HIPCK(hipGetLastError());
        HIPCK(hipStreamSynchronize(E->stream));
    }
    const u64 bw[2] = {(u64)bound, (u64)(bound >> 64)};
    HIPCK(hipMemcpy(&E->g->bound_lo, bw, 16, hipMemcpyHostToDevice));
    HIPCK(hipMemcpy(&status, E->d_status, 4, hipMemcpyDeviceToHost));
    if (status) return fail(TBGPU_STATUS_PANIC, "account table full");
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_upsert_accounts(tbgpu_t* E, const void* records, uint32_t n) {
    API_ENTER(E, true);
    if (E->node) return node_api_accounts_in(E->node, records, n, false);
    return upsert_accounts(E, records, n, false);
}

extern "C" int tbgpu_load_accounts(tbgpu_t* E, const void* records, uint32_t n) {
    API_ENTER(E, true);
    if (E->node) return node_api_accounts_in(E->node, records, n, true);
    return upsert_accounts(E, records, n, true);
}

static int upsert_transfers(tbgpu* E, const void* records, const uint8_t* state, uint32_t n, bool if_absent) {
    HIPCK(hipSetDevice(E->device));
    if (if_absent) {
        if (E->pending) {
            int st = engine_sync(E);
            if (st) return st;
        }
        int st = load_snapshot(E, records, n);
        if (st) return st;
    }
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    HIPCK(hipMemsetAsync(E->d_status, 0, 8, E->stream));
    for (u32 c = 0; c < n; c += E->lookup_cap) {
        const u32 m = std::min<u32>(E->lookup_cap, n - c);
        HIPCK(hipMemcpyAsync(E->lookup_out, (const u8*)records + (u64)c * 128, (u64)m * 128, hipMemcpyHostToDevice,
                             E->stream));
        HIPCK(hipMemcpyAsync(E->lookup_found, state + c, m, hipMemcpyHostToDevice, E->stream));
        HIPCK(hipMemsetAsync(E->d_status + 1, 0, 4, E->stream));
        hipLaunchKernelGGL(tb_upsert_transfers, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->T, E->lookup_out,
                           E->lookup_found, m, E->log_next, E->d_status + 1, E->d_status, if_absent ? 1u : 0u,
                           nullptr);
        HIPCK(hipGetLastError());
        u32 added = 0;
        HIPCK(hipMemcpyAsync(&added, E->d_status + 1, 4, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipStreamSynchronize(E->stream));
        E->log_next += added;
    }
    u32 status = 0;
    HIPCK(hipMemcpy(&status, E->d_status, 4, hipMemcpyDeviceToHost));
    if (status) return fail(TBGPU_STATUS_PANIC, "transfer log or index full");
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_upsert_transfers(tbgpu_t* E, const void* records, const uint8_t* state, uint32_t n) {
    API_ENTER(E, true);
    if (E->node) return node_api_transfers_in(E->node, records, state, n, false);
    return upsert_transfers(E, records, state, n, false);
}

extern "C" int tbgpu_load_transfers(tbgpu_t* E, const void* records, const uint8_t* posted_state, uint32_t n) {
    API_ENTER(E, true);
    if (E->node) return node_api_transfers_in(E->node, records, posted_state, n, true);
    // posted_state is {0 none, 1 posted, 2 voided}; the upsert kernel takes 1 + that.
    std::vector<u8> st(n);
    for (u32 i = 0; i < n; i++) {
        if (posted_state[i] > POSTED_VOIDED) return fail(TBGPU_STATUS_INVALID, "posted state %u", posted_state[i]);
        st[i] = (u8)(posted_state[i] + 1);
    }
    return upsert_transfers(E, records, st.data(), n, true);
}

// The replica writes commit_timestamp after every commit (= the prepare header's timestamp,
// src/vsr/replica.zig:3664-3665) and on state sync; the engine's commit asserts use that value.
// Bounded residency (k_evict.h): drop the written-back transfers older than the newest `keep` log
// positions.  Only what the last write-back covered can go (the forest holds it); the rest slides to
// the front of the log and the index is rebuilt from it.  Synchronous.
static int engine_evict(tbgpu_t* E, uint64_t keep, uint64_t* evicted) {
    *evicted = 0;
    HIPCK(hipSetDevice(E->device));
    if (E->wb.inflight) return fail(TBGPU_STATUS_INVALID, "an asynchronous write-back is in flight");
    int st = engine_sync(E);
    if (st) return st;
    // Only right after a write-back: a commit since then may post or void a pending transfer before
    // the cut, and the next write-back reads that record (tb_delta_posted) and its posted state.
    if (E->ckpt_valid && E->ckpt_pos != E->log_next)
        return fail(TBGPU_STATUS_INVALID, "%llu log positions written since the last write-back",
                    (unsigned long long)(E->log_next - E->ckpt_pos));
    const u64 written = E->ckpt_valid ? E->ckpt_pos : 0;  // positions the forest already holds
    const u64 cut = std::min<u64>(written, E->log_next > keep ? E->log_next - keep : 0);
    if (cut == 0) return TBGPU_STATUS_OK;
    const u64 n = E->log_next, kept = n - cut;
    u8* live = E->T.xdup;  // scratch (xidx_cap >= 2 x log bytes), zeroed again below
    u64* d_evicted = E->wb.d_cnt;  // scratch word (no write-back in flight)
    HIPCK(hipMemsetAsync(d_evicted, 0, 8, E->stream));
    const u32 grid = (u32)std::min<u64>(4096, std::max<u64>(1, (n + 255) / 256));
    hipLaunchKernelGGL(tb_evict_scan, dim3(grid), dim3(256), 0, E->stream, E->T, cut, n, E->bloom, E->bloom_mask, live,
                       d_evicted);
    HIPCK(hipGetLastError());
    // Slide the kept records (and their posted states) to the front, in chunks that never overlap
    // their sources, then rebuild the index over them.
    for (u64 a = 0; a < kept; a += cut) {
        const u64 m = std::min<u64>(cut, kept - a);
        HIPCK(hipMemcpyAsync(E->T.xlog + a, E->T.xlog + cut + a, m * sizeof(Transfer), hipMemcpyDeviceToDevice, E->stream));
        HIPCK(hipMemcpyAsync(E->T.xposted + a, E->T.xposted + cut + a, m, hipMemcpyDeviceToDevice, E->stream));
    }
    HIPCK(hipMemsetAsync(E->T.xlog + kept, 0, cut * sizeof(Transfer), E->stream));
    HIPCK(hipMemsetAsync(E->T.xposted + kept, 0, cut, E->stream));
    HIPCK(hipMemsetAsync(E->T.xidx, 0, E->xidx_cap * sizeof(u64), E->stream));
    if (kept) {
        hipLaunchKernelGGL(tb_evict_reindex, dim3((u32)std::min<u64>(4096, (kept + 255) / 256)), dim3(256), 0, E->stream,
                           E->T, kept, (const u8*)live);
        HIPCK(hipGetLastError());
    }
    HIPCK(hipMemsetAsync(E->T.xdup, 0, E->xidx_cap, E->stream));
    u64 h_evicted = 0;
    HIPCK(hipMemcpyAsync(&h_evicted, d_evicted, 8, hipMemcpyDeviceToHost, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    E->log_next = kept;
    E->ckpt_pos -= cut;
    E->evicted_total += h_evicted;
    E->dedup_force = true;
    // Live transfers resident: the evicted ones left.
    if (h_evicted) {
        HIPCK(hipMemcpy(E->h_globals, E->g, sizeof(Globals), hipMemcpyDeviceToHost));
        E->h_globals->transfer_count -= std::min<u64>(E->h_globals->transfer_count, h_evicted);
        HIPCK(hipMemcpy(&E->g->transfer_count, &E->h_globals->transfer_count, 8, hipMemcpyHostToDevice));
    }
    *evicted = h_evicted;
    return TBGPU_STATUS_OK;
}


extern "C" int tbgpu_evict_transfers(tbgpu_t* E, uint64_t keep, uint64_t* evicted) {
    API_ENTER(E, true);
    *evicted = 0;
    if (E->node) return node_api_evict(E->node, keep, evicted);
    return engine_evict(E, keep, evicted);
}

// The replica's prefetch after an eviction: which of n ids (lo, hi pairs) the engine may have evicted
// — not resident, maybe in the filter.  The caller loads those its forest holds (tbgpu_load_transfers)
// before committing the prepare that names them.
static int engine_maybe_cold(tbgpu_t* E, const uint64_t* ids, uint32_t n, uint8_t* cold) {
    if (n == 0) return TBGPU_STATUS_OK;
    if (E->evicted_total == 0) {  // nothing ever left: nothing is cold
        memset(cold, 0, n);
        return TBGPU_STATUS_OK;
    }
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        const int st = engine_sync(E);
        if (st) return st;
    }
    for (u32 i0 = 0; i0 < n; i0 += E->lookup_cap) {
        const u32 m = std::min<u32>(n - i0, E->lookup_cap);
        HIPCK(hipMemcpyAsync(E->lookup_ids, ids + 2 * (u64)i0, (u64)m * 16, hipMemcpyHostToDevice, E->stream));
        hipLaunchKernelGGL(tb_cold_query, dim3((m + 255) / 256), dim3(256), 0, E->stream, E->T, (const u64*)E->bloom,
                           E->bloom_mask, E->lookup_ids, m, E->lookup_found);
        HIPCK(hipGetLastError());
        HIPCK(hipMemcpyAsync(cold + i0, E->lookup_found, m, hipMemcpyDeviceToHost, E->stream));
        HIPCK(hipStreamSynchronize(E->stream));
    }
    return TBGPU_STATUS_OK;
}

extern "C" int tbgpu_transfers_maybe_cold(tbgpu_t* E, const uint64_t* ids, uint32_t n, uint8_t* cold) {
    API_ENTER(E, false);
    if (E->node) return node_api_maybe_cold(E->node, ids, n, cold);
    return engine_maybe_cold(E, ids, n, cold);
}

extern "C" int tbgpu_set_commit_timestamp(tbgpu_t* E, uint64_t timestamp) {
    API_ENTER(E, true);
    if (E->node) return node_api_set_commit_timestamp(E->node, timestamp);
    HIPCK(hipSetDevice(E->device));
    if (E->pending) {
        int st = engine_sync(E);
        if (st) return st;
    }
    E->commit_ts = timestamp;
    E->last_batch_ts = timestamp;
    HIPCK(hipMemcpyAsync(&E->g->commit_timestamp, &E->commit_ts, 8, hipMemcpyHostToDevice, E->stream));
    HIPCK(hipStreamSynchronize(E->stream));
    return TBGPU_STATUS_OK;
}

#include "node.h"
