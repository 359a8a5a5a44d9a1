//! state_machine_gpu.zig — the reference-side binding a maintainer adds to run
//! StateMachine.commit (create_accounts, create_transfers, lookup_accounts, lookup_transfers) on the
//! MI355X engine (include/tbgpu.h), with the reference's LSM forest kept as the durable store.
//!
//! SOURCE ONLY: this image has no Zig toolchain (Zig 0.11, scripts/install_zig.sh needs network),
//! so this file is checked by review against every member the reference's consumers use:
//!   * the replica (src/vsr/replica.zig): init (:832), deinit, reset (:7763), open (:662, :7835),
//!     prepare (:5137), prefetch (:3347), commit (:3654), compact (:3088), checkpoint (:3093), the
//!     fields prepare_timestamp / commit_timestamp (:3621-3665, :5122-5131, :6854-6861) and forest
//!     (state sync, :7903-7942), the decls Operation, Options, Forest;
//!   * the cluster harness (src/testing/cluster.zig:49-55, :514, :534): Forest, forest, Options;
//!   * clients / simulator / CLI: constants, Event, Result, Workload, PostedGrooveValue,
//!     forest_options (src/tigerbeetle/cli.zig:278, src/lsm/forest_fuzz.zig:59).
//! It is the reference StateMachine's shape (src/state_machine.zig:28-1150) with execute() replaced
//! by the engine; the forest, its grooves and their persistence are the reference's own.
//!
//! Data flow:
//!   commit      -> tbgpu_commit (the HBM tables are the state of record while the process lives);
//!   compact     -> at the last op of every bar, the objects the engine changed during the bar go
//!                  into the grooves (insert / upsert, src/lsm/groove.zig:902-963) before
//!                  forest.compact, so each bar's table_mutable receives what the reference's own
//!                  commits would have put there (bounded by the same value_count_max,
//!                  src/state_machine.zig:100-178);
//!   checkpoint  -> forest.checkpoint (the bar's write-back already happened in compact);
//!   open        -> forest.open; if the forest already holds objects (a restart), prefetch runs
//!                  the reference's groove prefetch and loads what a prepare reads and the engine
//!                  lacks (tbgpu_load_*), before the replica commits it.
//! Build: add include/ to the C include path and link tigerbeetle_amd/libtbgpu.so (INTEGRATION.md),
//! then instantiate ReplicaType with this StateMachineType (src/tigerbeetle/main.zig:28-32).

const std = @import("std");
const assert = std.debug.assert;
const mem = std.mem;
const log = std.log.scoped(.state_machine_gpu);

const tbgpu = @cImport({
    @cInclude("tbgpu.h");
});

const global_constants = @import("constants.zig");
const tb = @import("tigerbeetle.zig");
const Account = tb.Account;
const Transfer = tb.Transfer;
const GridType = @import("vsr/grid.zig").GridType;
const Header = @import("vsr.zig").Header;
const messages_max_replica = @import("message_pool.zig").messages_max_replica;
const ReferenceStateMachineType = @import("state_machine.zig").StateMachineType;

pub fn StateMachineType(
    comptime Storage: type,
    comptime config: global_constants.StateMachineConfig,
) type {
    // The reference type supplies the types (Forest and its grooves, Operation, Workload, ...);
    // no instance of it exists.
    const Base = ReferenceStateMachineType(Storage, config);

    return struct {
        const StateMachine = @This();
        const Grid = GridType(Storage);

        pub const Operation = Base.Operation;
        pub const Forest = Base.Forest;
        pub const Workload = Base.Workload;
        pub const constants = Base.constants;
        pub const Event = Base.Event;
        pub const Result = Base.Result;
        pub const PostedGrooveValue = Base.PostedGrooveValue;

        const AccountsGroove = std.meta.FieldType(Forest.Grooves, .accounts);
        const TransfersGroove = std.meta.FieldType(Forest.Grooves, .transfers);
        const PostedGroove = std.meta.FieldType(Forest.Grooves, .posted);

        /// The reference's options (src/state_machine.zig:216-221) plus the engine's HBM sizing.
        /// The cache_entries_* knobs size the groove caches, not the number of objects, so the
        /// engine has its own: every account and transfer the cluster will ever hold must fit the
        /// device (DESIGN.md §2b: at most 2^31 of each; init fails if HBM is short).
        pub const Options = struct {
            lsm_forest_node_count: u32,
            cache_entries_accounts: u32,
            cache_entries_transfers: u32,
            cache_entries_posted: u32,
            engine_accounts_max: u64 = 1 << 26,
            engine_transfers_max: u64 = 1 << 30,
            engine_device: i32 = 0,
            /// Two or more devices: one node engine with a shard per device (tbgpu_config.devices).
            engine_devices: []const i32 = &.{},
            /// prefetch starts the prepare body's DMA (tbgpu_prefetch) — worth it when the replica
            /// has work between prefetch and commit; otherwise commit's first kernel reads the body
            /// straight from its registered message (DESIGN.md §5b).
            engine_stage_bodies: bool = false,
            /// The caller guarantees every prepare body it passes lives in a MessagePool buffer, right
            /// after its sector-aligned header (src/message_pool.zig:98-120): the engine may then pin
            /// those buffers (tbgpu_register_host) for direct reads.  Off: bodies are copied from
            /// pageable memory, and the engine pins nothing it does not own (test / fuzzer / replay
            /// buffers from any allocator stay safe).
            engine_register_messages: bool = false,
            /// compact() writes each bar back ONE BAR BEHIND (tbgpu_checkpoint_delta_async: bar k's
            /// objects cross PCIe while bar k+1 commits and reach the grooves at bar k+1's end),
            /// except the bar ending at a checkpoint op, which drains synchronously
            /// (write_back_synchronous): its objects must be in its own table_mutable, which the
            /// trigger bar's compaction flushes before the checkpoint (src/lsm/tree.zig:1078-1099,
            /// src/vsr.zig:2009-2037); a later bar in flight at the checkpoint is replayed from the
            /// WAL.  The bound this needs: the checkpoint bar's table_mutable receives two bars of
            /// objects (the one in flight and its own), so every groove tree must be sized for
            /// 2 x value_count_max (src/state_machine.zig:100-178 — a constant doubled in the fork
            /// that links this wrapper); every other bar's table receives one.  Off: each bar is
            /// written back synchronously at its last op (one bar per table, ~4 ms per bar).
            engine_write_back_behind: bool = false,

            fn base(options: Options) Base.Options {
                return .{
                    .lsm_forest_node_count = options.lsm_forest_node_count,
                    .cache_entries_accounts = options.cache_entries_accounts,
                    .cache_entries_transfers = options.cache_entries_transfers,
                    .cache_entries_posted = options.cache_entries_posted,
                };
            }
        };

        pub fn forest_options(options: Options) Forest.GroovesOptions {
            return Base.forest_options(options.base());
        }

        // One bar of engine changes, the most the grooves accept per bar
        // (value_count_max, src/state_machine.zig:100-178).
        const bar_transfers_max = config.lsm_batch_multiple * constants.batch_max.create_transfers;
        const bar_accounts_max = config.lsm_batch_multiple *
            @max(constants.batch_max.create_accounts, 2 * constants.batch_max.create_transfers);
        // Objects one prepare can read (the groove prefetch_entries_max, :1091-1146).
        const prepare_accounts_max = @max(constants.batch_max.create_accounts, 2 * constants.batch_max.create_transfers);
        const prepare_transfers_max = 2 * constants.batch_max.create_transfers;

        /// One bar's write-back buffers (registered with the engine; the DMA target of a delta).
        const WriteBack = struct {
            accounts: []Account,
            accounts_before: [][4]u128,
            transfers: []Transfer,
            posted: [][2]u64,

            fn alloc(allocator: mem.Allocator) !WriteBack {
                const accounts = try allocator.alloc(Account, bar_accounts_max);
                errdefer allocator.free(accounts);
                const accounts_before = try allocator.alloc([4]u128, bar_accounts_max);
                errdefer allocator.free(accounts_before);
                const transfers = try allocator.alloc(Transfer, bar_transfers_max);
                errdefer allocator.free(transfers);
                const posted = try allocator.alloc([2]u64, bar_transfers_max);
                return .{ .accounts = accounts, .accounts_before = accounts_before, .transfers = transfers, .posted = posted };
            }

            fn free(set: *const WriteBack, allocator: mem.Allocator) void {
                allocator.free(set.posted);
                allocator.free(set.transfers);
                allocator.free(set.accounts_before);
                allocator.free(set.accounts);
            }

            fn register(set: *const WriteBack, engine: *tbgpu.tbgpu_t) bool {
                inline for (.{ set.accounts, set.accounts_before, set.transfers, set.posted }) |buffer| {
                    const bytes = mem.sliceAsBytes(buffer);
                    if (tbgpu.tbgpu_register_host(engine, @constCast(bytes.ptr), bytes.len) != tbgpu.TBGPU_STATUS_OK) {
                        return false;
                    }
                }
                return true;
            }

            fn unregister(set: *const WriteBack, engine: *tbgpu.tbgpu_t) void {
                inline for (.{ set.accounts, set.accounts_before, set.transfers, set.posted }) |buffer| {
                    check(tbgpu.tbgpu_unregister_host(engine, mem.sliceAsBytes(buffer).ptr));
                }
            }
        };

        const PrefetchContext = union(enum) {
            accounts: AccountsGroove.PrefetchContext,
            transfers: TransfersGroove.PrefetchContext,
            posted: PostedGroove.PrefetchContext,
        };

        prepare_timestamp: u64,
        commit_timestamp: u64,
        forest: Forest,

        engine: *tbgpu.tbgpu_t,
        /// commit_timestamp as the engine last saw it: the replica writes the field itself.
        engine_commit_timestamp: u64 = 0,
        /// The engine holds every object the forest holds (a freshly formatted cluster).  False
        /// after open() finds objects in the forest, for the rest of the process.
        engine_complete: bool = true,
        /// Transfers the engine evicted (tbgpu_evict_transfers: written back, dropped when the
        /// transfer log fills).  Non-zero: a create_transfers / lookup_transfers prefetch asks the
        /// engine which of its ids may be cold and takes the forest path when any is.
        engine_evicted: u64 = 0,

        prefetch_input: ?[]align(16) const u8 = null,
        prefetch_operation: Operation = undefined,
        /// The prefetch in flight loads only the ids transfers_cold flagged (cold_ids[0..n]); the
        /// engine resolves the rest from HBM and the body is staged as on the fast path.
        prefetch_cold: u32 = 0,
        prefetch_callback: ?*const fn (*StateMachine) void = null,
        prefetch_context: PrefetchContext = undefined,

        engine_stage_bodies: bool,
        engine_register_messages: bool,
        /// Message buffers registered with the engine, keyed by address (at most the pool's
        /// messages_max_replica, all allocated once by MessagePool.init_capacity).
        registered_messages: std.AutoHashMapUnmanaged(usize, void),

        open_callback: ?*const fn (*StateMachine) void = null,
        compact_callback: ?*const fn (*StateMachine) void = null,
        checkpoint_callback: ?*const fn (*StateMachine) void = null,

        /// Write-back sets in use: 1 (synchronous), 2 (engine_write_back_behind: one in flight).
        writeback_sets: u2,
        /// The set whose delta is in flight (engine_write_back_behind), and the next free one.
        writeback_inflight: ?u1 = null,
        writeback_next: u1 = 0,

        // Static allocation (allocated in init, never resized).
        writeback: [2]WriteBack,
        load_accounts: []Account,
        load_transfers: []Transfer,
        load_posted: []u8,
        cold_ids: [][2]u64,
        cold_flags: []u8,

        pub fn init(allocator: mem.Allocator, grid: *Grid, options: Options) !StateMachine {
            var forest = try Forest.init(allocator, grid, options.lsm_forest_node_count, forest_options(options));
            errdefer forest.deinit(allocator);

            var engine_config = mem.zeroes(tbgpu.tbgpu_config);
            engine_config.accounts_max = options.engine_accounts_max;
            engine_config.transfers_max = options.engine_transfers_max;
            engine_config.pass_events_max = constants.batch_max.create_transfers;
            engine_config.pass_batches_max = 1;
            engine_config.device = options.engine_device;
            if (options.engine_devices.len >= 2) {
                assert(options.engine_devices.len <= tbgpu.TBGPU_DEVICES_MAX);
                engine_config.device_count = @intCast(options.engine_devices.len);
                for (options.engine_devices, 0..) |d, i| engine_config.devices[i] = d;
            }
            // Eviction (evict_if_full) runs at a bar boundary once the log is three-quarters full
            // and keeps the newest quarter: the rest must hold a bar of commits plus the transfers
            // its prefetches load back (an id and a pending id per event), or a commit could find
            // the log full in the middle of a bar.
            if (options.engine_transfers_max / 4 < 3 * bar_transfers_max) return error.EngineInit;
            var engine: ?*tbgpu.tbgpu_t = null;
            if (tbgpu.tbgpu_init(&engine_config, &engine) != tbgpu.TBGPU_STATUS_OK) return error.EngineInit;
            errdefer tbgpu.tbgpu_deinit(engine);

            // A node engine's asynchronous write-back merges its shards at the call (tbgpu.h); the
            // contract, and so this wrapper, is the same as a single device's.
            const sets: u2 = if (options.engine_write_back_behind) 2 else 1;
            var writeback: [2]WriteBack = undefined;
            writeback[0] = try WriteBack.alloc(allocator);
            errdefer writeback[0].free(allocator);
            writeback[1] = if (sets == 2) try WriteBack.alloc(allocator) else writeback[0];
            errdefer if (sets == 2) writeback[1].free(allocator);
            const load_accounts = try allocator.alloc(Account, prepare_accounts_max);
            errdefer allocator.free(load_accounts);
            const load_transfers = try allocator.alloc(Transfer, prepare_transfers_max);
            errdefer allocator.free(load_transfers);
            const load_posted = try allocator.alloc(u8, prepare_transfers_max);
            errdefer allocator.free(load_posted);
            const cold_ids = try allocator.alloc([2]u64, prepare_transfers_max);
            errdefer allocator.free(cold_ids);
            const cold_flags = try allocator.alloc(u8, prepare_transfers_max);
            errdefer allocator.free(cold_flags);
            var registered_messages: std.AutoHashMapUnmanaged(usize, void) = .{};
            try registered_messages.ensureTotalCapacity(allocator, messages_max_replica);
            errdefer registered_messages.deinit(allocator);

            // The write-back buffers receive each bar's delta by DMA (registered once).
            for (writeback[0..sets]) |*set| {
                if (!set.register(engine.?)) return error.EngineInit;
            }

            return StateMachine{
                .prepare_timestamp = 0,
                .commit_timestamp = 0,
                .forest = forest,
                .engine = engine.?,
                .writeback_sets = sets,
                .writeback = writeback,
                .load_accounts = load_accounts,
                .load_transfers = load_transfers,
                .load_posted = load_posted,
                .cold_ids = cold_ids,
                .cold_flags = cold_flags,
                .engine_stage_bodies = options.engine_stage_bodies,
                .engine_register_messages = options.engine_register_messages,
                .registered_messages = registered_messages,
            };
        }

        pub fn deinit(self: *StateMachine, allocator: mem.Allocator) void {
            var it = self.registered_messages.keyIterator();
            while (it.next()) |address| check(tbgpu.tbgpu_unregister_host(self.engine, @ptrFromInt(address.*)));
            self.registered_messages.deinit(allocator);
            if (self.writeback_inflight != null) {
                var counts: tbgpu.tbgpu_delta_counts = undefined;
                check(tbgpu.tbgpu_checkpoint_delta_wait(self.engine, &counts)); // its buffers go away below
                self.writeback_inflight = null;
            }
            for (self.writeback[0..self.writeback_sets]) |*set| set.unregister(self.engine);
            allocator.free(self.cold_flags);
            allocator.free(self.cold_ids);
            allocator.free(self.load_posted);
            allocator.free(self.load_transfers);
            allocator.free(self.load_accounts);
            for (self.writeback[0..self.writeback_sets]) |*set| set.free(allocator);
            tbgpu.tbgpu_deinit(self.engine);
            self.forest.deinit(allocator);
        }

        pub fn reset(self: *StateMachine) void {
            self.forest.reset();
            check(tbgpu.tbgpu_reset(self.engine));
            self.prepare_timestamp = 0;
            self.commit_timestamp = 0;
            self.engine_commit_timestamp = 0;
            self.engine_complete = true;
            self.engine_evicted = 0;
            self.prefetch_input = null;
            self.prefetch_callback = null;
            self.open_callback = null;
            self.compact_callback = null;
            self.checkpoint_callback = null;
        }

        fn check(status: c_int) void {
            if (status != tbgpu.TBGPU_STATUS_OK) @panic(std.mem.span(tbgpu.tbgpu_last_error()));
        }

        pub fn open(self: *StateMachine, callback: *const fn (*StateMachine) void) void {
            assert(self.open_callback == null);
            self.open_callback = callback;
            self.forest.open(forest_open_callback);
        }

        fn forest_open_callback(forest: *Forest) void {
            const self = @fieldParentPtr(StateMachine, "forest", forest);
            const callback = self.open_callback.?;
            self.open_callback = null;
            // A forest with objects (a restart from a checkpoint): the engine starts empty and
            // loads objects on demand in prefetch.
            if (self.forest.grooves.accounts.objects.manifest.key_range() != null or
                self.forest.grooves.transfers.objects.manifest.key_range() != null)
            {
                self.engine_complete = false;
            }
            callback(self);
        }

        /// src/state_machine.zig:336-343.
        pub fn prepare(self: *StateMachine, operation: Operation, input: []align(16) u8) void {
            self.prepare_timestamp += switch (operation) {
                .create_accounts => mem.bytesAsSlice(Account, input).len,
                .create_transfers => mem.bytesAsSlice(Transfer, input).len,
                .lookup_accounts => 0,
                .lookup_transfers => 0,
            };
        }

        /// With every object resident in HBM, prefetch completes synchronously (a callback inside
        /// the call is allowed, src/lsm/groove.zig:723-742).  After a restart it runs the
        /// reference's groove prefetch (src/state_machine.zig:345-506) and then loads into the
        /// engine what the prepare reads.
        pub fn prefetch(
            self: *StateMachine,
            callback: *const fn (*StateMachine) void,
            op: u64,
            operation: Operation,
            input: []align(16) const u8,
        ) void {
            _ = op;
            assert(self.prefetch_input == null);
            assert(self.prefetch_callback == null);
            if (self.engine_complete) {
                const cold = self.transfers_cold(operation, input);
                if (cold == 0) {
                    self.stage_body(operation, input);
                    return callback(self);
                }
                // Only the flagged ids go through the groove (a Bloom false positive costs one
                // groove lookup, as the reference's own prefetch does for every id); the accounts
                // are resident (never evicted).
                self.prefetch_input = input;
                self.prefetch_operation = operation;
                self.prefetch_callback = callback;
                self.prefetch_cold = cold;
                self.forest.grooves.transfers.prefetch_setup(null);
                self.forest.grooves.posted.prefetch_setup(null);
                for (self.cold_ids[0..cold]) |pair| {
                    self.forest.grooves.transfers.prefetch_enqueue(@as(u128, pair[1]) << 64 | pair[0]);
                }
                self.prefetch_context = .{ .transfers = undefined };
                self.forest.grooves.transfers.prefetch(prefetch_transfers_done, &self.prefetch_context.transfers);
                return;
            }

            self.prefetch_input = input;
            self.prefetch_operation = operation;
            self.prefetch_callback = callback;
            self.forest.grooves.accounts.prefetch_setup(null);
            self.forest.grooves.transfers.prefetch_setup(null);
            self.forest.grooves.posted.prefetch_setup(null);
            switch (operation) {
                .create_accounts => {
                    for (mem.bytesAsSlice(Account, input)) |*a| self.forest.grooves.accounts.prefetch_enqueue(a.id);
                    self.prefetch_context = .{ .accounts = undefined };
                    self.forest.grooves.accounts.prefetch(prefetch_accounts_done, &self.prefetch_context.accounts);
                },
                .create_transfers => {
                    for (mem.bytesAsSlice(Transfer, input)) |*t| {
                        self.forest.grooves.transfers.prefetch_enqueue(t.id);
                        if (t.flags.post_pending_transfer or t.flags.void_pending_transfer) {
                            self.forest.grooves.transfers.prefetch_enqueue(t.pending_id);
                        }
                    }
                    self.prefetch_context = .{ .transfers = undefined };
                    self.forest.grooves.transfers.prefetch(prefetch_transfers_done, &self.prefetch_context.transfers);
                },
                // Lookups read the engine, which holds every object written since the restart;
                // older ones are loaded the same way.
                .lookup_accounts => {
                    for (mem.bytesAsSlice(u128, input)) |id| self.forest.grooves.accounts.prefetch_enqueue(id);
                    self.prefetch_context = .{ .accounts = undefined };
                    self.forest.grooves.accounts.prefetch(prefetch_accounts_done, &self.prefetch_context.accounts);
                },
                .lookup_transfers => {
                    for (mem.bytesAsSlice(u128, input)) |id| self.forest.grooves.transfers.prefetch_enqueue(id);
                    self.prefetch_context = .{ .transfers = undefined };
                    self.forest.grooves.transfers.prefetch(prefetch_transfers_done, &self.prefetch_context.transfers);
                },
            }
        }

        fn stage_body(self: *StateMachine, operation: Operation, input: []align(16) const u8) void {
            if (self.engine_stage_bodies and (operation == .create_accounts or operation == .create_transfers)) {
                self.register_message(input);
                check(tbgpu.tbgpu_prefetch(self.engine, @intFromEnum(operation), input.ptr, @intCast(input.len)));
            }
        }

        /// After an eviction: which transfers the prepare names may the engine have dropped (its ids,
        /// a post / void's pending id; lookup_transfers' ids)?  Compacts them into cold_ids and
        /// returns how many: only those go through the groove prefetch and are loaded
        /// (tbgpu_load_transfers) when the forest holds them.  A false positive (Bloom filter) only
        /// costs that id's groove lookup; a saturated filter degrades to the reference's own
        /// prefetch of every id, never to a wrong answer.
        fn transfers_cold(self: *StateMachine, operation: Operation, input: []align(16) const u8) u32 {
            if (self.engine_evicted == 0) return 0;
            var n: u32 = 0;
            switch (operation) {
                .create_transfers => for (mem.bytesAsSlice(Transfer, input)) |*t| {
                    self.cold_ids[n] = .{ @truncate(t.id), @truncate(t.id >> 64) };
                    n += 1;
                    if (t.flags.post_pending_transfer or t.flags.void_pending_transfer) {
                        self.cold_ids[n] = .{ @truncate(t.pending_id), @truncate(t.pending_id >> 64) };
                        n += 1;
                    }
                },
                .lookup_transfers => for (mem.bytesAsSlice(u128, input)) |id| {
                    self.cold_ids[n] = .{ @truncate(id), @truncate(id >> 64) };
                    n += 1;
                },
                else => return 0,
            }
            if (n == 0) return 0;
            check(tbgpu.tbgpu_transfers_maybe_cold(self.engine, @ptrCast(self.cold_ids.ptr), n, self.cold_flags.ptr));
            var cold: u32 = 0;
            for (self.cold_ids[0..n], self.cold_flags[0..n]) |pair, c| {
                if (c == 0) continue;
                self.cold_ids[cold] = pair;
                cold += 1;
            }
            return cold;
        }

        fn parent_of(comptime field: std.meta.FieldEnum(PrefetchContext), completion: anytype) *StateMachine {
            const context = @fieldParentPtr(PrefetchContext, @tagName(field), completion);
            return @fieldParentPtr(StateMachine, "prefetch_context", context);
        }

        fn prefetch_transfers_done(completion: *TransfersGroove.PrefetchContext) void {
            const self = parent_of(.transfers, completion);
            if (self.prefetch_cold > 0) {
                // The loaded transfers' posted entries (push_transfer reads them).
                for (self.cold_ids[0..self.prefetch_cold]) |pair| {
                    if (self.forest.grooves.transfers.get(@as(u128, pair[1]) << 64 | pair[0])) |t| {
                        self.forest.grooves.posted.prefetch_enqueue(t.timestamp);
                    }
                }
                self.prefetch_context = .{ .posted = undefined };
                self.forest.grooves.posted.prefetch(prefetch_posted_done, &self.prefetch_context.posted);
                return;
            }
            if (self.prefetch_operation == .lookup_transfers) return self.prefetch_finish();
            // src/state_machine.zig:434-458: the pending transfer's posted entry and accounts.
            for (mem.bytesAsSlice(Transfer, self.prefetch_input.?)) |*t| {
                if (t.flags.post_pending_transfer or t.flags.void_pending_transfer) {
                    if (self.forest.grooves.transfers.get(t.pending_id)) |p| {
                        self.forest.grooves.posted.prefetch_enqueue(p.timestamp);
                        self.forest.grooves.accounts.prefetch_enqueue(p.debit_account_id);
                        self.forest.grooves.accounts.prefetch_enqueue(p.credit_account_id);
                    }
                } else {
                    self.forest.grooves.accounts.prefetch_enqueue(t.debit_account_id);
                    self.forest.grooves.accounts.prefetch_enqueue(t.credit_account_id);
                }
            }
            self.prefetch_context = .{ .accounts = undefined };
            self.forest.grooves.accounts.prefetch(prefetch_accounts_done, &self.prefetch_context.accounts);
        }

        fn prefetch_accounts_done(completion: *AccountsGroove.PrefetchContext) void {
            const self = parent_of(.accounts, completion);
            if (self.prefetch_operation != .create_transfers) return self.prefetch_finish();
            self.prefetch_context = .{ .posted = undefined };
            self.forest.grooves.posted.prefetch(prefetch_posted_done, &self.prefetch_context.posted);
        }

        fn prefetch_posted_done(completion: *PostedGroove.PrefetchContext) void {
            parent_of(.posted, completion).prefetch_finish();
        }

        /// The prefetched objects are in the groove caches: hand the engine the ones it lacks
        /// (tbgpu_load_* keeps every object the engine already holds — those are newer).
        fn prefetch_finish(self: *StateMachine) void {
            const input = self.prefetch_input.?;
            var na: u32 = 0;
            var nt: u32 = 0;
            const grooves = &self.forest.grooves;
            if (self.prefetch_cold > 0) {
                for (self.cold_ids[0..self.prefetch_cold]) |pair| {
                    if (grooves.transfers.get(@as(u128, pair[1]) << 64 | pair[0])) |t| self.push_transfer(&nt, t);
                }
                if (nt > 0) {
                    check(tbgpu.tbgpu_load_transfers(self.engine, self.load_transfers.ptr, self.load_posted.ptr, nt));
                }
                self.prefetch_cold = 0;
                self.stage_body(self.prefetch_operation, input); // after the loads: the next commit's
                const callback_cold = self.prefetch_callback.?;
                self.prefetch_input = null;
                self.prefetch_callback = null;
                self.prefetch_context = undefined;
                return callback_cold(self);
            }
            switch (self.prefetch_operation) {
                .create_accounts => for (mem.bytesAsSlice(Account, input)) |*a| {
                    if (grooves.accounts.get(a.id)) |found| self.push_account(&na, found);
                },
                .lookup_accounts => for (mem.bytesAsSlice(u128, input)) |id| {
                    if (grooves.accounts.get(id)) |found| self.push_account(&na, found);
                },
                .lookup_transfers => for (mem.bytesAsSlice(u128, input)) |id| {
                    if (grooves.transfers.get(id)) |found| self.push_transfer(&nt, found);
                },
                .create_transfers => for (mem.bytesAsSlice(Transfer, input)) |*t| {
                    if (grooves.transfers.get(t.id)) |found| self.push_transfer(&nt, found);
                    var dr = t.debit_account_id;
                    var cr = t.credit_account_id;
                    if (t.flags.post_pending_transfer or t.flags.void_pending_transfer) {
                        if (grooves.transfers.get(t.pending_id)) |p| {
                            self.push_transfer(&nt, p);
                            dr = p.debit_account_id;
                            cr = p.credit_account_id;
                        }
                    }
                    if (grooves.accounts.get(dr)) |a| self.push_account(&na, a);
                    if (grooves.accounts.get(cr)) |a| self.push_account(&na, a);
                },
            }
            if (na > 0) check(tbgpu.tbgpu_load_accounts(self.engine, self.load_accounts.ptr, na));
            if (nt > 0) {
                check(tbgpu.tbgpu_load_transfers(self.engine, self.load_transfers.ptr, self.load_posted.ptr, nt));
            }
            const callback = self.prefetch_callback.?;
            self.prefetch_input = null;
            self.prefetch_callback = null;
            self.prefetch_context = undefined;
            callback(self);
        }

        fn push_account(self: *StateMachine, n: *u32, a: *const Account) void {
            // Duplicates are harmless (insert-if-absent); the buffer holds a prepare's worth.
            if (n.* == self.load_accounts.len) return;
            self.load_accounts[n.*] = a.*;
            n.* += 1;
        }

        fn push_transfer(self: *StateMachine, n: *u32, t: *const Transfer) void {
            if (n.* == self.load_transfers.len) return;
            self.load_transfers[n.*] = t.*;
            // Posted groove: {0 none, 1 posted, 2 voided} for tbgpu_load_transfers.
            self.load_posted[n.*] = if (self.forest.grooves.posted.get(t.timestamp)) |posted|
                @as(u8, switch (posted.fulfillment) {
                    .posted => 1,
                    .voided => 2,
                })
            else
                0;
            n.* += 1;
        }

        pub fn commit(
            self: *StateMachine,
            client: u128,
            op: u64,
            timestamp: u64,
            operation: Operation,
            input: []align(16) const u8,
            output: *align(16) [constants.message_body_size_max]u8,
        ) usize {
            _ = client;
            assert(op != 0);
            assert(timestamp > self.commit_timestamp or global_constants.aof_recovery);
            // The replica sets commit_timestamp to the header timestamp after every commit
            // (replica.zig:3664-3665) and from the checkpoint on open / sync: the engine follows.
            if (self.commit_timestamp != self.engine_commit_timestamp) {
                check(tbgpu.tbgpu_set_commit_timestamp(self.engine, self.commit_timestamp));
                self.engine_commit_timestamp = self.commit_timestamp;
            }
            self.register_message(input);
            var out_len: u32 = 0;
            check(tbgpu.tbgpu_commit(
                self.engine,
                @intFromEnum(operation),
                timestamp,
                input.ptr,
                @intCast(input.len),
                output,
                @intCast(output.len),
                &out_len,
            ));
            self.commit_timestamp = tbgpu.tbgpu_commit_timestamp(self.engine);
            self.engine_commit_timestamp = self.commit_timestamp;
            return out_len;
        }

        /// With engine_register_messages (the caller's promise that bodies come from the replica's
        /// MessagePool: each buffer allocated once, sector-aligned, message_size_max bytes, the body
        /// right after its header, src/message_pool.zig:98-120), the first commit from a buffer
        /// registers it with the engine, so every later body from it reaches the GPU by direct read.
        /// A body elsewhere, or a registration the runtime refuses, is simply left pageable: the
        /// commit copies it (the reference never panics on commit over where a body lives).
        fn register_message(self: *StateMachine, input: []align(16) const u8) void {
            if (!self.engine_register_messages) return;
            const address = @intFromPtr(input.ptr) -| @sizeOf(Header);
            if (address % global_constants.sector_size != 0) return;
            if (self.registered_messages.contains(address)) return;
            if (self.registered_messages.count() == messages_max_replica) return;
            if (tbgpu.tbgpu_register_host(self.engine, @ptrFromInt(address), global_constants.message_size_max) !=
                tbgpu.TBGPU_STATUS_OK)
            {
                log.warn("message buffer 0x{x} not registered ({s}); its bodies are copied", .{
                    address,
                    std.mem.span(tbgpu.tbgpu_last_error()),
                });
                return;
            }
            self.registered_messages.putAssumeCapacity(address, {});
        }

        pub fn compact(self: *StateMachine, callback: *const fn (*StateMachine) void, op: u64) void {
            assert(self.compact_callback == null);
            assert(self.checkpoint_callback == null);
            if ((op + 1) % config.lsm_batch_multiple == 0) {
                if (self.writeback_sets == 2 and !write_back_synchronous(op) and !self.log_needs_eviction()) {
                    self.write_back_behind();
                } else {
                    self.write_back_deliver(); // the bar in flight first: the grooves take bars in order
                    self.write_back();
                    // Only here may transfers leave: every commit is written back and no delta is
                    // in flight (tbgpu_evict_transfers refuses otherwise). One bar behind, a post /
                    // void of the bar in flight could name a pending transfer an eviction dropped.
                    self.evict_if_full();
                }
            }
            self.compact_callback = callback;
            self.forest.compact(compact_finish, op);
        }

        fn compact_finish(forest: *Forest) void {
            const self = @fieldParentPtr(StateMachine, "forest", forest);
            const callback = self.compact_callback.?;
            self.compact_callback = null;
            callback(self);
        }

        /// The bar's changes into the grooves, as the reference's commits would have put them:
        /// created objects by insert, re-balanced accounts by upsert against their previous version
        /// (which the groove must hold to diff the balance index trees: the engine returns the
        /// previous balances; the cache gets the old object first if it is not there).
        fn write_back(self: *StateMachine) void {
            assert(self.writeback_inflight == null);
            const set = &self.writeback[self.writeback_next];
            var counts: tbgpu.tbgpu_delta_counts = undefined;
            const status = tbgpu.tbgpu_checkpoint_delta(
                self.engine,
                set.accounts.ptr,
                set.accounts_before.ptr,
                set.accounts.len,
                set.transfers.ptr,
                set.transfers.len,
                @ptrCast(set.posted.ptr),
                set.posted.len,
                &counts,
            );
            // The buffers hold one bar's worth, the most a bar can change: STATUS_INVALID with
            // larger counts would mean the engine changed more objects than a bar's commits can
            // (an invariant failure, like the reference's TableMemory.put assert), so it panics.
            check(status);
            self.write_back_apply(set, &counts);
        }

        /// Checkpoint ops (vsr.Checkpoint.checkpoint_after: the first at journal_slot_count -
        /// lsm_batch_multiple - 1, then every journal_slot_count - lsm_batch_multiple ops): the bar
        /// ending there reaches the grooves before compact returns, with the bar in flight first.
        fn write_back_synchronous(op: u64) bool {
            const first = global_constants.journal_slot_count - global_constants.lsm_batch_multiple - 1;
            const every = global_constants.journal_slot_count - global_constants.lsm_batch_multiple;
            return op >= first and (op - first) % every == 0;
        }

        /// engine_write_back_behind: the previous bar's objects (landed while this bar committed)
        /// into the grooves, then this bar's capture started into the other set.
        fn write_back_behind(self: *StateMachine) void {
            self.write_back_deliver();
            const set = &self.writeback[self.writeback_next];
            check(tbgpu.tbgpu_checkpoint_delta_async(
                self.engine,
                set.accounts.ptr,
                set.accounts_before.ptr,
                set.accounts.len,
                set.transfers.ptr,
                set.transfers.len,
                @ptrCast(set.posted.ptr),
                set.posted.len,
            ));
            self.writeback_inflight = self.writeback_next;
            self.writeback_next ^= 1;
        }

        fn write_back_deliver(self: *StateMachine) void {
            const inflight = self.writeback_inflight orelse return;
            self.writeback_inflight = null;
            var counts: tbgpu.tbgpu_delta_counts = undefined;
            check(tbgpu.tbgpu_checkpoint_delta_wait(self.engine, &counts));
            self.write_back_apply(&self.writeback[inflight], &counts);
        }

        fn write_back_apply(self: *StateMachine, set: *const WriteBack, counts: *const tbgpu.tbgpu_delta_counts) void {
            const grooves = &self.forest.grooves;
            for (set.accounts[0..counts.accounts], set.accounts_before[0..counts.accounts]) |*a, before| {
                if (a.timestamp > counts.created_after) {
                    grooves.accounts.insert(a); // created since the previous write-back
                    continue;
                }
                if (grooves.accounts.get(a.id) == null) {
                    // The groove diffs the balance index trees against the old object: give its
                    // cache the version the forest holds (what a prefetch would have loaded).
                    var old = a.*;
                    old.debits_pending = before[0];
                    old.debits_posted = before[1];
                    old.credits_pending = before[2];
                    old.credits_posted = before[3];
                    grooves.accounts.objects_cache.upsert(&old);
                }
                grooves.accounts.upsert(a);
            }
            for (set.transfers[0..counts.transfers]) |*t| grooves.transfers.insert(t);
            for (set.posted[0..counts.posted]) |pair| {
                grooves.posted.insert(&PostedGrooveValue{
                    .timestamp = pair[0],
                    .fulfillment = if (pair[1] == 0) .posted else .voided,
                    .padding = [_]u8{0} ** 7,
                });
            }
        }

        /// The transfer log is three-quarters full: this bar writes back synchronously and evicts.
        fn log_needs_eviction(self: *StateMachine) bool {
            var stats: tbgpu.tbgpu_stats = undefined;
            check(tbgpu.tbgpu_get_stats(self.engine, &stats));
            return stats.log_capacity != 0 and stats.log_used * 4 >= stats.log_capacity * 3;
        }

        /// Bounded residency: once the bar is in the grooves (synchronously, nothing committed
        /// since), a transfer log three-quarters full drops what the forest now holds, keeping the
        /// newest quarter (tbgpu_evict_transfers); a later prefetch that names a dropped transfer
        /// loads it back (transfers_cold).
        fn evict_if_full(self: *StateMachine) void {
            if (!self.log_needs_eviction()) return;
            var stats: tbgpu.tbgpu_stats = undefined;
            check(tbgpu.tbgpu_get_stats(self.engine, &stats));
            var evicted: u64 = 0;
            check(tbgpu.tbgpu_evict_transfers(self.engine, stats.log_capacity / 4, &evicted));
            self.engine_evicted += evicted;
        }

        pub fn checkpoint(self: *StateMachine, callback: *const fn (*StateMachine) void) void {
            assert(self.compact_callback == null);
            assert(self.checkpoint_callback == null);
            // A bar in flight here (the trigger's) is not part of this checkpoint: its ops are after
            // the checkpoint op, so a restart replays them; it reaches the grooves one bar behind.
            self.checkpoint_callback = callback;
            self.forest.checkpoint(checkpoint_finish);
        }

        fn checkpoint_finish(forest: *Forest) void {
            const self = @fieldParentPtr(StateMachine, "forest", forest);
            const callback = self.checkpoint_callback.?;
            self.checkpoint_callback = null;
            callback(self);
        }
    };
}
