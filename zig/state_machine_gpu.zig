//! state_machine_gpu.zig — the reference-side binding a maintainer would add to route
//! StateMachine.commit(create_accounts | create_transfers | lookup_*) to the MI355X engine.
//!
//! SOURCE ONLY: this image has no Zig toolchain, so this file is not compiled here.  It shows the
//! wrapper shape against the reference's comptime duck-typed interface
//! (src/state_machine.zig:28-1150, consumers src/vsr/replica.zig and src/testing/cluster.zig:49-55,
//! SURVEY.md §8b).  Link with `-ltbgpu` and add `include/` to the C include path in build.zig.

const std = @import("std");
const assert = std.debug.assert;

const tbgpu = @cImport({
    @cInclude("tbgpu.h");
});

const ReferenceStateMachineType = @import("state_machine.zig").StateMachineType;

pub fn StateMachineType(comptime Storage: type, comptime config: @import("constants.zig").StateMachineConfig) type {
    // Keep the reference type for everything the engine does not replace (Forest, Workload,
    // prefetch plumbing, compaction and checkpoint of the LSM forest for durability).
    const Base = ReferenceStateMachineType(Storage, config);

    return struct {
        const StateMachine = @This();
        pub const Operation = Base.Operation;
        pub const Options = Base.Options;
        pub const Forest = Base.Forest;
        pub const Workload = Base.Workload;
        pub const constants = Base.constants;
        pub const Event = Base.Event;
        pub const Result = Base.Result;

        base: Base,
        engine: *tbgpu.tbgpu_t,

        // Mirrored fields the replica reads and writes (replica.zig:3621-3665, :5122-5131).
        prepare_timestamp: u64 = 0,
        commit_timestamp: u64 = 0,

        pub fn init(allocator: std.mem.Allocator, grid: anytype, options: Options) !StateMachine {
            var base = try Base.init(allocator, grid, options);
            errdefer base.deinit(allocator);
            const engine_config = tbgpu.tbgpu_config{
                .accounts_max = options.cache_entries_accounts,
                .transfers_max = options.cache_entries_transfers,
                .pass_events_max = constants.batch_max.create_transfers,
                .pass_batches_max = 1,
                .device = 0,
                .flags = 0,
            };
            var engine: ?*tbgpu.tbgpu_t = null;
            if (tbgpu.tbgpu_init(&engine_config, &engine) != tbgpu.TBGPU_STATUS_OK) return error.DeviceInit;
            return .{ .base = base, .engine = engine.? };
        }

        pub fn deinit(self: *StateMachine, allocator: std.mem.Allocator) void {
            tbgpu.tbgpu_deinit(self.engine);
            self.base.deinit(allocator);
        }

        pub fn reset(self: *StateMachine) void {
            self.base.reset();
            if (tbgpu.tbgpu_reset(self.engine) != tbgpu.TBGPU_STATUS_OK) @panic("tbgpu_reset");
            self.prepare_timestamp = 0;
            self.commit_timestamp = 0;
        }

        pub fn open(self: *StateMachine, callback: *const fn (*StateMachine) void) void {
            _ = self;
            _ = callback;
            @compileError("forward to Base.open with a callback adapter");
        }

        pub fn prepare(self: *StateMachine, operation: Operation, input: []align(16) u8) void {
            self.base.prepare_timestamp = self.prepare_timestamp;
            self.base.prepare(operation, input);
            self.prepare_timestamp = self.base.prepare_timestamp;
        }

        /// Objects are HBM-resident: complete synchronously (allowed, lsm/groove.zig:723-742).
        pub fn prefetch(
            self: *StateMachine,
            callback: *const fn (*StateMachine) void,
            op: u64,
            operation: Operation,
            input: []align(16) const u8,
        ) void {
            _ = op;
            _ = operation;
            _ = input;
            callback(self);
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
            var out_len: u32 = 0;
            const status = tbgpu.tbgpu_commit(
                self.engine,
                @intFromEnum(operation),
                timestamp,
                input.ptr,
                @intCast(input.len),
                output,
                @intCast(output.len),
                &out_len,
            );
            if (status != tbgpu.TBGPU_STATUS_OK) @panic(std.mem.span(tbgpu.tbgpu_last_error()));
            self.commit_timestamp = tbgpu.tbgpu_commit_timestamp(self.engine);
            return out_len;
        }

        /// Durability (write-back of dirty accounts / new transfers into the LSM forest) is the
        /// next row of SURVEY.md §8f; until then compaction has nothing from the engine to persist.
        pub fn compact(self: *StateMachine, callback: *const fn (*StateMachine) void, op: u64) void {
            _ = op;
            callback(self);
        }

        pub fn checkpoint(self: *StateMachine, callback: *const fn (*StateMachine) void) void {
            callback(self);
        }
    };
}
