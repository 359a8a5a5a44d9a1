"""Host-side mirror of the reference's StateMachine plugin interface, backed by the MI355X engine.

The reference's replica drives a comptime duck-typed `StateMachineType`
(src/state_machine.zig:28-1150; the contract is listed in SURVEY.md §8b):

    init(allocator, grid, options) / deinit / reset
    prepare(operation, input)                    -> prepare_timestamp += len(events)   (:336-343)
    prefetch(callback, op, operation, input)     -> async staging of objects          (:345-506)
    commit(client, op, timestamp, operation, input, output) -> reply bytes             (:508-540)
    compact(callback, op) / checkpoint(callback)                                        (:542-582)
    fields prepare_timestamp, commit_timestamp

`StateMachine` below keeps that shape; `commit` crosses into HIP through the C ABI
(include/tbgpu.h).  Objects live in HBM, so `prefetch` completes immediately (its callback fires
synchronously, which the reference allows: src/lsm/groove.zig:723-742).  `checkpoint` hands the
objects changed since the previous checkpoint (tbgpu_checkpoint_delta) to an optional write-back
sink — what a durable replica inserts / upserts into its forest; `compact` has nothing to do.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .types import ACCOUNT_DTYPE, BATCH_MAX, TRANSFER_DTYPE, U64_MAX, Operation


@dataclass
class Options:
    """StateMachine.Options (state_machine.zig:216-221) plus the HBM sizing the engine needs."""
    accounts_max: int = 1 << 16
    transfers_max: int = 1 << 20
    pass_events_max: int = 8190 * 64
    pass_batches_max: int = 512
    device: int = 0
    # Two or more HIP device ordinals: a node engine, one shard per entry (include/tbgpu.h
    # tbgpu_config.devices; an ordinal may repeat: logical shards sharing one GPU).
    devices: tuple = ()
    profile: bool = False
    sequential_fallback: bool = False  # ordered fallback on one lane (tb_replay) instead of tb_flow
    # Limit checks: "auto" (scan rounds while they decide enough, then the in-order sweep), "early"
    # (sweep after the first round) or "off" (rounds only, else the ordered run); the sweep is one
    # walker per limit account, or with "window" / "window-early" one wave walking the checks in
    # event order (round 2's form).  Identical results.
    bounds_sweep: str = "auto"
    # Reference cache options are accepted for interface parity; the HBM tables hold every object.
    lsm_forest_node_count: int = 0
    cache_entries_accounts: int = 0
    cache_entries_transfers: int = 0
    cache_entries_posted: int = 0


class Engine:
    """Thin ctypes handle over one tbgpu engine: one GPU, or a node of shards (Options.devices)."""

    def __init__(self, options=None, **kw):
        options = options or Options(**kw)
        self.options = options
        self.lib = _lib.load()
        cfg = _lib.tbgpu_config(options.accounts_max, options.transfers_max, options.pass_events_max,
                                options.pass_batches_max, options.device,
                                (_lib.CONFIG_PROFILE if options.profile else 0)
                                | (_lib.CONFIG_SEQUENTIAL_FALLBACK if options.sequential_fallback else 0)
                                | {"auto": 0, "early": _lib.CONFIG_SWEEP_EARLY,
                                   "off": _lib.CONFIG_SWEEP_OFF, "window": _lib.CONFIG_SWEEP_WINDOW,
                                   "window-early": _lib.CONFIG_SWEEP_WINDOW | _lib.CONFIG_SWEEP_EARLY,
                                   }[options.bounds_sweep])
        devices = list(options.devices or ())
        if len(devices) > len(cfg.devices):
            raise ValueError("at most %d devices" % len(cfg.devices))
        cfg.device_count = len(devices)
        for i, d in enumerate(devices):
            cfg.devices[i] = int(d)
        h = ctypes.c_void_p()
        _lib.check(self.lib.tbgpu_init(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            for _caps, bufs in (getattr(self, "_delta_bufs", None) or {}).values():
                for arr in bufs:
                    self.lib.tbgpu_unregister_host(self.h, arr.ctypes.data)
            self._delta_bufs = None
            self.lib.tbgpu_deinit(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.tbgpu_reset(self.h))

    # -- commit ------------------------------------------------------------------------------
    def commit(self, operation, timestamp, body):
        """StateMachine.commit: returns the reply body bytes."""
        body = bytes(body)
        op = int(operation)
        if op in (Operation.lookup_accounts, Operation.lookup_transfers):
            cap = max(len(body) // 16 * 128, 128)
        else:
            cap = max(len(body) // 128 * 8, 8)
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint32(0)
        src = ctypes.create_string_buffer(body, len(body)) if body else None
        _lib.check(self.lib.tbgpu_commit(self.h, op, timestamp, src, len(body), out, cap, ctypes.byref(n)))
        return out.raw[:n.value]

    def commit_many(self, operation, timestamps, bodies):
        """N prepares in one device pass; returns the N reply bodies."""
        n = len(bodies)
        if n == 0:
            return []
        bufs = [ctypes.create_string_buffer(bytes(b), len(b)) if len(b) else None for b in bodies]
        outs = [ctypes.create_string_buffer(max(len(b) // 128 * 8, 8)) for b in bodies]
        ts = (ctypes.c_uint64 * n)(*timestamps)
        ins = (ctypes.c_void_p * n)(*[ctypes.cast(b, ctypes.c_void_p) if b is not None else None for b in bufs])
        lens = (ctypes.c_uint32 * n)(*[len(b) for b in bodies])
        outp = (ctypes.c_void_p * n)(*[ctypes.cast(o, ctypes.c_void_p) for o in outs])
        out_lens = (ctypes.c_uint32 * n)()
        _lib.check(self.lib.tbgpu_commit_many(self.h, int(operation), n, ts, ins, lens, outp, out_lens))
        return [outs[k].raw[:out_lens[k]] for k in range(n)]

    def commit_pipelined(self, operation, timestamps, lens, events, chunk_batches=0, latency=False, replies=None):
        """tbgpu_commit_pipelined over prepares stored back to back in the host array `events`
        (uint8; register it with register_host for DMA at full PCIe rate).  Returns (reply_bytes
        uint32[n], replies uint8 buffer with prepare k's reply at 8 * its first event, latency_ms
        float64[n] or None)."""
        n = len(lens)
        lens = np.asarray(lens, dtype=np.uint64)
        first = np.zeros(n, dtype=np.uint64)
        if n > 1:
            first[1:] = np.cumsum(lens[:-1])
        total = int(lens.sum())
        assert events.dtype == np.uint8 and events.flags["C_CONTIGUOUS"] and events.nbytes >= total * 128
        if replies is None or replies.nbytes < total * 8:
            replies = np.empty(max(total, 1) * 8, dtype=np.uint8)
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        ins = (first * 128 + np.uint64(events.ctypes.data)).astype(np.uint64)
        outs = (first * 8 + np.uint64(replies.ctypes.data)).astype(np.uint64)
        in_lens = (lens * 128).astype(np.uint32)
        out_lens = np.zeros(n, dtype=np.uint32)
        lat = np.zeros(n, dtype=np.float64) if latency else None
        P = ctypes.c_void_p
        _lib.check(self.lib.tbgpu_commit_pipelined(
            self.h, int(operation), n, ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            ins.ctypes.data_as(ctypes.POINTER(P)), in_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            outs.ctypes.data_as(ctypes.POINTER(P)), out_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            int(chunk_batches), lat.ctypes.data if lat is not None else None))
        return out_lens, replies, lat

    def commit_pipelined_ptrs(self, operation, timestamps, lens, in_ptrs, replies, chunk_batches=0, latency=False):
        """tbgpu_commit_pipelined over prepares at explicit host addresses (in_ptrs[k]: prepare k's
        body, lens[k] events); replies: a uint8 host buffer, prepare k's reply at 8 * its first event
        (prepares in order).  Returns (reply_bytes uint32[n], latency_ms float64[n] or None)."""
        n = len(lens)
        lens = np.asarray(lens, dtype=np.uint64)
        first = np.zeros(n, dtype=np.uint64)
        if n > 1:
            first[1:] = np.cumsum(lens[:-1])
        assert replies.dtype == np.uint8 and replies.nbytes >= int(lens.sum()) * 8
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        ins = np.ascontiguousarray(in_ptrs, dtype=np.uint64)
        outs = (first * 8 + np.uint64(replies.ctypes.data)).astype(np.uint64)
        in_lens = (lens * 128).astype(np.uint32)
        out_lens = np.zeros(n, dtype=np.uint32)
        lat = np.zeros(n, dtype=np.float64) if latency else None
        P = ctypes.c_void_p
        _lib.check(self.lib.tbgpu_commit_pipelined(
            self.h, int(operation), n, ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
            ins.ctypes.data_as(ctypes.POINTER(P)), in_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            outs.ctypes.data_as(ctypes.POINTER(P)), out_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            int(chunk_batches), lat.ctypes.data if lat is not None else None))
        return out_lens, lat

    def register_host(self, array):
        """Pin a host array for DMA (the replica's message pool; tbgpu_register_host)."""
        _lib.check(self.lib.tbgpu_register_host(self.h, array.ctypes.data, array.nbytes))

    def unregister_host(self, array):
        _lib.check(self.lib.tbgpu_unregister_host(self.h, array.ctypes.data))

    def commit_device_async(self, operation, timestamps, lens, events_dev, results_dev, reply_bytes_dev):
        n = len(lens)
        # numpy's conversion, not a per-element ctypes array: 12K prepares took ~1.2 ms of host time
        # before the call reached the engine (a headline step is ~18 ms)
        ts = np.ascontiguousarray(timestamps, dtype=np.uint64)
        ls = np.ascontiguousarray(lens, dtype=np.uint32)
        assert len(ts) == n
        _lib.check(self.lib.tbgpu_commit_device_async(self.h, int(operation), n,
                                                      ts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                      ls.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                      events_dev, results_dev, reply_bytes_dev))

    def sync(self):
        _lib.check(self.lib.tbgpu_sync(self.h))

    def log_window(self, events):
        """Device address where the next `events` transfer records go (tbgpu_log_window): prepares
        placed there and committed with commit_device_async(129, ..., events_dev=window) are committed
        in place."""
        w = ctypes.c_void_p(0)
        _lib.check(self.lib.tbgpu_log_window(self.h, int(events), ctypes.byref(w)))
        return int(w.value)

    @property
    def commit_timestamp(self):
        return self.lib.tbgpu_commit_timestamp(self.h)

    def set_balances(self, account_id, dp, dpost, cp, cpost):
        arr = (ctypes.c_uint64 * 8)()
        for i, v in enumerate((dp, dpost, cp, cpost)):
            arr[2 * i] = v & U64_MAX
            arr[2 * i + 1] = v >> 64
        _lib.check(self.lib.tbgpu_test_set_balances(self.h, account_id & U64_MAX, account_id >> 64, arr))

    # -- parity read-back --------------------------------------------------------------------
    def _export(self, fn, dtype, cap):
        out = np.zeros(max(cap, 1), dtype=dtype)
        n = ctypes.c_uint64(0)
        _lib.check(fn(self.h, out.ctypes.data, cap, ctypes.byref(n)))
        return out[:n.value]

    def export_accounts(self, cap=None):
        return self._export(self.lib.tbgpu_export_accounts, ACCOUNT_DTYPE, cap or self.options.accounts_max)

    def export_transfers(self, cap=None):
        return self._export(self.lib.tbgpu_export_transfers, TRANSFER_DTYPE, cap or self.options.transfers_max)

    def export_posted(self, cap=None):
        cap = cap or self.options.transfers_max
        out = np.zeros((max(cap, 1), 2), dtype=np.uint64)
        n = ctypes.c_uint64(0)
        _lib.check(self.lib.tbgpu_export_posted(self.h, out.ctypes.data, cap, ctypes.byref(n)))
        return out[:n.value]

    def stats(self):
        s = _lib.tbgpu_stats()
        _lib.check(self.lib.tbgpu_get_stats(self.h, ctypes.byref(s)))
        return {f: (list(getattr(s, f)) if f in ("flow_phase_ms", "walk_dbg", "span_ms", "span_launches", "node_shard_account_bytes") else getattr(s, f)) for f, _ in s._fields_}

    def reset_stats(self):
        self.lib.tbgpu_reset_stats(self.h)

    PROF_VALIDATE, PROF_RESOLVE, PROF_REPLAY, PROF_CLEAR, PROF_PASS, PROF_APPLY, PROF_ALL = 1, 2, 4, 8, 16, 32, 63
    PROF_SPANS = 64  # the device-clock launch spans only (no HIP event pair)

    def checkpoint_delta(self, caps=None, copy=True):
        """Objects changed since the previous call (groove write-back): a Delta of accounts (in no
        particular order), transfers (by timestamp) and posted pairs {pending timestamp,
        fulfillment}.  caps: initial buffer sizes (accounts, transfers, posted); grown and retried
        when too small (the engine says what suffices).  copy=False returns views of the buffers the
        engine keeps registered for DMA: valid only until the next write-back."""
        counts = _lib.tbgpu_delta_counts()
        caps = list(caps) if caps else [1024, 1024, 1024]
        if getattr(self, "_wb_inflight", None) is not None:  # its buffers belong to the engine until the wait
            raise _lib.EngineError(_lib.STATUS_INVALID, "an asynchronous write-back is in flight "
                                                        "(checkpoint_delta_wait first)")
        while True:
            a, before, t, p = self._delta_buffers(caps, 0)
            st = self.lib.tbgpu_checkpoint_delta(self.h, a.ctypes.data, before.ctypes.data, caps[0], t.ctypes.data,
                                                 caps[1], p.ctypes.data, caps[2], ctypes.byref(counts))
            need = [counts.accounts, counts.transfers, counts.posted]
            if st == _lib.STATUS_INVALID and any(n > c for n, c in zip(need, caps)):
                caps = [max(c, n) for c, n in zip(caps, need)]
                continue
            _lib.check(st)
            return self._delta(a, before, t, p, counts, copy)

    def checkpoint_delta_async(self, caps):
        """tbgpu_checkpoint_delta_async into one of two registered buffer sets of at least `caps`
        (accounts, transfers, posted) entries — size them for a bar, as the Zig wrapper does; the
        objects land while later commits run.  checkpoint_delta_wait() returns the Delta."""
        if getattr(self, "_wb_inflight", None) is not None:  # never touch a set the engine may be copying into
            raise _lib.EngineError(_lib.STATUS_INVALID, "an asynchronous write-back is in flight "
                                                        "(checkpoint_delta_wait first)")
        which = 1 - getattr(self, "_wb_set", 1)
        a, before, t, p = self._delta_buffers(list(caps), which)
        _lib.check(self.lib.tbgpu_checkpoint_delta_async(self.h, a.ctypes.data, before.ctypes.data, caps[0],
                                                         t.ctypes.data, caps[1], p.ctypes.data, caps[2]))
        self._wb_set = which  # flipped only once the call succeeded
        self._wb_inflight = (a, before, t, p)

    def checkpoint_delta_wait(self, copy=True):
        counts = _lib.tbgpu_delta_counts()
        _lib.check(self.lib.tbgpu_checkpoint_delta_wait(self.h, ctypes.byref(counts)))
        a, before, t, p = self._wb_inflight
        self._wb_inflight = None
        return self._delta(a, before, t, p, counts, copy)

    @staticmethod
    def _delta(a, before, t, p, counts, copy):
        need = [counts.accounts, counts.transfers, counts.posted]
        parts = (a[:need[0]], t[:need[1]], p[:need[2]], before[:need[0]])
        if copy:
            parts = tuple(x.copy() for x in parts)
        return Delta(*parts, counts.created_after)

    def _delta_buffers(self, caps, which):
        """Write-back buffer set `which` (0 / 1) of at least `caps` entries, kept (and registered)
        across calls."""
        sets = getattr(self, "_delta_bufs", None) or {}
        have = sets.get(which)
        if have is not None and all(h >= c for h, c in zip(have[0], caps)):
            return have[1]
        if have is not None:
            for arr in have[1]:
                _lib.check(self.lib.tbgpu_unregister_host(self.h, arr.ctypes.data))
        caps = [max(c, 1) for c in caps]
        bufs = (np.empty(caps[0], dtype=ACCOUNT_DTYPE), np.empty((caps[0], 8), dtype=np.uint64),
                np.empty(caps[1], dtype=TRANSFER_DTYPE), np.empty((caps[2], 2), dtype=np.uint64))
        for arr in bufs:
            _lib.check(self.lib.tbgpu_register_host(self.h, arr.ctypes.data, arr.nbytes))
        sets[which] = (caps, bufs)
        self._delta_bufs = sets
        return bufs

    def ledger_summary(self):
        """{"debits_pending", "debits_posted", "credits_pending", "credits_posted": u128 sums over every
        account (every shard of a node), "accounts": live accounts, "stray": balances held by a shard
        that is not the account's owner (node engines; must be 0)} — tbgpu_bench_ledger_summary."""
        s = _lib.tbgpu_ledger_summary()
        _lib.check(self.lib.tbgpu_bench_ledger_summary(self.h, ctypes.byref(s)))
        names = ("debits_pending", "debits_posted", "credits_pending", "credits_posted")
        out = {n: int(s.sums[2 * i]) | (int(s.sums[2 * i + 1]) << 64) for i, n in enumerate(names)}
        out.update(accounts=int(s.accounts), stray=int(s.stray))
        return out

    def checkpoint_mark(self):
        """Take the current state as written back (tbgpu_bench_checkpoint_mark)."""
        _lib.check(self.lib.tbgpu_bench_checkpoint_mark(self.h))

    def shard(self, d):
        """A node engine's shard d as an Engine sharing its handle (tbgpu_bench_node_shard): device
        buffers, copies and the generators on shard d's GPU.  Never closed on its own."""
        h = ctypes.c_void_p()
        _lib.check(self.lib.tbgpu_bench_node_shard(self.h, int(d), ctypes.byref(h)))
        view = Engine.__new__(Engine)
        view.options, view.lib, view.h = self.options, self.lib, h
        view.close = lambda: None
        return view

    def walk_merge_max(self, segments):
        """Heavy segments the limit-check sweep walks merged on one wave at most (0: a wave each)."""
        _lib.check(self.lib.tbgpu_bench_walk_merge_max(self.h, int(segments)))

    def legs_min_events(self, events):
        """Passes of >= events transfers use the sorted balance legs (0: every pass)."""
        _lib.check(self.lib.tbgpu_bench_legs_min_events(self.h, int(events)))

    MIX_PARTS = ("stream", "probe", "cas", "stream+probe", "stream+cas", "probe+cas", "all")

    def access_mix(self, transfers):
        """Mean ms of kernel 1's memory-access mix without its logic, per part (tbgpu_bench.h)."""
        out = (ctypes.c_double * 7)()
        _lib.check(self.lib.tbgpu_bench_access_mix(self.h, int(transfers), out))
        return dict(zip(self.MIX_PARTS, list(out)))

    def profile_mask(self, mask):
        """Kernels timed with HIP events when profiling (include/tbgpu_bench.h)."""
        _lib.check(self.lib.tbgpu_bench_profile_mask(self.h, mask))

    # -- multi-GPU primitives (include/tbgpu_shard.h; driven by tigerbeetle_amd.sharded) -------
    def route_init(self, world, events_max):
        _lib.check(self.lib.tbgpu_route_init(self.h, world, events_max))

    def fetch_accounts(self, ids):
        """ids: uint64 [n, 2] (lo, hi).  Returns (ACCOUNT_DTYPE[n], found uint8[n])."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        n = ids.shape[0]
        out = np.zeros(n, dtype=ACCOUNT_DTYPE)
        found = np.zeros(n, dtype=np.uint8)
        if n:
            _lib.check(self.lib.tbgpu_fetch_accounts(self.h, ids.ctypes.data, n, out.ctypes.data, found.ctypes.data))
        return out, found

    def fetch_transfers(self, ids):
        """ids: uint64 [n, 2].  Returns (TRANSFER_DTYPE[n], state uint8[n]: 0 absent, 1 + posted)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        n = ids.shape[0]
        out = np.zeros(n, dtype=TRANSFER_DTYPE)
        state = np.zeros(n, dtype=np.uint8)
        if n:
            _lib.check(self.lib.tbgpu_fetch_transfers(self.h, ids.ctypes.data, n, out.ctypes.data, state.ctypes.data))
        return out, state

    def upsert_accounts(self, records):
        records = np.ascontiguousarray(records, dtype=ACCOUNT_DTYPE)
        if len(records):
            _lib.check(self.lib.tbgpu_upsert_accounts(self.h, records.ctypes.data, len(records)))

    def load_accounts(self, records):
        """Insert the accounts the engine lacks (replica restart warm-up, tbgpu_load_accounts)."""
        records = np.ascontiguousarray(records, dtype=ACCOUNT_DTYPE)
        if len(records):
            _lib.check(self.lib.tbgpu_load_accounts(self.h, records.ctypes.data, len(records)))

    def load_transfers(self, records, posted_state):
        records = np.ascontiguousarray(records, dtype=TRANSFER_DTYPE)
        posted_state = np.ascontiguousarray(posted_state, dtype=np.uint8)
        if len(records):
            _lib.check(self.lib.tbgpu_load_transfers(self.h, records.ctypes.data, posted_state.ctypes.data,
                                                     len(records)))

    def evict_transfers(self, keep):
        """Drop the written-back transfers older than the newest `keep` log positions
        (tbgpu_evict_transfers); returns how many left."""
        n = ctypes.c_uint64(0)
        _lib.check(self.lib.tbgpu_evict_transfers(self.h, int(keep), ctypes.byref(n)))
        return n.value

    def transfers_maybe_cold(self, ids):
        """ids: uint64 [n, 2] (lo, hi).  Returns bool[n]: not resident and maybe evicted (load them
        from the forest before the commit that names them)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(ids), dtype=np.uint8)
        if len(ids):
            _lib.check(self.lib.tbgpu_transfers_maybe_cold(self.h, ids.ctypes.data, len(ids), out.ctypes.data))
        return out.astype(bool)

    def set_commit_timestamp(self, timestamp):
        _lib.check(self.lib.tbgpu_set_commit_timestamp(self.h, int(timestamp)))

    def upsert_transfers(self, records, state):
        records = np.ascontiguousarray(records, dtype=TRANSFER_DTYPE)
        state = np.ascontiguousarray(state, dtype=np.uint8)
        if len(records):
            _lib.check(self.lib.tbgpu_upsert_transfers(self.h, records.ctypes.data, state.ctypes.data, len(records)))

    # -- device memory + workload generation (bench) -----------------------------------------
    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        _lib.check(self.lib.tbgpu_device_alloc(self.h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, ptr):
        _lib.check(self.lib.tbgpu_device_free(self.h, ptr))

    def to_host(self, ptr, nbytes):
        out = np.empty(nbytes, dtype=np.uint8)
        _lib.check(self.lib.tbgpu_copy_to_host(self.h, out.ctypes.data, ptr, nbytes))
        return out

    def to_device(self, ptr, array):
        array = np.ascontiguousarray(array)
        _lib.check(self.lib.tbgpu_copy_to_device(self.h, ptr, array.ctypes.data, array.nbytes))

    def generate_accounts(self, out_dev, first, count, seed=42, limit_permille=0, account_count=0, hot_limited=0):
        """hot_limited > 0 (the hottest Zipf ranks get a limit flag too) needs account_count."""
        w = _lib.tbgpu_workload(seed, account_count, 0, limit_permille, 0.0, hot_limited, 0)
        _lib.check(self.lib.tbgpu_bench_generate_accounts(self.h, out_dev, first, count, ctypes.byref(w)))

    def generate_transfers(self, out_dev, first, count, account_count, seed=42, kind=0, limit_permille=0,
                           zipf_s=1.2, hot_limited=0):
        """kind 0: C2 uniform; 1: C3 Zipf + limit-account funding; 2: C4 chains / two-phase / balancing
        (include/tbgpu_bench.h).  limit_permille must match generate_accounts' for kind 1."""
        w = _lib.tbgpu_workload(seed, account_count, kind, limit_permille, zipf_s, hot_limited, 0)
        _lib.check(self.lib.tbgpu_bench_generate_transfers(self.h, out_dev, first, count, ctypes.byref(w)))

    def reset_transfers(self):
        _lib.check(self.lib.tbgpu_bench_reset_transfers(self.h))

    def pass_latencies(self, cap=1 << 20):
        out = np.zeros(cap, dtype=np.float64)
        n = ctypes.c_uint64(0)
        _lib.check(self.lib.tbgpu_bench_pass_latencies(self.h, out.ctypes.data, cap, ctypes.byref(n)))
        return out[:n.value]

    def marker(self, slot):
        _lib.check(self.lib.tbgpu_marker(self.h, slot))

    def marker_elapsed_ms(self, a, b):
        return self.lib.tbgpu_marker_elapsed_ms(self.h, a, b)


@dataclass
class Delta:
    """One groove write-back (tbgpu_checkpoint_delta)."""
    accounts: np.ndarray
    transfers: np.ndarray
    posted: np.ndarray
    # [n, 8] u64: {dp, dpost, cp, cpost} (lo, hi) of each account as of the previous write-back
    accounts_before: np.ndarray = None
    # accounts with a timestamp above this were created since the previous write-back (insert)
    created_after: int = 0


class StateMachine:
    """The reference's StateMachine interface over one Engine."""

    Operation = Operation
    batch_max = BATCH_MAX

    def __init__(self, options=None, write_back=None, **kw):
        self.engine = Engine(options, **kw)
        self.write_back = write_back  # called by checkpoint with a Delta
        self.prepare_timestamp = 0
        self.commit_timestamp = 0

    def deinit(self):
        self.engine.close()

    def reset(self):
        self.engine.reset()
        self.prepare_timestamp = 0
        self.commit_timestamp = 0

    @staticmethod
    def event_count(operation, body):
        if operation in (Operation.create_accounts, Operation.create_transfers):
            return len(body) // 128
        return 0

    def prepare(self, operation, body):
        """state_machine.zig:336-343."""
        self.prepare_timestamp += self.event_count(Operation(operation), body)

    def prefetch(self, callback, op, operation, body):
        """state_machine.zig:345-506.  Every object is HBM-resident: complete synchronously."""
        assert op != 0
        callback(self)

    def commit(self, client, op, timestamp, operation, body):
        """state_machine.zig:508-540.  Returns the reply body (bytes)."""
        del client
        assert op != 0
        reply = self.engine.commit(int(operation), timestamp, body)
        self.commit_timestamp = self.engine.commit_timestamp
        return reply

    def compact(self, callback, op):
        del op
        callback(self)

    def checkpoint(self, callback):
        delta = self.engine.checkpoint_delta()
        if self.write_back is not None:
            self.write_back(delta)
        callback(self)
