"""Multi-GPU commit of the create_accounts / create_transfers path.

One engine per GPU, one process per GPU, collectives over torch.distributed (backend "nccl" =
RCCL over xGMI on an MI355X node; "gloo" for the CPU tests and for several ranks sharing one GPU).
The partition and the pass protocol are documented in include/tbgpu_shard.h and DESIGN.md §6:

* account records (their immutable fields) are replicated: every rank commits every
  create_accounts prepare;
* account balances are owner-partitioned: they live on owner(id) = tbgpu_home(id, world) only
  (every other rank holds zeros), and the legs of committed transfers are routed to the owners;
* a transfer lives on its home rank, tbgpu_home(id, world).

Global order.  A collective pass takes every rank's prepares.  The global prepare order is rank 0's
prepares, then rank 1's, ..., and timestamps must increase in that order: the results are exactly
those of one StateMachine committing the concatenation (src/state_machine.zig:508-540).

A clean create_transfers pass is routed: one all-to-all of events (+ their execute timestamps) to
their homes, a routed commit on every home, one all-to-all of the committed transfers' balance
legs to the accounts' owners, one all-to-all of result codes back.  A dirty pass
(linked / post / void / balancing event, limit-flag account, or no global overflow certificate)
is committed by rank 0 on a scratch engine after prefetching the referenced transfers from their
homes and the summed balances of the touched accounts (the reference's prefetch -> commit split,
src/state_machine.zig:345-506), then its effects are written back.
"""
import dataclasses

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .types import ACCOUNT_DTYPE, TRANSFER_DTYPE, U64_MAX, Operation, TransferFlags

U64 = 1 << 64
U128 = 1 << 128
_BAL_FIELDS = ("debits_pending", "debits_posted", "credits_pending", "credits_posted")
_ROUTED_NEVER = int(TransferFlags.linked | TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer
                    | TransferFlags.balancing_debit | TransferFlags.balancing_credit)


@dataclasses.dataclass
class RoutePlan:
    counts: list  # events for each home rank
    S: int        # saturating sum of every amount of this rank's share of the pass
    bound: int    # this engine's balance bound
    dirty: int    # _lib.DIRTY_* bits


class PassResult:
    """Replies of this rank's prepares of one pass.  Prepare k's reply is the {index, result} u32
    pairs results[2*offsets[k] : 2*offsets[k] + reply_bytes[k] // 4] (tensors, possibly on the GPU)."""

    def __init__(self, results, reply_bytes, offsets):
        self.results = results
        self.reply_bytes = reply_bytes
        self.offsets = offsets

    def replies(self):
        rb = self.reply_bytes.cpu().numpy().astype(np.int64)
        if rb.sum() == 0:
            return [b""] * len(rb)
        res = self.results.cpu().numpy().view(np.uint32)
        out = []
        for k, nbytes in enumerate(rb):
            o = 2 * int(self.offsets[k])
            out.append(res[o:o + nbytes // 4].tobytes())
        return out

    @staticmethod
    def from_bytes(replies, lens, device):
        offsets = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
        results = np.zeros(2 * max(int(offsets[-1]), 1), dtype=np.uint32)
        rb = np.zeros(len(lens), dtype=np.int32)
        for k, r in enumerate(replies):
            a = np.frombuffer(r, dtype=np.uint32)
            results[2 * offsets[k]:2 * offsets[k] + len(a)] = a
            rb[k] = len(r)
        return PassResult(torch.from_numpy(results.view(np.int32)).to(device), torch.from_numpy(rb).to(device), offsets)


DEMOTED = 0xFE  # a routed event its home did not commit: a dependent event reads its id


def _key64(ids):
    """A 64-bit key of {lo, hi} int64 pairs for set membership (a collision only demotes an extra
    event to the sequencer, which is always exact)."""
    return ids[:, 0] ^ (ids[:, 1] * -7046029254386353131)  # 0x9E3779B97F4A7C15 as int64


def _host_array(values, dtype, ctype):
    """values as a C array for the engine (at least one element): numpy's conversion, and the array
    object with it so that the buffer outlives the call."""
    import ctypes
    a = np.zeros(max(len(values), 1), dtype=dtype)
    a[:len(values)] = np.asarray(values, dtype=dtype)
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def _stream_sync(device):
    """Wait for torch's current stream on `device` (its work, and the RCCL collectives it waits
    on), not the whole device: a copy of the next pass on another stream keeps running."""
    torch.cuda.current_stream(device).synchronize()


def _events_np(events):
    return events.cpu().numpy().reshape(-1).view(TRANSFER_DTYPE)


def _u128(lo, hi):
    return (int(hi) << 64) | int(lo)


def _ids(lo, hi):
    return np.stack([np.asarray(lo, dtype=np.uint64), np.asarray(hi, dtype=np.uint64)], axis=1)


def _unique_ids(ids):
    ids = ids[~(((ids[:, 0] == 0) & (ids[:, 1] == 0)) | ((ids[:, 0] == U64_MAX) & (ids[:, 1] == U64_MAX)))]
    if len(ids) == 0:
        return ids.reshape(0, 2)
    return np.unique(ids, axis=0)


class GpuShard:
    """Backend of one rank: the HIP engine on this rank's GPU (include/tbgpu_shard.h)."""

    def __init__(self, engine, world, events_max, device=None):
        self.engine = engine
        self.lib = engine.lib
        self.world = world
        self.device = device if device is not None else torch.device("cuda", engine.options.device)
        self.events_max = events_max
        engine.route_init(world, events_max)
        self._scratch = None

    # -- clean pass ------------------------------------------------------------------------
    def plan(self, timestamps, lens, events, skip=None):
        import ctypes
        n = events.shape[0]
        nb = len(lens)
        send_events = torch.empty_like(events)
        slots = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        p = _lib.tbgpu_route_plan()
        ts = _host_array(timestamps, np.uint64, ctypes.c_uint64)
        ls = _host_array(lens, np.uint32, ctypes.c_uint32)
        _stream_sync(self.device)
        _lib.check(self.lib.tbgpu_route_plan_build(self.engine.h, nb, ts, ls, events.data_ptr(),
                                                   skip.data_ptr() if skip is not None else None,
                                                   send_events.data_ptr(), slots.data_ptr(), ctypes.byref(p)))
        plan = RoutePlan([int(p.send_counts[i]) for i in range(self.world)], _u128(p.sum_lo, p.sum_hi),
                         _u128(p.bound_lo, p.bound_hi), int(p.dirty))
        return plan, send_events[:sum(plan.counts)], slots[:n]

    def commit_routed(self, events, ts_max, cert):
        m = events.shape[0]
        codes = torch.empty(max(m, 1), dtype=torch.uint8, device=self.device)
        if m:
            _stream_sync(self.device)
            _lib.check(self.lib.tbgpu_commit_routed_async(self.engine.h, m, events.data_ptr(), ts_max, cert,
                                                          codes.data_ptr()))
            self.engine.sync()
        return codes[:m]

    def dependents(self, lens, events, marked):
        """Per-event dependency classes of a dirty pass (tbgpu_route_dependents): uint8 tensor."""
        import ctypes
        n, nb = events.shape[0], len(lens)
        dep = torch.zeros(max(n, 1), dtype=torch.uint8, device=self.device)
        if n:
            ls = _host_array(lens, np.uint32, ctypes.c_uint32)
            marked = np.ascontiguousarray(marked, dtype=np.uint64).reshape(-1, 2)
            _stream_sync(self.device)
            _lib.check(self.lib.tbgpu_route_dependents(self.engine.h, nb, ls, events.data_ptr(),
                                                       marked.ctypes.data if len(marked) else None, len(marked),
                                                       dep.data_ptr()))
        return dep[:n]

    def homes(self, ids):
        """home(id) of an int64 [m, 2] {lo, hi} tensor on the device: uint8 tensor."""
        out = torch.empty(max(ids.shape[0], 1), dtype=torch.uint8, device=self.device)
        if ids.shape[0]:
            ids = ids.contiguous()
            _stream_sync(self.device)
            _lib.check(self.lib.tbgpu_route_homes(self.engine.h, ids.data_ptr(), ids.shape[0], self.world, out.data_ptr()))
        return out[:ids.shape[0]]

    def commit_routed_owner(self, events, ts_max, cert, rank):
        """The home's routed commit with owner-partitioned balances: result codes, plus the legs of
        every committed transfer grouped by owner (a [sum, 5] int64 tensor, owner by owner) and the
        per-owner counts (host list)."""
        m = events.shape[0]
        codes = torch.empty(max(m, 1), dtype=torch.uint8, device=self.device)
        cap = max(2 * m, 1)
        legs = torch.empty((self.world * cap, 5), dtype=torch.int64, device=self.device)
        counts = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        _stream_sync(self.device)
        _lib.check(self.lib.tbgpu_commit_routed_owner_async(self.engine.h, m, events.data_ptr(), ts_max, cert,
                                                            codes.data_ptr(), self.world, rank, legs.data_ptr(), cap,
                                                            counts.data_ptr()))
        self.engine.sync()
        c = [int(x) for x in counts.cpu().tolist()]
        send = torch.cat([legs[o * cap:o * cap + c[o]] for o in range(self.world)])
        return codes[:m], send, c

    def apply_owner_legs(self, legs, cert):
        if legs.shape[0]:
            _stream_sync(self.device)
            _lib.check(self.lib.tbgpu_apply_owner_legs_async(self.engine.h, legs.data_ptr(), legs.shape[0], cert))

    def replies(self, lens, slots, codes_back):
        import ctypes
        nb = len(lens)
        n = int(sum(lens))
        results = torch.empty(2 * max(n, 1), dtype=torch.int32, device=self.device)
        reply_bytes = torch.zeros(max(nb, 1), dtype=torch.int32, device=self.device)
        if nb:
            ls = _host_array(lens, np.uint32, ctypes.c_uint32)
            _stream_sync(self.device)
            _lib.check(self.lib.tbgpu_route_replies_async(self.engine.h, nb, ls, slots.data_ptr(), codes_back.data_ptr(),
                                                          results.data_ptr(), reply_bytes.data_ptr()))
            self.engine.sync()
        offsets = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
        return PassResult(results, reply_bytes[:nb], offsets)

    # -- host-side primitives ----------------------------------------------------------------
    def commit_batches(self, operation, timestamps, bodies):
        return self.engine.commit_many(operation, timestamps, bodies)

    def fetch_accounts(self, ids):
        return self.engine.fetch_accounts(ids)

    def fetch_transfers(self, ids):
        return self.engine.fetch_transfers(ids)

    def upsert_accounts(self, records):
        self.engine.upsert_accounts(records)

    def upsert_transfers(self, records, state):
        self.engine.upsert_transfers(records, state)

    @property
    def commit_timestamp(self):
        return self.engine.commit_timestamp

    def export_accounts(self):
        return self.engine.export_accounts()

    def export_transfers(self):
        return self.engine.export_transfers()

    def export_posted(self):
        return self.engine.export_posted()

    def scratch(self, accounts, transfers):
        """A scratch engine on this GPU for dirty passes, sized for the pass (grown on demand)."""
        from .state_machine import Engine, Options
        need_a = max(1024, 1 << int(accounts).bit_length())
        need_t = max(1024, 1 << int(transfers).bit_length())
        s = self._scratch
        if s is None or s.options.accounts_max < need_a or s.options.transfers_max < need_t:
            if s is not None:
                s.close()
            o = self.engine.options
            s = Engine(Options(accounts_max=need_a, transfers_max=need_t, pass_events_max=8190 * 64,
                               pass_batches_max=512, device=o.device))
            self._scratch = s
        else:
            s.reset()
        return _ScratchGpu(s)


class _ScratchGpu:
    def __init__(self, engine):
        self.engine = engine

    def upsert_accounts(self, records):
        self.engine.upsert_accounts(records)

    def upsert_transfers(self, records, state):
        self.engine.upsert_transfers(records, state)

    def fetch_accounts(self, ids):
        return self.engine.fetch_accounts(ids)

    def fetch_transfers(self, ids):
        return self.engine.fetch_transfers(ids)

    def commit_batches(self, operation, timestamps, bodies):
        return self.engine.commit_many(operation, timestamps, bodies)

    @property
    def commit_timestamp(self):
        return self.engine.commit_timestamp


class ShardedStateMachine:
    """Collective create/lookup over every rank of a process group (one backend per rank)."""

    def __init__(self, backend, group=None):
        self.b = backend
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        assert backend.world == self.world
        self.comm_device = torch.device("cpu") if dist.get_backend(group) == "gloo" else backend.device
        self.commit_timestamp = 0
        self.passes_clean = 0
        self.passes_dirty = 0
        self.passes_split = 0
        self.demoted = 0  # routed events their homes demoted to the sequencer (split passes)

    # -- collectives helpers -----------------------------------------------------------------
    def _all_gather_i64(self, values):
        t = torch.tensor(values, dtype=torch.int64, device=self.comm_device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return np.stack([o.cpu().numpy() for o in out])

    def _a2a(self, send, send_counts, recv_counts):
        """all_to_all_single on rows; `send` rows grouped by destination rank.  Returns the received
        rows (grouped by source rank) on the backend device."""
        shape = tuple(send.shape[1:])
        out = torch.empty((int(sum(recv_counts)),) + shape, dtype=send.dtype, device=self.comm_device)
        src = send.to(self.comm_device)
        if self.comm_device.type == "cuda":
            _stream_sync(self.comm_device)
        dist.all_to_all_single(out, src.contiguous(), [int(c) for c in recv_counts], [int(c) for c in send_counts],
                               group=self.group)
        return out.to(self.b.device)

    def _bcast_np(self, arr, dtype):
        """Broadcast a numpy array (root 0) of `dtype`; returns it on every rank."""
        dtype = np.dtype(dtype)
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1) if self.rank == 0 else None
        size = torch.tensor([raw.size if raw is not None else 0], dtype=torch.int64, device=self.comm_device)
        dist.broadcast(size, 0, group=self.group)
        n = int(size.item())
        t = (torch.from_numpy(raw.copy()).to(self.comm_device) if self.rank == 0
             else torch.empty(n, dtype=torch.uint8, device=self.comm_device))
        if n:
            dist.broadcast(t, 0, group=self.group)
        return t.cpu().numpy().view(dtype)

    def _gather_np(self, arr, dtype):
        """Gather a numpy array from every rank to rank 0 (list by rank there, None elsewhere)."""
        dtype = np.dtype(dtype)
        raw = np.ascontiguousarray(arr, dtype=dtype).view(np.uint8).reshape(-1)
        sizes = self._all_gather_i64([raw.size])[:, 0]
        send_counts = [raw.size if r == 0 else 0 for r in range(self.world)]
        recv_counts = list(sizes) if self.rank == 0 else [0] * self.world
        out = self._a2a(torch.from_numpy(raw.copy()), send_counts, recv_counts).cpu().numpy()
        if self.rank != 0:
            return None
        parts, o = [], 0
        for s in sizes:
            parts.append(out[o:o + s].view(dtype))
            o += s
        return parts

    def _sum_balances(self, records):
        """Records identical on every rank but the balances: sum the balances over ranks (mod 2^128)."""
        n = len(records)
        if n == 0:
            return records
        limbs = np.zeros((n, 4, 4), dtype=np.int64)
        for f, name in enumerate(_BAL_FIELDS):
            lo = records[name + "_lo"].astype(np.uint64)
            hi = records[name + "_hi"].astype(np.uint64)
            limbs[:, f, 0] = (lo & 0xFFFFFFFF).astype(np.int64)
            limbs[:, f, 1] = (lo >> np.uint64(32)).astype(np.int64)
            limbs[:, f, 2] = (hi & 0xFFFFFFFF).astype(np.int64)
            limbs[:, f, 3] = (hi >> np.uint64(32)).astype(np.int64)
        t = torch.from_numpy(limbs).to(self.comm_device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        s = t.cpu().numpy()
        for k in range(3):  # carry propagation; the top limb wraps (mod 2^128)
            s[:, :, k + 1] += s[:, :, k] >> 32
            s[:, :, k] &= 0xFFFFFFFF
        s[:, :, 3] &= 0xFFFFFFFF
        out = records.copy()
        su = s.astype(np.uint64)
        for f, name in enumerate(_BAL_FIELDS):
            out[name + "_lo"] = su[:, f, 0] | (su[:, f, 1] << np.uint64(32))
            out[name + "_hi"] = su[:, f, 2] | (su[:, f, 3] << np.uint64(32))
        return out

    def _homes(self, ids):
        lib = _lib.load()
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(ids), dtype=np.uint32)
        if len(ids):
            lib.tbgpu_homes(ids.ctypes.data, len(ids), self.world, out.ctypes.data)
        return out

    def _finish(self, local_ts):
        t = torch.tensor([int(local_ts)], dtype=torch.int64, device=self.comm_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.commit_timestamp = max(self.commit_timestamp, int(t.item()))

    # -- commit ------------------------------------------------------------------------------
    def commit(self, operation, timestamps, lens, events):
        """Collective: commit this rank's prepares (batch k = lens[k] events at timestamps[k],
        back to back in `events`, a uint8 [n, 128] tensor on the backend device).  Returns a
        PassResult for this rank's prepares."""
        operation = Operation(int(operation))
        lens = [int(x) for x in lens]
        timestamps = [int(t) for t in timestamps]
        assert events.shape[0] == sum(lens) and len(lens) == len(timestamps)
        if operation == Operation.create_accounts:
            self._check_order(self._all_gather_i64(self._order_row(timestamps, lens)))
            return self._commit_replicated(operation, timestamps, lens, events)
        if operation != Operation.create_transfers:
            raise ValueError("commit: create operations only (use lookup_accounts / lookup_transfers)")
        # One all-gather carries the ordering check, every rank's plan and the home count matrix.
        plan, send_events, slots = self.b.plan(timestamps, lens, events)
        limbs = lambda v: [(v >> (32 * k)) & 0xFFFFFFFF for k in range(4)]  # noqa: E731
        g = self._all_gather_i64(self._order_row(timestamps, lens) + [plan.dirty] + limbs(plan.S) + limbs(plan.bound)
                                 + plan.counts)
        self._check_order(g[:, :4])
        dirty = int(np.bitwise_or.reduce(g[:, 4]))
        total = sum(int(g[r, 5 + k]) << (32 * (k % 4)) for r in range(self.world) for k in range(8))
        if total >= U128 - 1:  # a saturated S (maxInt) is a lower bound: no certificate
            self.passes_dirty += 1
            return self._commit_dirty(operation, timestamps, lens, events)
        if dirty:
            self.passes_split += 1
            return self._commit_split(timestamps, lens, events, _lib.CERT_U64 if total < U64 else _lib.CERT_U128)
        self.passes_clean += 1
        cert = _lib.CERT_U64 if total < U64 else _lib.CERT_U128
        return self._commit_routed(plan, send_events, slots, lens, g[:, 13 + self.rank], cert)

    def _order_row(self, timestamps, lens):
        prev = None
        for t, L in zip(timestamps, lens):
            if prev is not None and not (t - L + 1 > prev and t > prev):
                raise _lib.EnginePanic(_lib.STATUS_PANIC, "prepare timestamps not increasing")
            prev = t
        first = timestamps[0] - lens[0] + 1 if lens else 0
        return [len(lens), first, timestamps[-1] if lens else 0, int(self.b.commit_timestamp)]

    def _check_order(self, g):
        """g[r] = [prepares, first event timestamp, last prepare timestamp, engine commit ts]: the
        global order is rank-major and must start after the global commit timestamp
        (state_machine.zig:518-519, :645)."""
        self.commit_timestamp = max(self.commit_timestamp, int(g[:, 3].max()))
        last = self.commit_timestamp
        for r in range(self.world):
            if g[r, 0] == 0:
                continue
            if not (g[r, 1] > last and g[r, 2] > last):
                raise _lib.EnginePanic(_lib.STATUS_PANIC, "timestamp <= commit timestamp (rank %d)" % r)
            last = int(g[r, 2])
        self._pass_ts_max = last

    def sync_commit_timestamp(self):
        """Collective: the global commit_timestamp (max over every engine) after the last pass."""
        self._finish(self.b.commit_timestamp)
        return self.commit_timestamp

    def _commit_routed(self, plan, send_events, slots, lens, recv_counts, cert):
        """Clean pass: events to their homes (all-to-all #1), the home commits them, the legs of the
        committed transfers to the owners of their accounts (all-to-all #2, after a count exchange)
        where the balances live, and the result codes back to the sources (all-to-all #3)."""
        recv_events = self._a2a(send_events, plan.counts, recv_counts)
        codes, legs, leg_counts = self.b.commit_routed_owner(recv_events, self._pass_ts_max, cert, self.rank)
        legs_in_counts = self._a2a(torch.tensor(leg_counts, dtype=torch.int64), [1] * self.world, [1] * self.world)
        legs_in = self._a2a(legs, leg_counts, [int(x) for x in legs_in_counts.cpu().tolist()])
        self.b.apply_owner_legs(legs_in, cert)
        codes_back = self._a2a(codes, recv_counts, plan.counts)
        return self.b.replies(lens, slots, codes_back)

    def _owner_mask(self, records):
        """True for the accounts this rank owns (their balances live here)."""
        return self._homes(_ids(records["id_lo"], records["id_hi"])) == self.rank

    def _commit_replicated(self, operation, timestamps, lens, events):
        """create_accounts: every rank commits every prepare of the pass (records are replicated)."""
        meta = self._all_gather_i64([len(lens), events.shape[0]])
        ts_all = self._gather_all_np(np.asarray(timestamps, dtype=np.uint64), meta[:, 0])
        lens_all = self._gather_all_np(np.asarray(lens, dtype=np.uint64), meta[:, 0])
        n_max = int(meta[:, 1].max())
        padded = torch.zeros((max(n_max, 1), 128), dtype=torch.uint8, device=self.comm_device)
        padded[:events.shape[0]] = events.to(self.comm_device)
        parts = [torch.empty_like(padded) for _ in range(self.world)]
        dist.all_gather(parts, padded, group=self.group)
        bodies, stamps, own = [], [], None
        for r in range(self.world):
            ev = parts[r][:int(meta[r, 1])].cpu().numpy().reshape(-1)
            o = 0
            if r == self.rank:
                own = (len(bodies), len(bodies) + int(meta[r, 0]))
            for t, L in zip(ts_all[r], lens_all[r]):
                bodies.append(ev[o:o + int(L) * 128].tobytes())
                stamps.append(int(t))
                o += int(L) * 128
        replies = self.b.commit_batches(int(operation), stamps, bodies) if bodies else []
        self._finish(self.b.commit_timestamp)
        return PassResult.from_bytes(replies[own[0]:own[1]], lens, self.b.device)

    def _gather_all_np(self, arr, counts):
        """All-gather a 1-D uint64 array of per-rank length counts[r]."""
        m = max(int(counts.max()), 1)
        pad = np.zeros(m, dtype=np.int64)
        pad[:len(arr)] = arr.view(np.int64)
        g = self._all_gather_i64(list(pad))
        return [g[r, :int(counts[r])].view(np.uint64) for r in range(self.world)]

    # -- split dirty pass: clean events routed, the dependent subsequence sequenced --------------
    def _commit_split(self, timestamps, lens, events, cert):
        """A dirty pass under the global certificate.  Every rank classifies its events
        (tbgpu_route_dependents: chain members, post/void, balancing, limit-flag accounts, accounts
        a balancing event of the pass touches); the others are routed and committed by their homes
        exactly as in a clean pass, except that a home DEMOTES a routed event whose id a dependent
        event reads (its own id, or a post/void's pending id, sent to the home as probes), since its
        existence must follow the global order.  The dependent and demoted events — the pass's
        dependent subsequence — are committed by rank 0 in global order, runs of consecutive events
        of a prepare as sub-prepares with their original execute timestamps (chains never leave a
        run), with the referenced transfers and balances prefetched from their homes and owners
        (state_machine.zig:345-506).  Nothing a dependent event reads is written by a routed one:
        ids are demoted, constrained balances are only touched by dependent events, free balances
        feed no check under the certificate."""
        W, rank, dev = self.world, self.rank, self.b.device
        n = events.shape[0]
        # 1. accounts touched by balancing events anywhere in the pass (all-gather of their ids).
        fl = events[:, 118].to(torch.int32) | (events[:, 119].to(torch.int32) << 8) if n else \
            torch.zeros(0, dtype=torch.int32, device=dev)
        bal = (fl & 48) != 0
        mine = torch.cat([events[bal][:, 16:32], events[bal][:, 32:48]]).cpu().numpy().view(np.uint64).reshape(-1, 2) \
            if n else np.zeros((0, 2), dtype=np.uint64)
        sizes = self._all_gather_i64([len(mine)])[:, 0]
        marked = np.concatenate(self._gather_all_np(mine.reshape(-1), sizes * 2)).reshape(-1, 2) if sizes.sum() else \
            np.zeros((0, 2), dtype=np.uint64)
        if len(marked):
            marked = np.unique(marked, axis=0)
            marked = marked[np.lexsort((marked[:, 0], marked[:, 1]))]
        dep = self.b.dependents(lens, events, marked)
        depm = dep != 0
        # 2. the routed part: plan without the dependent events; counts for the all-to-alls.
        plan, send_events, slots = self.b.plan(timestamps, lens, events, skip=dep)
        counts = self._all_gather_i64(plan.counts)
        recv_counts = counts[:, rank]
        # 3. probes: the ids (and pending ids) dependent events read, to their homes.
        dev_ev = events[depm]
        pv = ((fl[depm] & 12) != 0) if n else fl
        keys = torch.cat([dev_ev[:, 0:16], dev_ev[pv][:, 64:80]]).contiguous().view(torch.int64).reshape(-1, 2)
        kh = self.b.homes(keys).to(torch.int64)
        order = torch.argsort(kh, stable=True)
        keys = keys[order]
        kcount = torch.bincount(kh, minlength=W).cpu().tolist() if keys.shape[0] else [0] * W
        kin = self._a2a(torch.tensor(kcount, dtype=torch.int64), [1] * W, [1] * W)
        probe_keys = self._a2a(keys, kcount, [int(x) for x in kin.cpu().tolist()])
        # 4. homes: demote, commit the rest, legs to the owners, codes back.
        recv = self._a2a(send_events, plan.counts, recv_counts)
        rid = recv[:, 0:16].contiguous().view(torch.int64).reshape(-1, 2)
        demote = torch.isin(_key64(rid), _key64(probe_keys)) if (rid.shape[0] and probe_keys.shape[0]) else \
            torch.zeros(rid.shape[0], dtype=torch.bool, device=dev)
        keep = ~demote
        codes_kept, legs, leg_counts = self.b.commit_routed_owner(recv[keep], self._pass_ts_max, cert, rank)
        legs_in_counts = self._a2a(torch.tensor(leg_counts, dtype=torch.int64), [1] * W, [1] * W)
        self.b.apply_owner_legs(self._a2a(legs, leg_counts, [int(x) for x in legs_in_counts.cpu().tolist()]), cert)
        codes = torch.full((rid.shape[0],), DEMOTED, dtype=torch.uint8, device=dev)
        codes[keep] = codes_kept.to(dev)
        codes_back = self._a2a(codes, recv_counts, plan.counts)
        # 5. dense codes at the source; the sequenced events: dependent ones and demoted ones.
        sl = slots.to(torch.int64)
        dense = torch.full((n,), 3, dtype=torch.uint8, device=dev)  # SLOT_LOCAL: timestamp_must_be_zero
        routed = sl >= 0
        dense[routed] = codes_back.to(dev)[sl[routed]] if codes_back.shape[0] else dense[routed]
        demoted = routed & (dense == DEMOTED)
        self.demoted += int(demoted.sum().item())
        seq = depm | demoted
        seq_idx = torch.nonzero(seq).reshape(-1)
        # 6. the sequencer: every rank's sequenced events to rank 0, in global order.
        seq_codes = self._sequence(timestamps, lens, events, seq_idx)
        if seq_idx.shape[0]:
            dense[seq_idx] = seq_codes.to(dev)
        ident = torch.arange(max(n, 1), dtype=torch.int32, device=dev)[:n]
        return self.b.replies(lens, ident, dense)

    def _sequence(self, timestamps, lens, events, seq_idx):
        """Commit the sequenced events of every rank on rank 0 (scratch engine, prefetch / write-back
        as in _commit_dirty); returns this rank's codes for its seq_idx events."""
        W, root = self.world, self.rank == 0
        starts = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)])
        pos = seq_idx.cpu().numpy().astype(np.int64)
        k = np.searchsorted(starts, pos, side="right") - 1  # prepare of each sequenced event
        ts = np.asarray(timestamps, dtype=np.int64)
        Ls = np.asarray(lens, dtype=np.int64)
        ets = (ts[k] - Ls[k] + 1 + (pos - starts[k])) if len(pos) else np.zeros(0, dtype=np.int64)  # execute ts (:645)
        # Runs of consecutive events of one prepare become sub-prepares (chains stay whole).
        brk = np.ones(len(pos), dtype=bool)
        if len(pos) > 1:
            brk[1:] = (k[1:] != k[:-1]) | (pos[1:] != pos[:-1] + 1)
        meta = np.stack([brk.astype(np.int64), ets], axis=1).reshape(-1)
        recs = events[seq_idx].cpu().numpy() if len(pos) else np.zeros((0, 128), dtype=np.uint8)
        meta_parts = self._gather_np(meta, np.int64)
        rec_parts = self._gather_np(recs.reshape(-1), np.uint8)
        counts = self._all_gather_i64([len(pos)])[:, 0]
        if root:
            allm = np.concatenate(meta_parts).reshape(-1, 2) if counts.sum() else np.zeros((0, 2), dtype=np.int64)
            allr = np.concatenate(rec_parts).reshape(-1, 128) if counts.sum() else np.zeros((0, 128), dtype=np.uint8)
            # A run also breaks between ranks (a rank's first event starts a sub-prepare).
            firsts = np.concatenate([[0], np.cumsum(counts)[:-1]])
            for f, c in zip(firsts, counts):
                if c:
                    allm[f, 0] = 1
            run_start = np.nonzero(allm[:, 0])[0] if len(allm) else np.zeros(0, dtype=np.int64)
            run_end = np.concatenate([run_start[1:], [len(allm)]]) if len(run_start) else run_start
            bodies = [allr[a:b].tobytes() for a, b in zip(run_start, run_end)]
            stamps = [int(allm[b - 1, 1]) for b in run_end]
            ev = allr.reshape(-1).view(TRANSFER_DTYPE) if len(allr) else np.zeros(0, dtype=TRANSFER_DTYPE)
            codes = np.zeros(len(allm), dtype=np.uint8)
        else:
            ev, bodies, stamps = None, None, None
        replies = self._scratch_commit(ev, bodies, stamps)
        if root:
            for (a, _b), r in zip(zip(run_start, run_end), replies):
                p = np.frombuffer(r, dtype=np.uint32).reshape(-1, 2)
                codes[a + p[:, 0].astype(np.int64)] = p[:, 1]
        # Codes back to their ranks (rank r's events are rank r's slice, in order).
        send_counts = [int(c) for c in counts] if root else [0] * W
        out = self._a2a(torch.from_numpy(codes if root else np.zeros(0, dtype=np.uint8)), send_counts,
                        [int(counts[self.rank]) if r == 0 else 0 for r in range(W)])
        return out

    def _scratch_commit(self, ev, bodies, stamps):
        """Collective: rank 0 commits `bodies` (prepares at `stamps`) on a scratch engine loaded with
        the transfers and accounts they read, then writes the effects back to their homes and
        owners.  Returns the replies on rank 0 (None elsewhere)."""
        W, root = self.world, self.rank == 0
        if root:
            pv = (ev["flags"] & (TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)) != 0
            tids = _unique_ids(np.concatenate([_ids(ev["id_lo"], ev["id_hi"]),
                                               _ids(ev["pending_id_lo"][pv], ev["pending_id_hi"][pv])]))
        tids = self._bcast_np(tids if root else None, np.uint64).reshape(-1, 2)
        homes = self._homes(tids)
        mine = np.nonzero(homes == self.rank)[0]
        recs, state = self.b.fetch_transfers(tids[mine])
        recs_parts = self._gather_np(recs, TRANSFER_DTYPE)
        state_parts = self._gather_np(state, np.uint8)
        if root:
            fetched = np.zeros(len(tids), dtype=TRANSFER_DTYPE)
            fstate = np.zeros(len(tids), dtype=np.uint8)
            for r in range(W):
                idx = np.nonzero(homes == r)[0]
                fetched[idx] = recs_parts[r]
                fstate[idx] = state_parts[r]
            present = fstate != 0
            aids = _unique_ids(np.concatenate([
                _ids(ev["debit_account_id_lo"], ev["debit_account_id_hi"]),
                _ids(ev["credit_account_id_lo"], ev["credit_account_id_hi"]),
                _ids(fetched["debit_account_id_lo"][present], fetched["debit_account_id_hi"][present]),
                _ids(fetched["credit_account_id_lo"][present], fetched["credit_account_id_hi"][present])]))
        aids = self._bcast_np(aids if root else None, np.uint64).reshape(-1, 2)
        accts, afound = self.b.fetch_accounts(aids)
        accts = self._sum_balances(accts)
        afound = afound.astype(bool)
        replies = None
        if root:
            scratch = self.b.scratch(int(afound.sum()) + 1, int(present.sum()) + len(ev) + 1)
            scratch.upsert_accounts(accts[afound])
            scratch.upsert_transfers(fetched[present], fstate[present])
            replies = scratch.commit_batches(int(Operation.create_transfers), stamps, bodies) if bodies else []
            after, astate = scratch.fetch_transfers(tids)
            changed = (astate != 0) & (astate != fstate)
            wb_t, wb_s = after[changed], astate[changed]
            acc_after, _ = scratch.fetch_accounts(aids[afound])
            local_ts = scratch.commit_timestamp
        else:
            local_ts = 0
        wb_t = self._bcast_np(wb_t if root else None, TRANSFER_DTYPE)
        wb_s = self._bcast_np(wb_s if root else None, np.uint8)
        if len(wb_t):
            h = self._homes(_ids(wb_t["id_lo"], wb_t["id_hi"]))
            sel = h == self.rank
            self.b.upsert_transfers(wb_t[sel], wb_s[sel])
        acc_after = self._bcast_np(acc_after if root else None, ACCOUNT_DTYPE)
        wb_a = acc_after.copy()
        not_mine = ~self._owner_mask(wb_a)
        for name in _BAL_FIELDS:
            wb_a[name + "_lo"][not_mine] = 0
            wb_a[name + "_hi"][not_mine] = 0
        self.b.upsert_accounts(wb_a)
        self._finish(local_ts)
        return replies

    # -- dirty pass: prefetch on rank 0, commit on a scratch engine, write back -----------------
    def _commit_dirty(self, operation, timestamps, lens, events):
        W, root = self.world, self.rank == 0
        meta = self._all_gather_i64([len(lens), events.shape[0]])
        ts_all = self._gather_all_np(np.asarray(timestamps, dtype=np.uint64), meta[:, 0])
        lens_all = self._gather_all_np(np.asarray(lens, dtype=np.uint64), meta[:, 0])
        send_counts = [events.shape[0] if r == 0 else 0 for r in range(W)]
        recv_counts = list(meta[:, 1]) if root else [0] * W
        gathered = self._a2a(events, send_counts, recv_counts)

        # 1. transfers the pass reads: every event id, and the pending id of post/void events.
        if root:
            ev = _events_np(gathered)
            pv = (ev["flags"] & (TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)) != 0
            tids = _unique_ids(np.concatenate([_ids(ev["id_lo"], ev["id_hi"]),
                                               _ids(ev["pending_id_lo"][pv], ev["pending_id_hi"][pv])]))
        tids = self._bcast_np(tids if root else None, np.uint64).reshape(-1, 2)
        homes = self._homes(tids)
        mine = np.nonzero(homes == self.rank)[0]
        recs, state = self.b.fetch_transfers(tids[mine])
        recs_parts = self._gather_np(recs, TRANSFER_DTYPE)
        state_parts = self._gather_np(state, np.uint8)
        if root:
            fetched = np.zeros(len(tids), dtype=TRANSFER_DTYPE)
            fstate = np.zeros(len(tids), dtype=np.uint8)
            for r in range(W):
                idx = np.nonzero(homes == r)[0]
                fetched[idx] = recs_parts[r]
                fstate[idx] = state_parts[r]
            present = fstate != 0
            aids = _unique_ids(np.concatenate([
                _ids(ev["debit_account_id_lo"], ev["debit_account_id_hi"]),
                _ids(ev["credit_account_id_lo"], ev["credit_account_id_hi"]),
                _ids(fetched["debit_account_id_lo"][present], fetched["debit_account_id_hi"][present]),
                _ids(fetched["credit_account_id_lo"][present], fetched["credit_account_id_hi"][present])]))

        # 2. the touched accounts with their true (summed) balances.
        aids = self._bcast_np(aids if root else None, np.uint64).reshape(-1, 2)
        accts, afound = self.b.fetch_accounts(aids)
        accts = self._sum_balances(accts)
        afound = afound.astype(bool)

        # 3. rank 0 commits the pass on the scratch engine.
        if root:
            scratch = self.b.scratch(int(afound.sum()) + 1, int(present.sum()) + len(ev) + 1)
            scratch.upsert_accounts(accts[afound])
            scratch.upsert_transfers(fetched[present], fstate[present])
            bodies, stamps, o = [], [], 0
            evb = gathered.cpu().numpy().reshape(-1)
            for r in range(W):
                for t, L in zip(ts_all[r], lens_all[r]):
                    bodies.append(evb[o:o + int(L) * 128].tobytes())
                    stamps.append(int(t))
                    o += int(L) * 128
            replies = scratch.commit_batches(int(operation), stamps, bodies)
            after, astate = scratch.fetch_transfers(tids)
            changed = (astate != 0) & (astate != fstate)
            wb_t, wb_s = after[changed], astate[changed]
            acc_after, _ = scratch.fetch_accounts(aids[afound])
            local_ts = scratch.commit_timestamp
            rlens = np.asarray([len(r) for r in replies], dtype=np.int64)
            rbytes = np.frombuffer(b"".join(replies), dtype=np.uint8)
        else:
            local_ts = 0

        # 4. write back: new transfers and posted states to their homes, each touched account's
        #    balances to its owner (every other rank holds zeros for it).
        wb_t = self._bcast_np(wb_t if root else None, TRANSFER_DTYPE)
        wb_s = self._bcast_np(wb_s if root else None, np.uint8)
        if len(wb_t):
            h = self._homes(_ids(wb_t["id_lo"], wb_t["id_hi"]))
            sel = h == self.rank
            self.b.upsert_transfers(wb_t[sel], wb_s[sel])
        acc_after = self._bcast_np(acc_after if root else None, ACCOUNT_DTYPE)
        wb_a = acc_after.copy()
        not_mine = ~self._owner_mask(wb_a)
        for name in _BAL_FIELDS:
            wb_a[name + "_lo"][not_mine] = 0
            wb_a[name + "_hi"][not_mine] = 0
        self.b.upsert_accounts(wb_a)

        # 5. replies back to their ranks.
        rlens = self._bcast_np(rlens if root else None, np.int64)
        rbytes = self._bcast_np(rbytes if root else None, np.uint8)
        first = int(meta[:self.rank, 0].sum())
        offs = np.concatenate([[0], np.cumsum(rlens)])
        mine_r = [rbytes[offs[k]:offs[k + 1]].tobytes() for k in range(first, first + len(lens))]
        self._finish(local_ts)
        return PassResult.from_bytes(mine_r, lens, self.b.device)

    def test_set_balances(self, account_id, dp, dpost, cp, cpost):
        """Collective test-only `setup` action (state_machine.zig:1398-1407): the owner holds the
        balances, every other rank zeros."""
        ids = np.array([[account_id & U64_MAX, account_id >> 64]], dtype=np.uint64)
        recs, found = self.b.fetch_accounts(ids)
        if not found[0]:
            raise _lib.EnginePanic(_lib.STATUS_PANIC, "setup of a missing account")
        mine = bool(self._owner_mask(recs)[0])
        for name, v in zip(_BAL_FIELDS, (dp, dpost, cp, cpost)):
            v = v if mine else 0
            recs[name + "_lo"] = v & U64_MAX
            recs[name + "_hi"] = v >> 64
        self.b.upsert_accounts(recs)

    # -- lookups (execute_lookup_accounts / _transfers, state_machine.zig:700-736) -------------
    def lookup_accounts(self, ids):
        """Collective: found accounts in input order, with the summed balances."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        recs, found = self.b.fetch_accounts(ids)
        recs = self._sum_balances(recs)
        return recs[found.astype(bool)]

    def lookup_transfers(self, ids):
        """Collective: found transfers in input order (each lives on exactly one home)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        homes = self._homes(ids)
        recs = np.zeros(len(ids), dtype=TRANSFER_DTYPE)
        mine = np.nonzero(homes == self.rank)[0]
        r, st = self.b.fetch_transfers(ids[mine])
        found = np.zeros(len(ids), dtype=np.int64)
        recs[mine] = r
        found[mine] = st != 0
        words = torch.from_numpy(recs.view(np.int64).reshape(-1).copy()).to(self.comm_device)
        f = torch.from_numpy(found).to(self.comm_device)
        dist.all_reduce(words, op=dist.ReduceOp.SUM, group=self.group)  # one non-zero term per id
        dist.all_reduce(f, op=dist.ReduceOp.SUM, group=self.group)
        out = words.cpu().numpy().view(TRANSFER_DTYPE)
        return out[f.cpu().numpy() != 0]

    # -- parity read-back ------------------------------------------------------------------------
    def export_accounts(self):
        """Collective: every account (sorted by id) with summed balances."""
        return self._sum_balances(self.b.export_accounts())

    def export_transfers(self):
        """Collective: rank 0 receives every transfer sorted by id (None elsewhere)."""
        parts = self._gather_np(self.b.export_transfers(), TRANSFER_DTYPE)
        if parts is None:
            return None
        t = np.concatenate(parts)
        order = np.lexsort((t["id_lo"], t["id_hi"]))
        return t[order]

    def export_posted(self):
        """Collective: rank 0 receives the posted groove {pending timestamp, fulfillment}, sorted."""
        parts = self._gather_np(np.ascontiguousarray(self.b.export_posted(), dtype=np.uint64).reshape(-1), np.uint64)
        if parts is None:
            return None
        p = np.concatenate(parts).reshape(-1, 2)
        return p[np.lexsort((p[:, 1], p[:, 0]))]
