"""CPU test double of one rank's multi-GPU backend (tigerbeetle_amd.sharded.GpuShard) — TEST
INFRASTRUCTURE ONLY.

It implements the same per-rank primitives (include/tbgpu_shard.h) over the CPU oracle, with the
routing kernels (tb_route_classify / _scatter / _replies, k_route.h) restated in numpy, so the
collective protocol of ShardedStateMachine — clean routed passes, the dirty-pass prefetch /
scratch commit / write-back, lookups and exports — runs with gloo on CPU at world_size 2.  The
GPU backend itself is covered by tests/test_gpu_sharded.py.
"""
import numpy as np
import torch

from tigerbeetle_amd import _lib
from tigerbeetle_amd.sharded import _ROUTED_NEVER, PassResult, RoutePlan
from tigerbeetle_amd.types import TRANSFER_DTYPE, U128_MAX, AccountFlags

from .oracle import OracleEngine

U64_MASK = (1 << 64) - 1
_LIMITS = int(AccountFlags.debits_must_not_exceed_credits | AccountFlags.credits_must_not_exceed_debits)


def homes_of(ids, world):
    lib = _lib.load()
    ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
    out = np.zeros(len(ids), dtype=np.uint32)
    if len(ids):
        lib.tbgpu_homes(ids.ctypes.data, len(ids), world, out.ctypes.data)
    return out


class OracleShard:
    def __init__(self, world):
        self.world = world
        self.device = torch.device("cpu")
        self.o = OracleEngine(1 << 12, 1 << 14)

    def dependents(self, lens, events, marked):
        """tb_route_dependents restated: 1 chain member, 2 post/void, 4 balancing, 8 limit-flag
        account, 16 an account a balancing event of the pass touches."""
        ev = events.numpy().reshape(-1).view(TRANSFER_DTYPE)
        n = len(ev)
        dep = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return torch.from_numpy(dep)
        fl = ev["flags"].astype(np.int64)
        linked = (fl & 1) != 0
        first = np.zeros(n, dtype=bool)
        first[np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)] = True
        prev_linked = np.zeros(n, dtype=bool)
        prev_linked[1:] = linked[:-1]
        prev_linked &= ~first
        dep |= np.where(linked | prev_linked, 1, 0).astype(np.uint8)
        dep |= np.where((fl & 12) != 0, 2, 0).astype(np.uint8)
        dep |= np.where((fl & 48) != 0, 4, 0).astype(np.uint8)
        mk = {(int(lo), int(hi)) for lo, hi in np.asarray(marked, dtype=np.uint64).reshape(-1, 2)}
        for side in ("debit_account_id", "credit_account_id"):
            ids = np.stack([ev[side + "_lo"], ev[side + "_hi"]], axis=1)
            recs, found = self.o.fetch_accounts(ids)
            lim = ((recs["flags"] & _LIMITS) != 0) & found.astype(bool)
            dep |= np.where(lim, 8, 0).astype(np.uint8)
            if mk:
                hit = np.array([(int(a), int(b)) in mk for a, b in ids], dtype=bool)
                dep |= np.where(hit, 16, 0).astype(np.uint8)
        return torch.from_numpy(dep)

    def homes(self, ids):
        return torch.from_numpy(homes_of(ids.numpy().view(np.uint64).reshape(-1, 2), self.world).astype(np.uint8))

    def plan(self, timestamps, lens, events, skip=None):
        ev = events.numpy().reshape(-1).view(TRANSFER_DTYPE)
        n = len(ev)
        homes = homes_of(np.stack([ev["id_lo"], ev["id_hi"]], axis=1), self.world)
        dirty = 0
        if n:
            if np.any(ev["flags"] & _ROUTED_NEVER):
                dirty |= _lib.DIRTY_FLAGS
            clean = (ev["flags"] & _ROUTED_NEVER) == 0
            for side in ("debit_account_id", "credit_account_id"):
                ids = np.stack([ev[side + "_lo"][clean], ev[side + "_hi"][clean]], axis=1)
                recs, found = self.o.fetch_accounts(ids)
                if np.any(((recs["flags"] & _LIMITS) != 0) & found.astype(bool)):
                    dirty |= _lib.DIRTY_LIMIT
        ts = np.zeros(n, dtype=np.uint64)
        o = 0
        for t, L in zip(timestamps, lens):
            ts[o:o + L] = int(t) - L + 1 + np.arange(L, dtype=np.uint64)
            o += L
        skipped = skip.numpy().astype(bool) if skip is not None else np.zeros(n, dtype=bool)
        local = (ev["timestamp"] != 0) & ~skipped  # timestamp_must_be_zero: answered here, never routed
        homes = np.where(local | skipped, self.world, homes)
        order = np.argsort(homes, kind="stable")
        slots = np.empty(n, dtype=np.int64)
        slots[order] = np.arange(n)
        slots[local] = -1
        slots[skipped] = -2  # SLOT_DEP: the sequencer commits it
        routed = ev.copy()
        routed["timestamp"] = ts
        counts = np.bincount(homes[~(local | skipped)], minlength=self.world).tolist() if n else [0] * self.world
        S = 0
        for lo, hi in zip(ev["amount_lo"][~local], ev["amount_hi"][~local]):
            S = min(S + ((int(hi) << 64) | int(lo)), U128_MAX)
        plan = RoutePlan(counts, S, self.o.balance_bound(), dirty)
        send = torch.from_numpy(routed.view(np.uint8).reshape(-1, 128)[order[:sum(counts)]].copy())
        return plan, send, torch.from_numpy(slots)

    def commit_routed(self, events, ts_max, cert):
        del ts_max, cert
        return torch.from_numpy(self.o.commit_routed(events.numpy()).copy())

    def commit_routed_owner(self, events, ts_max, cert, rank):
        """Routed commit with owner-partitioned balances (tbgpu_commit_routed_owner_async): the
        oracle applies every committed transfer locally; each leg owned elsewhere is cancelled here
        and sent to its owner (the GPU also sends self-owned legs of independent events to itself;
        the final balances are the same)."""
        codes = self.commit_routed(events, ts_max, cert)
        ev = events.numpy().reshape(-1).view(TRANSFER_DTYPE)
        ok = codes.numpy() == 0
        per_owner = [[] for _ in range(self.world)]
        for t in ev[ok]:
            amount = (int(t["amount_hi"]) << 64) | int(t["amount_lo"])
            pend = int(t["flags"]) & 2
            for side, field in (("debit_account_id", 0 if pend else 1), ("credit_account_id", 2 if pend else 3)):
                lo, hi = int(t[side + "_lo"]), int(t[side + "_hi"])
                owner = int(homes_of(np.array([[lo, hi]], dtype=np.uint64), self.world)[0])
                if owner == rank:
                    continue
                self._add_balance(lo, hi, field, (1 << 128) - amount)
                per_owner[owner].append([lo, hi, amount & U64_MASK, amount >> 64, field])
        counts = [len(p) for p in per_owner]
        rows = [r for p in per_owner for r in p]
        legs = np.array(rows, dtype=np.uint64).reshape(-1, 5).view(np.int64)
        return codes, torch.from_numpy(legs.copy()), counts

    def _add_balance(self, lo, hi, field, delta):
        names = ("debits_pending", "debits_posted", "credits_pending", "credits_posted")
        recs, found = self.o.fetch_accounts(np.array([[lo, hi]], dtype=np.uint64))
        assert found[0], "leg for a missing account"
        name = names[field]
        v = ((int(recs[name + "_hi"][0]) << 64) | int(recs[name + "_lo"][0])) + delta
        v &= (1 << 128) - 1
        recs[name + "_lo"] = v & U64_MASK
        recs[name + "_hi"] = v >> 64
        self.o.upsert_accounts(recs)

    def apply_owner_legs(self, legs, cert):
        del cert
        for w in legs.numpy().view(np.uint64).reshape(-1, 5):
            self._add_balance(int(w[0]), int(w[1]), int(w[4]), (int(w[3]) << 64) | int(w[2]))

    def replies(self, lens, slots, codes_back):
        s = slots.numpy()
        cb = codes_back.numpy()
        codes = np.where(s < 0, 3, cb[np.maximum(s, 0)] if len(cb) else 0).astype(np.uint8) if len(s) \
            else np.zeros(0, dtype=np.uint8)
        out, o = [], 0
        for L in lens:
            c = codes[o:o + L]
            nz = np.nonzero(c)[0]
            pairs = np.stack([nz.astype(np.uint32), c[nz].astype(np.uint32)], axis=1)
            out.append(pairs.tobytes())
            o += L
        return PassResult.from_bytes(out, lens, self.device)

    def commit_batches(self, operation, timestamps, bodies):
        return self.o.commit_many(operation, timestamps, bodies)

    def fetch_accounts(self, ids):
        return self.o.fetch_accounts(ids)

    def fetch_transfers(self, ids):
        return self.o.fetch_transfers(ids)

    def upsert_accounts(self, records):
        self.o.upsert_accounts(records)

    def upsert_transfers(self, records, state):
        self.o.upsert_transfers(records, state)

    @property
    def commit_timestamp(self):
        return self.o.commit_timestamp

    def export_accounts(self):
        return self.o.export_accounts()

    def export_transfers(self):
        return self.o.export_transfers()

    def export_posted(self):
        return self.o.export_posted()

    def scratch(self, accounts, transfers):
        return OracleEngine(accounts, transfers)
