"""ctypes adapter for the CPU oracle (oracle/liboracle.so) — test infrastructure only."""
import ctypes
import os
import subprocess

import numpy as np

from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE, U64_MAX

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

STATUS_OK, STATUS_INVALID, STATUS_PANIC = 0, 1, 2


class OraclePanic(RuntimeError):
    """The reference would have panicked (ReleaseSafe trap / assert)."""


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        L = ctypes.CDLL(ORACLE_SO)
        c = ctypes
        L.tbo_init.restype = c.c_void_p
        L.tbo_init.argtypes = [c.c_uint64, c.c_uint64]
        L.tbo_deinit.argtypes = [c.c_void_p]
        L.tbo_reset.argtypes = [c.c_void_p]
        L.tbo_commit.restype = c.c_int
        L.tbo_commit.argtypes = [c.c_void_p, c.c_uint8, c.c_uint64, c.c_void_p, c.c_uint32,
                                 c.c_void_p, c.c_uint32, c.POINTER(c.c_uint32)]
        L.tbo_set_balances.restype = c.c_int
        L.tbo_set_balances.argtypes = [c.c_void_p, c.c_uint64, c.c_uint64, c.POINTER(c.c_uint64)]
        for name in ("tbo_commit_timestamp", "tbo_account_count", "tbo_transfer_count"):
            getattr(L, name).restype = c.c_uint64
            getattr(L, name).argtypes = [c.c_void_p]
        for name in ("tbo_export_accounts", "tbo_export_transfers"):
            getattr(L, name).restype = c.c_uint64
            getattr(L, name).argtypes = [c.c_void_p, c.c_void_p, c.c_uint64]
        L.tbo_export_posted.restype = c.c_uint64
        L.tbo_export_posted.argtypes = [c.c_void_p, c.c_void_p, c.c_uint64]
        L.tbo_commit_routed.restype = c.c_int
        L.tbo_commit_routed.argtypes = [c.c_void_p, c.c_uint64, c.c_void_p, c.c_void_p]
        for name in ("tbo_fetch_accounts", "tbo_fetch_transfers"):
            getattr(L, name).restype = c.c_int
            getattr(L, name).argtypes = [c.c_void_p, c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p]
        L.tbo_upsert_accounts.restype = c.c_int
        L.tbo_upsert_accounts.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32]
        L.tbo_upsert_transfers.restype = c.c_int
        L.tbo_upsert_transfers.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32]
        L.tbo_balance_bound.restype = None
        L.tbo_balance_bound.argtypes = [c.c_void_p, c.c_void_p]
        L.tbo_sum_overflows_u64.restype = c.c_int
        L.tbo_sum_overflows_u64.argtypes = [c.c_uint64, c.c_uint64]
        L.tbo_sum_overflows_u128.restype = c.c_int
        L.tbo_sum_overflows_u128.argtypes = [c.c_uint64] * 4
        _lib = L
    return _lib


def _split_balances(values):
    arr = (ctypes.c_uint64 * 8)()
    for i, v in enumerate(values):
        arr[2 * i] = v & U64_MAX
        arr[2 * i + 1] = v >> 64
    return arr


class OracleEngine:
    """The CPU restatement behind the same engine interface the GPU engine offers."""

    def __init__(self, accounts_hint=1024, transfers_hint=1024):
        self.L = lib()
        self.h = self.L.tbo_init(accounts_hint, transfers_hint)

    def close(self):
        if self.h:
            self.L.tbo_deinit(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def reset(self):
        self.L.tbo_reset(self.h)

    def commit_raw(self, operation, timestamp, body, out_cap=None):
        body = bytes(body)
        if out_cap is None:
            out_cap = max(len(body) // 128 * 8, len(body) // 16 * 128, 8)
        out = ctypes.create_string_buffer(out_cap)
        n = ctypes.c_uint32(0)
        src = ctypes.create_string_buffer(body, len(body)) if body else None
        st = self.L.tbo_commit(self.h, operation, timestamp, src, len(body), out, out_cap, ctypes.byref(n))
        return st, out.raw[:n.value]

    def commit(self, operation, timestamp, body):
        st, reply = self.commit_raw(operation, timestamp, body)
        if st == STATUS_PANIC:
            raise OraclePanic("oracle panic (reference would trap)")
        if st != STATUS_OK:
            raise RuntimeError("oracle commit status %d" % st)
        return reply

    def set_balances(self, account_id, dp, dpost, cp, cpost):
        st = self.L.tbo_set_balances(self.h, account_id & U64_MAX, account_id >> 64,
                                     _split_balances([dp, dpost, cp, cpost]))
        if st != STATUS_OK:
            raise OraclePanic("setup of a missing account")

    @property
    def commit_timestamp(self):
        return self.L.tbo_commit_timestamp(self.h)

    def export_accounts(self):
        n = self.L.tbo_account_count(self.h)
        out = np.zeros(n, dtype=ACCOUNT_DTYPE)
        m = self.L.tbo_export_accounts(self.h, out.ctypes.data, n)
        return out[:m]

    def export_transfers(self):
        n = self.L.tbo_transfer_count(self.h)
        out = np.zeros(n, dtype=TRANSFER_DTYPE)
        m = self.L.tbo_export_transfers(self.h, out.ctypes.data, n)
        return out[:m]

    def export_posted(self):
        n = self.L.tbo_transfer_count(self.h)
        out = np.zeros((max(n, 1), 2), dtype=np.uint64)
        m = self.L.tbo_export_posted(self.h, out.ctypes.data, n)
        return out[:m]

    # -- shard test double primitives (tbo_* restatements of include/tbgpu_shard.h) -----------
    def commit_routed(self, events):
        events = np.ascontiguousarray(events, dtype=np.uint8).reshape(-1)
        n = events.size // 128
        codes = np.zeros(max(n, 1), dtype=np.uint8)
        st = self.L.tbo_commit_routed(self.h, n, events.ctypes.data, codes.ctypes.data)
        if st == STATUS_PANIC:
            raise OraclePanic("oracle panic in a routed commit")
        if st != STATUS_OK:
            raise RuntimeError("routed commit status %d" % st)
        return codes[:n]

    def fetch_accounts(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(ids), dtype=ACCOUNT_DTYPE)
        found = np.zeros(len(ids), dtype=np.uint8)
        if len(ids):
            self.L.tbo_fetch_accounts(self.h, ids.ctypes.data, len(ids), out.ctypes.data, found.ctypes.data)
        return out, found

    def fetch_transfers(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1, 2)
        out = np.zeros(len(ids), dtype=TRANSFER_DTYPE)
        state = np.zeros(len(ids), dtype=np.uint8)
        if len(ids):
            self.L.tbo_fetch_transfers(self.h, ids.ctypes.data, len(ids), out.ctypes.data, state.ctypes.data)
        return out, state

    def upsert_accounts(self, records):
        records = np.ascontiguousarray(records, dtype=ACCOUNT_DTYPE)
        if len(records) and self.L.tbo_upsert_accounts(self.h, records.ctypes.data, len(records)) != STATUS_OK:
            raise OraclePanic("upsert_accounts")

    def upsert_transfers(self, records, state):
        records = np.ascontiguousarray(records, dtype=TRANSFER_DTYPE)
        state = np.ascontiguousarray(state, dtype=np.uint8)
        if len(records) and self.L.tbo_upsert_transfers(self.h, records.ctypes.data, state.ctypes.data,
                                                        len(records)) != STATUS_OK:
            raise OraclePanic("upsert_transfers")

    def balance_bound(self):
        out = (ctypes.c_uint64 * 2)()
        self.L.tbo_balance_bound(self.h, out)
        return (out[1] << 64) | out[0]

    def commit_many(self, operation, timestamps, bodies):
        return [self.commit(operation, t, b) for t, b in zip(timestamps, bodies)]

    commit_batches = commit_many
