"""Account / Transfer layouts, flags, operations and result codes.

Mirrors src/tigerbeetle.zig:7-249 and src/state_machine.zig:208-214 of the reference (and the C
header src/clients/c/tb_client.h:17-165).  u128 fields are stored little-endian as two u64 words
(`<name>_lo`, `<name>_hi`); the structured dtypes below are byte-identical to the 128-byte extern
structs.
"""
import enum
import struct

import numpy as np

U128_MAX = (1 << 128) - 1
U64_MAX = (1 << 64) - 1

# Operation (state_machine.zig:208-214; vsr_operations_reserved = 128, constants.zig:38).
class Operation(enum.IntEnum):
    create_accounts = 128
    create_transfers = 129
    lookup_accounts = 130
    lookup_transfers = 131


# batch_max (state_machine.zig:46-65) for the production config: message_body_size_max =
# 1 MiB - 128 B header (config.zig:137, vsr.zig:401, constants.zig:167-168).
MESSAGE_BODY_SIZE_MAX = (1 << 20) - 128
BATCH_MAX = MESSAGE_BODY_SIZE_MAX // 128  # 8191


class AccountFlags(enum.IntFlag):
    linked = 1 << 0
    debits_must_not_exceed_credits = 1 << 1
    credits_must_not_exceed_debits = 1 << 2


class TransferFlags(enum.IntFlag):
    linked = 1 << 0
    pending = 1 << 1
    post_pending_transfer = 1 << 2
    void_pending_transfer = 1 << 3
    balancing_debit = 1 << 4
    balancing_credit = 1 << 5


# Values == declaration index (asserted at tigerbeetle.zig:139-143, :224-228).
CreateAccountResult = enum.IntEnum("CreateAccountResult", [(n, i) for i, n in enumerate("""
ok linked_event_failed linked_event_chain_open timestamp_must_be_zero reserved_field reserved_flag
id_must_not_be_zero id_must_not_be_int_max flags_are_mutually_exclusive debits_pending_must_be_zero
debits_posted_must_be_zero credits_pending_must_be_zero credits_posted_must_be_zero
ledger_must_not_be_zero code_must_not_be_zero exists_with_different_flags
exists_with_different_user_data_128 exists_with_different_user_data_64
exists_with_different_user_data_32 exists_with_different_ledger exists_with_different_code exists
""".split())])

CreateTransferResult = enum.IntEnum("CreateTransferResult", [(n, i) for i, n in enumerate("""
ok linked_event_failed linked_event_chain_open timestamp_must_be_zero reserved_flag
id_must_not_be_zero id_must_not_be_int_max flags_are_mutually_exclusive
debit_account_id_must_not_be_zero debit_account_id_must_not_be_int_max
credit_account_id_must_not_be_zero credit_account_id_must_not_be_int_max accounts_must_be_different
pending_id_must_be_zero pending_id_must_not_be_zero pending_id_must_not_be_int_max
pending_id_must_be_different timeout_reserved_for_pending_transfer amount_must_not_be_zero
ledger_must_not_be_zero code_must_not_be_zero debit_account_not_found credit_account_not_found
accounts_must_have_the_same_ledger transfer_must_have_the_same_ledger_as_accounts
pending_transfer_not_found pending_transfer_not_pending
pending_transfer_has_different_debit_account_id pending_transfer_has_different_credit_account_id
pending_transfer_has_different_ledger pending_transfer_has_different_code
exceeds_pending_transfer_amount pending_transfer_has_different_amount
pending_transfer_already_posted pending_transfer_already_voided pending_transfer_expired
exists_with_different_flags exists_with_different_debit_account_id
exists_with_different_credit_account_id exists_with_different_amount
exists_with_different_pending_id exists_with_different_user_data_128
exists_with_different_user_data_64 exists_with_different_user_data_32
exists_with_different_timeout exists_with_different_code exists overflows_debits_pending
overflows_credits_pending overflows_debits_posted overflows_credits_posted overflows_debits
overflows_credits overflows_timeout exceeds_credits exceeds_debits
""".split())])

assert len(CreateAccountResult) == 22 and len(CreateTransferResult) == 56


def _u128(name):
    return [(name + "_lo", "<u8"), (name + "_hi", "<u8")]


# Account (tigerbeetle.zig:7-29): 128 bytes, align 16, no padding.
ACCOUNT_DTYPE = np.dtype(
    _u128("id") + _u128("debits_pending") + _u128("debits_posted") + _u128("credits_pending")
    + _u128("credits_posted") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("reserved", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")])

# Transfer (tigerbeetle.zig:64-89).
TRANSFER_DTYPE = np.dtype(
    _u128("id") + _u128("debit_account_id") + _u128("credit_account_id") + _u128("amount")
    + _u128("pending_id") + _u128("user_data_128")
    + [("user_data_64", "<u8"), ("user_data_32", "<u4"), ("timeout", "<u4"), ("ledger", "<u4"),
       ("code", "<u2"), ("flags", "<u2"), ("timestamp", "<u8")])

# {index: u32, result: u32} (tigerbeetle.zig:231-249).
RESULT_DTYPE = np.dtype([("index", "<u4"), ("result", "<u4")])

assert ACCOUNT_DTYPE.itemsize == 128 and TRANSFER_DTYPE.itemsize == 128 and RESULT_DTYPE.itemsize == 8

ACCOUNT_FIELDS = ("id", "debits_pending", "debits_posted", "credits_pending", "credits_posted",
                  "user_data_128", "user_data_64", "user_data_32", "reserved", "ledger", "code",
                  "flags", "timestamp")
TRANSFER_FIELDS = ("id", "debit_account_id", "credit_account_id", "amount", "pending_id",
                   "user_data_128", "user_data_64", "user_data_32", "timeout", "ledger", "code",
                   "flags", "timestamp")
_U128_FIELDS = {"id", "debits_pending", "debits_posted", "credits_pending", "credits_posted",
                "user_data_128", "debit_account_id", "credit_account_id", "amount", "pending_id"}

_ACCOUNT_STRUCT = struct.Struct("<" + "QQ" * 6 + "QIIIHHQ")
_TRANSFER_STRUCT = struct.Struct("<" + "QQ" * 6 + "QIIIHHQ")


def _split(v):
    return (v & U64_MAX, v >> 64)


def pack_account(id, debits_pending=0, debits_posted=0, credits_pending=0, credits_posted=0,
                 user_data_128=0, user_data_64=0, user_data_32=0, reserved=0, ledger=0, code=0,
                 flags=0, timestamp=0):
    return _ACCOUNT_STRUCT.pack(*_split(id), *_split(debits_pending), *_split(debits_posted),
                                *_split(credits_pending), *_split(credits_posted),
                                *_split(user_data_128), user_data_64, user_data_32, reserved,
                                ledger, code, flags, timestamp)


def pack_transfer(id, debit_account_id=0, credit_account_id=0, amount=0, pending_id=0,
                  user_data_128=0, user_data_64=0, user_data_32=0, timeout=0, ledger=0, code=0,
                  flags=0, timestamp=0):
    return _TRANSFER_STRUCT.pack(*_split(id), *_split(debit_account_id),
                                 *_split(credit_account_id), *_split(amount), *_split(pending_id),
                                 *_split(user_data_128), user_data_64, user_data_32, timeout,
                                 ledger, code, flags, timestamp)


def unpack_account(b):
    v = _ACCOUNT_STRUCT.unpack(b)
    out, i = {}, 0
    for f in ACCOUNT_FIELDS:
        if f in _U128_FIELDS:
            out[f] = v[i] | (v[i + 1] << 64)
            i += 2
        else:
            out[f] = v[i]
            i += 1
    return out


def unpack_transfer(b):
    v = _TRANSFER_STRUCT.unpack(b)
    out, i = {}, 0
    for f in TRANSFER_FIELDS:
        if f in _U128_FIELDS:
            out[f] = v[i] | (v[i + 1] << 64)
            i += 2
        else:
            out[f] = v[i]
            i += 1
    return out


def u128_column(arr, name):
    """Python ints of a u128 column of a structured array."""
    lo = arr[name + "_lo"].astype(object)
    hi = arr[name + "_hi"].astype(object)
    return [int(a) | (int(b) << 64) for a, b in zip(lo, hi)]
