"""The reference's table DSL and `check()` harness, restated in Python.

* `parse()` follows src/testing/table.zig:8-100 (row tokens, `_` defaults, letter labels,
  `-N` = maxInt - N for unsigned fields, trailing `//` comments).
* The action schema follows TestAction / TestCreateAccount / TestCreateTransfer of
  src/state_machine.zig:1247-1371.
* `check()` follows src/state_machine.zig:1373-1529: it builds each request, the expected sparse
  reply and the expected lookup records, bumps `prepare_timestamp` exactly as the reference test
  does, commits through an engine and compares reply bytes exactly.

An "engine" is any object with:
    commit(operation:int, timestamp:int, body:bytes) -> bytes   (raises on a non-OK status)
    set_balances(account_id:int, dp:int, dpost:int, cp:int, cpost:int)
"""
import re

from tigerbeetle_amd.types import (CreateAccountResult, CreateTransferResult, Operation,
                                   U64_MAX, pack_account, pack_transfer, unpack_account,
                                   unpack_transfer)

_BITS = {"u1": 1, "u10": 10, "u13": 13, "u16": 16, "u32": 32, "u64": 64, "u128": 128}

# (name, kind, default-or-REQUIRED).  kind: an int type, ("flag", "LNK"), or "result".
REQUIRED = object()
ACCOUNT_COLUMNS = [
    ("id", "u128", REQUIRED), ("debits_pending", "u128", 0), ("debits_posted", "u128", 0),
    ("credits_pending", "u128", 0), ("credits_posted", "u128", 0), ("user_data_128", "u128", 0),
    ("user_data_64", "u64", 0), ("user_data_32", "u32", 0), ("reserved", "u1", 0),
    ("ledger", "u32", REQUIRED), ("code", "u16", REQUIRED), ("flags_linked", ("flag", "LNK"), None),
    ("flags_debits_must_not_exceed_credits", ("flag", "D<C"), None),
    ("flags_credits_must_not_exceed_debits", ("flag", "C<D"), None),
    ("flags_padding", "u13", 0), ("timestamp", "u64", 0), ("result", "account_result", REQUIRED),
]
TRANSFER_COLUMNS = [
    ("id", "u128", REQUIRED), ("debit_account_id", "u128", REQUIRED),
    ("credit_account_id", "u128", REQUIRED), ("amount", "u128", 0), ("pending_id", "u128", 0),
    ("user_data_128", "u128", 0), ("user_data_64", "u64", 0), ("user_data_32", "u32", 0),
    ("timeout", "u32", 0), ("ledger", "u32", REQUIRED), ("code", "u16", REQUIRED),
    ("flags_linked", ("flag", "LNK"), None), ("flags_pending", ("flag", "PEN"), None),
    ("flags_post_pending_transfer", ("flag", "POS"), None),
    ("flags_void_pending_transfer", ("flag", "VOI"), None),
    ("flags_balancing_debit", ("flag", "BDR"), None), ("flags_balancing_credit", ("flag", "BCR"), None),
    ("flags_padding", "u10", 0), ("timestamp", "u64", 0), ("result", "transfer_result", REQUIRED),
]


class _Tokens:
    def __init__(self, tokens):
        self.tokens = tokens
        self.i = 0

    def next(self):
        t = self.tokens[self.i]
        self.i += 1
        return t

    def peek(self):
        return self.tokens[self.i] if self.i < len(self.tokens) else None


def parse_int(token, kind):
    """table.zig:37-47: skip one leading letter; `-N` on an unsigned type means maxInt - N."""
    bits = _BITS[kind]
    maxv = (1 << bits) - 1
    off = 1 if token[0].isalpha() else 0
    if token[off] == "-":
        v = maxv - int(token[off + 1:], 10)
    else:
        v = int(token[off:], 10)
    if not 0 <= v <= maxv:
        raise ValueError("integer out of range for %s: %r" % (kind, token))
    return v


def _parse_value(tokens, kind):
    if kind in _BITS:
        return parse_int(tokens.next(), kind)
    if isinstance(kind, tuple) and kind[0] == "flag":
        t = tokens.next()
        if t != kind[1]:
            raise ValueError("unknown flag %r (expected %r)" % (t, kind[1]))
        return t
    if kind == "account_result":
        return CreateAccountResult[tokens.next()]
    if kind == "transfer_result":
        return CreateTransferResult[tokens.next()]
    raise ValueError(kind)


def _parse_struct(tokens, columns):
    row = {}
    for name, kind, default in columns:
        if default is not REQUIRED and tokens.peek() == "_":  # table.zig:59-62 (eat "_")
            tokens.next()
            row[name] = default
        else:
            row[name] = _parse_value(tokens, kind)
    return row


def parse(text):
    """Parse a table into a list of (variant, data) actions (table.zig:8-23 + TestAction)."""
    actions = []
    for line in text.split("\n"):
        tokens = line.split()
        if not tokens:
            continue
        toks = _Tokens(tokens)
        variant = toks.next()
        if variant == "setup":
            data = [parse_int(toks.next(), "u128") for _ in range(5)]
        elif variant == "tick":
            data = parse_int(toks.next(), "u64")
        elif variant == "commit":
            data = Operation[toks.next()]
        elif variant == "account":
            data = _parse_struct(toks, ACCOUNT_COLUMNS)
        elif variant == "transfer":
            data = _parse_struct(toks, TRANSFER_COLUMNS)
        elif variant == "lookup_account":
            account_id = parse_int(toks.next(), "u128")
            if toks.peek() == "_":
                toks.next()
                balance = None
            else:
                balance = [parse_int(toks.next(), "u128") for _ in range(4)]
            data = (account_id, balance)
        elif variant == "lookup_transfer":
            transfer_id = parse_int(toks.next(), "u128")
            kind = toks.next()
            if kind == "exists":
                t = toks.next()
                value = {"0": False, "false": False, "F": False, "1": True, "true": True, "T": True}[t]
            elif kind == "amount":
                value = parse_int(toks.next(), "u128")
            else:
                raise ValueError("unknown lookup_transfer variant %r" % kind)
            data = (transfer_id, kind, value)
        else:
            raise ValueError("unknown row variant %r" % variant)
        rest = toks.peek()
        if rest is not None and rest != "//":  # table.zig:19-20
            raise ValueError("trailing token %r in row %r" % (rest, line))
        actions.append((variant, data))
    return actions


def account_event(a):
    """TestCreateAccount.event (state_machine.zig:1300-1321)."""
    flags = ((1 if a["flags_linked"] else 0) | (2 if a["flags_debits_must_not_exceed_credits"] else 0)
             | (4 if a["flags_credits_must_not_exceed_debits"] else 0) | (a["flags_padding"] << 3))
    return pack_account(a["id"], a["debits_pending"], a["debits_posted"], a["credits_pending"],
                        a["credits_posted"], a["user_data_128"], a["user_data_64"], a["user_data_32"],
                        a["reserved"], a["ledger"], a["code"], flags, a["timestamp"])


def transfer_event(t):
    """TestCreateTransfer.event (state_machine.zig:1346-1370)."""
    flags = ((1 if t["flags_linked"] else 0) | (2 if t["flags_pending"] else 0)
             | (4 if t["flags_post_pending_transfer"] else 0)
             | (8 if t["flags_void_pending_transfer"] else 0)
             | (16 if t["flags_balancing_debit"] else 0) | (32 if t["flags_balancing_credit"] else 0)
             | (t["flags_padding"] << 6))
    return pack_transfer(t["id"], t["debit_account_id"], t["credit_account_id"], t["amount"],
                         t["pending_id"], t["user_data_128"], t["user_data_64"], t["user_data_32"],
                         t["timeout"], t["ledger"], t["code"], flags, t["timestamp"])


def _result(index, code):
    return index.to_bytes(4, "little") + int(code).to_bytes(4, "little")


def _zero_timestamps(reply):
    """state_machine.zig:1500-1506: lookups zero the timestamp of every returned record."""
    out = bytearray(reply)
    for off in range(0, len(out), 128):
        out[off + 120:off + 128] = b"\x00" * 8
    return bytes(out)


class TableMismatch(AssertionError):
    pass


def check(text, engine):
    """Run one table against `engine` (state_machine.zig:1373-1529)."""
    accounts = {}
    transfers = {}
    request = bytearray()
    reply = bytearray()
    operation = None
    prepare_timestamp = 0

    for variant, data in parse(text):
        if variant == "setup":
            assert operation is None
            engine.set_balances(*data)
        elif variant == "tick":
            assert data > 0
            prepare_timestamp += data
            assert prepare_timestamp <= U64_MAX
        elif variant == "account":
            assert operation in (None, Operation.create_accounts)
            operation = Operation.create_accounts
            event = account_event(data)
            request += event
            if data["result"] == CreateAccountResult.ok:
                accounts[data["id"]] = event
            else:
                reply += _result(len(request) // 128 - 1, data["result"])
        elif variant == "transfer":
            assert operation in (None, Operation.create_transfers)
            operation = Operation.create_transfers
            event = transfer_event(data)
            request += event
            if data["result"] == CreateTransferResult.ok:
                transfers[data["id"]] = event
            else:
                reply += _result(len(request) // 128 - 1, data["result"])
        elif variant == "lookup_account":
            assert operation in (None, Operation.lookup_accounts)
            operation = Operation.lookup_accounts
            account_id, balance = data
            request += account_id.to_bytes(16, "little")
            if balance is not None:
                a = unpack_account(accounts[account_id])
                a["debits_pending"], a["debits_posted"], a["credits_pending"], a["credits_posted"] = balance
                reply += pack_account(**a)
        elif variant == "lookup_transfer":
            assert operation in (None, Operation.lookup_transfers)
            operation = Operation.lookup_transfers
            transfer_id, kind, value = data
            request += transfer_id.to_bytes(16, "little")
            if kind == "exists":
                if value:
                    reply += transfers[transfer_id]
            else:
                t = unpack_transfer(transfers[transfer_id])
                t["amount"] = value
                reply += pack_transfer(**t)
        elif variant == "commit":
            assert operation in (None, data)
            prepare_timestamp += 1
            # StateMachine.prepare (state_machine.zig:336-343).
            if data in (Operation.create_accounts, Operation.create_transfers):
                prepare_timestamp += len(request) // 128
            assert prepare_timestamp <= U64_MAX
            actual = engine.commit(int(data), prepare_timestamp, bytes(request))
            if data in (Operation.lookup_accounts, Operation.lookup_transfers):
                actual = _zero_timestamps(actual)
            if bytes(actual) != bytes(reply):
                raise TableMismatch(describe_mismatch(data, bytes(reply), bytes(actual)))
            request = bytearray()
            reply = bytearray()
            operation = None
        else:
            raise AssertionError(variant)
    assert operation is None and not request and not reply


def describe_mismatch(op, expected, actual):
    lines = ["reply mismatch for %s (expected %d bytes, got %d)" % (Operation(op).name, len(expected), len(actual))]
    if op in (Operation.create_accounts, Operation.create_transfers):
        enum_t = CreateAccountResult if op == Operation.create_accounts else CreateTransferResult

        def decode(b):
            return [(int.from_bytes(b[i:i + 4], "little"), enum_t(int.from_bytes(b[i + 4:i + 8], "little")).name)
                    for i in range(0, len(b), 8)]
        lines.append("expected: %s" % decode(expected))
        lines.append("actual:   %s" % decode(actual))
    else:
        unpack = unpack_account if op == Operation.lookup_accounts else unpack_transfer
        lines.append("expected: %s" % [unpack(expected[i:i + 128]) for i in range(0, len(expected), 128)])
        lines.append("actual:   %s" % [unpack(actual[i:i + 128]) for i in range(0, len(actual), 128)])
    return "\n".join(lines)


def load_tables(path):
    """Read tests/golden/state_machine_tables.txt -> list of (name, table_text)."""
    tables, name, rows = [], None, None
    for line in open(path, encoding="utf-8"):
        line = line.rstrip("\n")
        if line.startswith("@table "):
            name = re.sub(r"\s+\(state_machine.*$", "", line[len("@table "):])
            rows = []
        elif line == "@end":
            tables.append((name, "\n".join(rows)))
            name, rows = None, None
        elif rows is not None:
            rows.append(line)
    return tables
