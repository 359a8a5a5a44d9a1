"""AOF (append-only file) replay as a batch source — SURVEY.md §8f rank 4.

The reference's replica can log every prepare it commits to an AOF (`src/aof.zig`); `aof replay`
(`:344-390`) feeds the entries back through a cluster.  Here an AOF is read as the exact sequence
of committed prepares — operation, timestamp and body of every `prepare` entry in op order — and
committed straight into a state machine (the HIP engine, the oracle or the C++ host mirror), so a
production-recorded batch stream can be checked engine-vs-oracle with its original timestamps.

On-disk format restated from the reference (data layout only):

* `AOFEntry` (`src/aof.zig:37-59`): `magic_number` u128 (`:24`), `AOFEntryMetadata`
  (`:26-35`: primary u64, replica u64, 4064 reserved bytes — 4096 bytes with the magic), then the
  message (`message_size_max` bytes, sector aligned).  On disk an entry takes
  `sector_ceil(4096 + header.size)` bytes (`calculate_disk_size`, `:55-59`; `sector_ceil`,
  `src/vsr.zig:1560-1563`, sector 4096).
* The message starts with the 128-byte `vsr.Header` (`src/vsr.zig:235-352`): checksum @0,
  checksum_body @16, parent @32, client @48, context @64, request u32 @80, cluster u32 @84,
  epoch u32 @88, view u32 @92, op u64 @96, commit u64 @104, timestamp u64 @112, size u32 @120,
  replica u8 @124, command u8 @125 (`prepare` = 6, `:111-121`), operation u8 @126, version u8
  @127.  The body follows the header (`size` includes the header).

Checksums are Aegis128L MACs (`vsr.checksum`); they are not recomputed here (no Aegis
implementation in this repo), so a reader checks the magic number, the sizes and the hash chain
(`parent` == previous entry's `checksum`, as the reference's iterator does, `:221-226`) but not
the MAC values themselves — parity on a recorded AOF is pinned by the replay, not by the MACs.
`write_aof` writes the same layout with placeholder (non-MAC) checksums that keep the chain
consistent; it exists to make fixtures.
"""
import struct
from dataclasses import dataclass

MAGIC = 312960301372567410560647846651901451202  # src/aof.zig:24
SECTOR = 4096
META = 4096          # magic (16) + AOFEntryMetadata (8 + 8 + 4064)
HEADER = 128         # vsr.Header
COMMAND_PREPARE = 6  # vsr.Command.prepare
VSR_OPERATIONS_RESERVED = 128  # operations below are VSR-internal (vsr.Operation.vsr_reserved)

_HDR = struct.Struct("<16s16s16s16s16sIIIIQQQIBBBB")
assert _HDR.size == HEADER


class AofError(ValueError):
    pass


@dataclass
class AofPrepare:
    op: int
    timestamp: int
    operation: int
    body: bytes
    checksum: bytes = b"\0" * 16
    parent: bytes = b"\0" * 16
    replica: int = 0
    primary: int = 0


def _sector_ceil(n):
    return (n + SECTOR - 1) // SECTOR * SECTOR


def read_entries(path, validate_chain=True):
    """Every entry of an AOF file, in file order (AOF.Iterator.next, src/aof.zig:197-233)."""
    with open(path, "rb") as f:
        data = f.read()
    out, off, last = [], 0, None
    while off < len(data):
        if off + META + HEADER > len(data):
            raise AofError("short read at offset %d" % off)
        magic = int.from_bytes(data[off:off + 16], "little")
        if magic != MAGIC:
            raise AofError("magic number mismatch at offset %d" % off)
        primary, replica = struct.unpack_from("<QQ", data, off + 16)
        h = _HDR.unpack_from(data, off + META)
        checksum, _cbody, parent = h[0], h[1], h[2]
        op, timestamp, size, command, operation = h[9], h[11], h[12], h[14], h[15]
        if size < HEADER:
            raise AofError("header size %d < %d at offset %d" % (size, HEADER, off))
        disk = _sector_ceil(META + size)
        if off + disk > len(data):
            raise AofError("short read at offset %d" % off)
        if validate_chain and last is not None and parent != last:
            raise AofError("checksum chain mismatch at op %d" % op)
        last = checksum
        body = data[off + META + HEADER:off + META + size]
        out.append((command, AofPrepare(op, timestamp, operation, body, checksum, parent, replica, primary)))
        off += disk
    return out


def read_prepares(path, validate_chain=True):
    """The committed prepares of an AOF in op order: `prepare` entries of state-machine operations
    (the replay skips VSR-reserved ones, src/aof.zig:349-350), one per op (duplicates — an AOF
    can backtrack, :80-84 — must be identical)."""
    by_op = {}
    for command, p in read_entries(path, validate_chain):
        if command != COMMAND_PREPARE or p.operation < VSR_OPERATIONS_RESERVED:
            continue
        prev = by_op.get(p.op)
        if prev is not None and (prev.timestamp, prev.operation, prev.body) != (p.timestamp, p.operation, p.body):
            raise AofError("op %d logged twice with different contents" % p.op)
        by_op[p.op] = p
    return [by_op[k] for k in sorted(by_op)]


def write_aof(path, prepares, replica=0, primary=0):
    """Write prepares (op, timestamp, operation, body) in the AOF layout; placeholder checksums
    (op-derived, not Aegis MACs) chained through `parent`."""
    parent = b"\0" * 16
    with open(path, "wb") as f:
        for p in prepares:
            size = HEADER + len(p.body)
            checksum = struct.pack("<QQ", 0x41_4F_46_00 ^ p.op, p.timestamp)
            hdr = _HDR.pack(checksum, b"\0" * 16, parent, b"\0" * 16, b"\0" * 16, 0, 0, 0, 0, p.op, p.op, p.timestamp,
                            size, replica, COMMAND_PREPARE, p.operation, 0)
            meta = MAGIC.to_bytes(16, "little") + struct.pack("<QQ", primary, replica) + b"\0" * 4064
            entry = meta + hdr + p.body
            f.write(entry + b"\0" * (_sector_ceil(len(entry)) - len(entry)))
            parent = checksum


def replay(prepares, state_machine):
    """Commit every prepare into `state_machine` (anything with commit(operation, timestamp, body))
    in op order; returns the replies."""
    return [state_machine.commit(p.operation, p.timestamp, p.body) for p in prepares]
