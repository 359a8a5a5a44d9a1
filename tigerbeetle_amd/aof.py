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

Checksums are `vsr.checksum` (Aegis-128L MAC, zero key: `src/vsr/checksum.zig`), computed by the
engine library's host-side `tbgpu_checksum` (pinned by the reference's checksum vectors,
tests/test_checksum.py).  The reader verifies what the reference's iterator verifies
(`src/aof.zig:197-233`): the magic number, the sizes, the header checksum (over header bytes
[16, 128), `src/vsr.zig:405-411`), the body checksum (`:413-420`) and the hash chain (`parent` ==
the previous entry's `checksum`, `:221-226`); `read_prepares` also refuses a gap in the op
sequence.  `write_aof` writes the same layout with real checksums; it makes fixtures.
"""
import struct
from dataclasses import dataclass

from ._lib import checksum as vsr_checksum

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


def read_entries(path, validate_chain=True, validate_checksums=True):
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
        if validate_checksums:
            header = data[off + META:off + META + HEADER]
            if vsr_checksum(header[16:]).to_bytes(16, "little") != checksum:
                raise AofError("header checksum mismatch at offset %d" % off)
            if vsr_checksum(data[off + META + HEADER:off + META + size]).to_bytes(16, "little") != _cbody:
                raise AofError("body checksum mismatch at op %d" % op)
        if validate_chain and last is not None and parent != last:
            raise AofError("checksum chain mismatch at op %d" % op)
        last = checksum
        body = data[off + META + HEADER:off + META + size]
        out.append((command, AofPrepare(op, timestamp, operation, body, checksum, parent, replica, primary)))
        off += disk
    return out


def read_prepares(path, validate_chain=True, validate_checksums=True, require_contiguous=True):
    """The committed prepares of an AOF in op order: `prepare` entries of state-machine operations
    (the replay skips VSR-reserved ones, src/aof.zig:349-350), one per op (duplicates — an AOF
    can backtrack, :80-84 — must be identical).

    require_contiguous (default on) is a check BEYOND the reference's iterator, which validates
    only the checksums and the parent chain (src/aof.zig:214-260): the prepare ops, VSR-reserved
    ones included, must form one contiguous range, since a missing op would replay a different
    history.  Pass False to read every file the reference's replay would read."""
    by_op, all_ops = {}, set()
    for command, p in read_entries(path, validate_chain, validate_checksums):
        if command != COMMAND_PREPARE:
            continue
        all_ops.add(p.op)
        if p.operation < VSR_OPERATIONS_RESERVED:
            continue
        prev = by_op.get(p.op)
        if prev is not None and (prev.timestamp, prev.operation, prev.body) != (p.timestamp, p.operation, p.body):
            raise AofError("op %d logged twice with different contents" % p.op)
        by_op[p.op] = p
    if require_contiguous and all_ops and len(all_ops) != max(all_ops) - min(all_ops) + 1:
        missing = sorted(set(range(min(all_ops), max(all_ops) + 1)) - all_ops)
        raise AofError("op sequence has gaps (first missing op %d, %d missing; this check goes beyond the "
                       "reference iterator: read_prepares(..., require_contiguous=False) skips it)"
                       % (missing[0], len(missing)))
    return [by_op[k] for k in sorted(by_op)]


def write_aof(path, prepares, replica=0, primary=0):
    """Write prepares (op, timestamp, operation, body) in the AOF layout, with real checksums
    (body, then header: set_checksum_body / set_checksum, src/vsr.zig:422-429) chained through
    `parent`."""
    parent = b"\0" * 16
    with open(path, "wb") as f:
        for p in prepares:
            size = HEADER + len(p.body)
            cbody = vsr_checksum(p.body).to_bytes(16, "little")
            rest = _HDR.pack(b"\0" * 16, cbody, parent, b"\0" * 16, b"\0" * 16, 0, 0, 0, 0, p.op, p.op, p.timestamp,
                             size, replica, COMMAND_PREPARE, p.operation, 0)[16:]
            checksum = vsr_checksum(rest).to_bytes(16, "little")
            hdr = checksum + rest
            meta = MAGIC.to_bytes(16, "little") + struct.pack("<QQ", primary, replica) + b"\0" * 4064
            entry = meta + hdr + p.body
            f.write(entry + b"\0" * (_sector_ceil(len(entry)) - len(entry)))
            parent = checksum


def replay(prepares, state_machine):
    """Commit every prepare into `state_machine` in op order; returns the replies.  A StateMachine
    (the reference interface: prepare / prefetch / commit(client, op, timestamp, operation, body),
    src/state_machine.zig:336-540) is driven the way the replica drives it; an Engine or the oracle
    takes commit(operation, timestamp, body)."""
    if hasattr(state_machine, "prefetch"):
        out = []
        for p in prepares:
            state_machine.prepare(p.operation, p.body)
            state_machine.prefetch(lambda _sm: None, p.op, p.operation, p.body)
            out.append(state_machine.commit(0, p.op, p.timestamp, p.operation, p.body))
        return out
    return [state_machine.commit(p.operation, p.timestamp, p.body) for p in prepares]
