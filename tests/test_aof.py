"""AOF replay (tigerbeetle_amd/aof.py, the reference's src/aof.zig layout): the reader against the
writer, its format checks, and a replay through the oracle equal to committing the same prepares
directly.  CPU only; tests/test_gpu_aof.py replays through the GPU engine."""
import struct

import pytest

from tests.harness.oracle import OracleEngine
from tests.harness.workload import make_scenario, run_oracle
from tigerbeetle_amd import aof


def scenario_prepares(seed, **kw):
    sc = make_scenario(seed, **kw)
    assert all(step[0] == "commit" for step in sc.steps)
    return sc, [aof.AofPrepare(op=k + 1, timestamp=ts, operation=op, body=b"".join(events))
                for k, (_, op, ts, events) in enumerate(sc.steps)]


def test_round_trip_and_layout(tmp_path):
    _, prepares = scenario_prepares(3)
    path = tmp_path / "replica.aof"
    aof.write_aof(path, prepares)
    data = path.read_bytes()
    # First entry: magic, then the header at 4096 with size = 128 + body; entries sector aligned.
    assert int.from_bytes(data[:16], "little") == aof.MAGIC
    size = struct.unpack_from("<I", data, 4096 + 120)[0]
    assert size == 128 + len(prepares[0].body)
    assert data[4096 + 125] == aof.COMMAND_PREPARE and data[4096 + 126] == prepares[0].operation
    assert len(data) % aof.SECTOR == 0
    got = aof.read_prepares(path)
    assert [(p.op, p.timestamp, p.operation, p.body) for p in got] == \
        [(p.op, p.timestamp, p.operation, p.body) for p in prepares]


def test_format_errors(tmp_path):
    _, prepares = scenario_prepares(4)
    path = tmp_path / "bad.aof"
    aof.write_aof(path, prepares)
    data = bytearray(path.read_bytes())
    second = aof._sector_ceil(aof.META + aof.HEADER + len(prepares[0].body))
    broken = bytearray(data)
    broken[second + 4096 + 32] ^= 1  # parent of entry 2 (covered by its header checksum)
    path.write_bytes(bytes(broken))
    with pytest.raises(aof.AofError, match="header checksum"):
        aof.read_prepares(path)
    with pytest.raises(aof.AofError, match="chain"):
        aof.read_prepares(path, validate_checksums=False)
    assert len(aof.read_prepares(path, validate_chain=False, validate_checksums=False)) == len(prepares)
    broken = bytearray(data)
    broken[second + 4096 + 128 + 5] ^= 1  # a body byte of entry 2 (src/aof.zig:218)
    path.write_bytes(bytes(broken))
    with pytest.raises(aof.AofError, match="body checksum"):
        aof.read_prepares(path)
    broken = bytearray(data)
    broken[second] ^= 1  # magic of entry 2
    path.write_bytes(bytes(broken))
    with pytest.raises(aof.AofError, match="magic"):
        aof.read_prepares(path)
    path.write_bytes(bytes(data[:-10]))
    with pytest.raises(aof.AofError, match="short"):
        aof.read_prepares(path)


def test_duplicates_and_order(tmp_path):
    _, prepares = scenario_prepares(5)
    shuffled = prepares[3:] + prepares[:3] + prepares[:2]  # out of op order, two ops logged twice
    path = tmp_path / "dup.aof"
    aof.write_aof(path, shuffled)
    got = aof.read_prepares(path, validate_chain=False)
    assert [p.op for p in got] == [p.op for p in prepares]
    bad = list(prepares) + [aof.AofPrepare(1, prepares[0].timestamp, prepares[0].operation, b"x" * 128)]
    aof.write_aof(path, bad)
    with pytest.raises(aof.AofError, match="twice"):
        aof.read_prepares(path, validate_chain=False)


def test_op_gap_refused(tmp_path):
    _, prepares = scenario_prepares(6)
    path = tmp_path / "gap.aof"
    aof.write_aof(path, prepares[:3] + prepares[4:])  # op 4 missing; the chain stays consistent
    with pytest.raises(aof.AofError, match="gaps"):
        aof.read_prepares(path)
    # The reference's iterator checks only checksums and the parent chain: with the extra check off
    # the file reads like the reference would read it.
    got = aof.read_prepares(path, require_contiguous=False)
    assert [p.op for p in got] == [p.op for p in prepares if p.op != 4]
    # VSR-reserved prepares (operation < 128) fill their ops: no gap, and they are not replayed.
    reserved = aof.AofPrepare(op=4, timestamp=prepares[3].timestamp, operation=3, body=b"")
    aof.write_aof(path, prepares[:3] + [reserved] + prepares[4:])
    assert [p.op for p in aof.read_prepares(path)] == [p.op for p in prepares if p.op != 4]


def test_written_checksums_verify(tmp_path):
    from tigerbeetle_amd._lib import checksum
    _, prepares = scenario_prepares(7)
    path = tmp_path / "ck.aof"
    aof.write_aof(path, prepares[:2])
    data = path.read_bytes()
    hdr = data[4096:4096 + 128]
    assert checksum(hdr[16:]).to_bytes(16, "little") == hdr[:16]
    assert checksum(prepares[0].body).to_bytes(16, "little") == hdr[16:32]


@pytest.mark.parametrize("seed", [11, 12])
def test_replay_through_oracle(tmp_path, seed):
    sc, prepares = scenario_prepares(seed, p_linked=0.2, p_post_void=0.3, p_pending=0.4)
    path = tmp_path / "r.aof"
    aof.write_aof(path, prepares)
    direct = run_oracle(sc, OracleEngine())
    o = OracleEngine()
    replayed = aof.replay(aof.read_prepares(path), o)
    assert replayed == direct
