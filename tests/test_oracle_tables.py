"""The CPU oracle against the reference's own golden vectors.

* every table-driven StateMachine test of src/state_machine.zig:1531-2074 (18 check() calls,
  committed verbatim as tests/golden/state_machine_tables.txt);
* the sum_overflows known answers of src/state_machine.zig:1164-1179.
"""
import os

import pytest

from tests.conftest import GOLDEN
from tests.harness import table
from tests.harness.oracle import OracleEngine, lib

TABLES = table.load_tables(os.path.join(GOLDEN, "state_machine_tables.txt"))


def test_fixture_has_every_reference_table():
    assert len(TABLES) == 18
    names = {n.rsplit(" #", 1)[0] for n, _ in TABLES}
    assert len(names) == 17  # 17 test blocks, "linked accounts" calls check() twice


@pytest.mark.parametrize("name,text", TABLES, ids=[n for n, _ in TABLES])
def test_oracle_reproduces_reference_table(name, text):
    engine = OracleEngine()
    table.check(text, engine)


def test_table_mismatch_is_detected():
    # A deliberately wrong expected result must fail the harness (the harness is not vacuous).
    text = "\n".join([
        " account A1  0  0  0  0  _  _  _ _ L1 C1   _   _   _ _ _ ok",
        " account A1  0  0  0  0  _  _  _ _ L1 C1   _   _   _ _ _ ok",
        " commit create_accounts",
    ])
    with pytest.raises(table.TableMismatch):
        table.check(text, OracleEngine())


@pytest.mark.parametrize("bits", [64, 128])
def test_sum_overflows_vectors(bits):
    L = lib()
    m = (1 << bits) - 1

    def so(a, b):
        if bits == 64:
            return bool(L.tbo_sum_overflows_u64(a, b))
        return bool(L.tbo_sum_overflows_u128(a & (2**64 - 1), a >> 64, b & (2**64 - 1), b >> 64))

    assert so(m, 0) is False
    assert so(m - 1, 1) is False
    assert so(1, m - 1) is False
    assert so(m, 1) is True
    assert so(1, m) is True
    assert so(m, m) is True


def test_parse_int_dsl():
    # src/testing/table.zig:193-210 "int" test.
    assert table.parse_int("1", "u64") == 1
    assert table.parse_int("A3", "u64") == 3
    assert table.parse_int("a4", "u64") == 4
    assert table.parse_int("-5", "u64") == 2**64 - 1 - 5
    assert table.parse_int("-0", "u128") == 2**128 - 1
