"""GPU parity on the reference's golden vectors: every table-driven StateMachine test of
src/state_machine.zig:1531-2074, committed through the C ABI exactly as the reference harness
commits (one prepare per commit, state_machine.zig:1480-1517)."""
import os

import pytest

from tests.conftest import GOLDEN
from tests.harness import table

TABLES = table.load_tables(os.path.join(GOLDEN, "state_machine_tables.txt"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,text", TABLES, ids=[n for n, _ in TABLES])
def test_gpu_reproduces_reference_table(name, text, gpu_engine_factory):
    engine = gpu_engine_factory()
    table.check(text, engine)
