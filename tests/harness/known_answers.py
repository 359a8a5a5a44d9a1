"""Runner of tests/golden/client_known_answers.json (the reference's client integration-test known
answers, tests/golden/make_client_fixtures.py) against anything with commit(operation, timestamp,
body) -> reply bytes: the oracle, an Engine, or a multi-device NodeEngine."""
import json
import os

import numpy as np

from tigerbeetle_amd.types import (ACCOUNT_DTYPE, TRANSFER_DTYPE, CreateAccountResult, CreateTransferResult,
                                   Operation, pack_account, pack_transfer, unpack_account, unpack_transfer)

PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "golden",
                    "client_known_answers.json")


def load():
    with open(PATH) as f:
        return json.load(f)["scenarios"]


def _ids_body(ids):
    return b"".join(int(i).to_bytes(16, "little") for i in ids)


def run(scenario, engine, t0=1000):
    """Commit every step in order (timestamps as the reference harness: prepare_timestamp += events,
    then +1 per commit, state_machine.zig:1480-1485) and assert every expected answer."""
    t = t0
    for k, step in enumerate(scenario["steps"]):
        op = step["op"]
        where = "%s step %d (%s)" % (scenario["name"], k, op)
        if op in ("create_accounts", "create_transfers"):
            pack = pack_account if op == "create_accounts" else pack_transfer
            body = b"".join(pack(**ev) for ev in step["events"])
            t += len(step["events"]) + 1
            reply = engine.commit(Operation[op], t, body)
            enum = CreateAccountResult if op == "create_accounts" else CreateTransferResult
            got = [[int(i), enum(int(r)).name] for i, r in np.frombuffer(reply, dtype=np.uint32).reshape(-1, 2)]
            assert got == step["results"], "%s: results %r, expected %r" % (where, got, step["results"])
        else:
            t += 1
            reply = engine.commit(Operation[op], t, _ids_body(step["ids"]))
            unpack = unpack_account if op == "lookup_accounts" else unpack_transfer
            recs = [unpack(reply[i:i + 128]) for i in range(0, len(reply), 128)]
            assert len(recs) == len(step["expect"]), "%s: %d records, expected %d" % (where, len(recs),
                                                                                     len(step["expect"]))
            for rec, exp in zip(recs, step["expect"]):
                for field, value in exp.items():
                    if field.endswith("_nonzero"):
                        assert rec[field[:-len("_nonzero")]] != 0, "%s: %s is zero" % (where, field)
                    else:
                        assert rec[field] == value, "%s: id %d %s = %d, expected %d" % (where, rec["id"], field,
                                                                                      rec[field], value)
    return t


__all__ = ["load", "run", "ACCOUNT_DTYPE", "TRANSFER_DTYPE"]
