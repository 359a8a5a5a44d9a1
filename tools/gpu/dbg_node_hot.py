"""Debug: the node engine (2 logical shards) against the oracle and the single engine on the hot_ids
differential workload, one prepare per call; at the first differing reply, prints the event, each
engine's code and each engine's stored transfer for its id."""
import sys

import numpy as np

sys.path.insert(0, ".")
from tests.harness.oracle import OracleEngine  # noqa: E402
from tests.harness.workload import make_scenario  # noqa: E402
from tests.test_gpu_differential import CONFIGS  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402
from tigerbeetle_amd.types import TRANSFER_DTYPE  # noqa: E402

config = sys.argv[1] if len(sys.argv) > 1 else "hot_ids"
sc = make_scenario(5003 + sum(map(ord, config)), **CONFIGS[config])
opts = dict(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64)
oracle = OracleEngine()
node = Engine(Options(devices=(0, 0), **opts))
single = Engine(Options(**opts))


def codes(reply):
    r = np.frombuffer(reply, dtype=np.uint32).reshape(-1, 2)
    return {int(i): int(c) for i, c in r}


def show(t):
    return dict(id=int(t["id_lo"]), dr=int(t["debit_account_id_lo"]), cr=int(t["credit_account_id_lo"]),
                amount=int(t["amount_lo"]), pid=int(t["pending_id_lo"]), code=int(t["code"]), flags=int(t["flags"]),
                ledger=int(t["ledger"]), ts=int(t["timestamp"]), ud128=int(t["user_data_128_lo"]))


for k, step in enumerate(sc.steps):
    if step[0] == "setup":
        for e in (oracle, node, single):
            e.set_balances(*step[1:])
        continue
    _, op, ts, events = step
    body = b"".join(events)
    ro, rn, rs = oracle.commit(op, ts, body), node.commit(op, ts, body), single.commit(op, ts, body)
    if ro == rn and ro == rs:
        continue
    print("step", k, "op", op, "ts", ts, "events", len(events), "node ok" if ro == rn else "NODE DIFFERS",
          "single ok" if ro == rs else "SINGLE DIFFERS")
    co, cn, cs = codes(ro), codes(rn), codes(rs)
    ev = np.frombuffer(body, dtype=TRANSFER_DTYPE) if op == 129 else None
    for i in sorted(set(co) | set(cn) | set(cs)):
        if co.get(i, 0) == cn.get(i, 0) == cs.get(i, 0):
            continue
        print(" event", i, "oracle", co.get(i, 0), "node", cn.get(i, 0), "single", cs.get(i, 0))
        if ev is not None:
            t = ev[i]
            print("   event", show(t))
            ids = np.zeros((1, 2), dtype=np.uint64)
            ids[0, 0], ids[0, 1] = t["id_lo"], t["id_hi"]
            for name, e in (("oracle", oracle), ("node", node), ("single", single)):
                got = e.commit(131, ts + 1, ids.tobytes())
                if got:
                    print("   %-6s stored" % name, show(np.frombuffer(got, dtype=TRANSFER_DTYPE)[0]))
                else:
                    print("   %-6s stored none" % name)
            # every earlier event of the scenario with this id
            for kk, st in enumerate(sc.steps[:k + 1]):
                if st[0] != "commit" or st[1] != 129:
                    continue
                arr = np.frombuffer(b"".join(st[3]), dtype=TRANSFER_DTYPE)
                for j in np.nonzero((arr["id_lo"] == t["id_lo"]) & (arr["id_hi"] == t["id_hi"]))[0]:
                    print("     step %d event %d" % (kk, j), show(arr[j]))
        break
    print(node.stats())
    break
else:
    print("all replies equal")
