"""Debug helper: run one differential scenario on the GPU and the oracle, print the first mismatch
with the events around it (used while developing kernels; not a test)."""
import sys

sys.path.insert(0, ".")
from tests.harness.oracle import OracleEngine  # noqa: E402
from tests.harness.workload import make_scenario  # noqa: E402
from tests.test_gpu_differential import CONFIGS  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402
from tigerbeetle_amd.types import CreateTransferResult, unpack_transfer  # noqa: E402


def decode(b):
    return [(int.from_bytes(b[i:i + 4], "little"), int.from_bytes(b[i + 4:i + 8], "little")) for i in range(0, len(b), 8)]


def main(config, seed, many):
    sc = make_scenario(seed * 7919 + sum(map(ord, config)), **CONFIGS[config])
    o = OracleEngine()
    g = Engine(Options(accounts_max=4096, transfers_max=1 << 17, pass_events_max=8192 * 4, pass_batches_max=64))
    k = 0
    for step in sc.steps:
        if step[0] == "setup":
            o.set_balances(*step[1:]); g.set_balances(*step[1:]); continue
        _, op, ts, events = step
        body = b"".join(events)
        e = o.commit(op, ts, body)
        a = g.commit(op, ts, body)
        if e != a:
            E, A = dict(decode(e)), dict(decode(a))
            idx = sorted(set(E) | set(A))
            bad = [i for i in idx if E.get(i) != A.get(i)]
            print("prepare %d op %d: %d mismatching indices, first %s" % (k, op, len(bad), bad[:10]))
            print("stats", g.stats())
            for i in bad[:6]:
                lo = max(0, i - 3)
                for j in range(lo, min(len(events), i + 2)):
                    t = unpack_transfer(events[j]) if op == 129 else None
                    name = lambda c: CreateTransferResult(c).name if c is not None and op == 129 else c
                    print("  %s ev %d exp=%s act=%s %s" % ("*" if j == i else " ", j, name(E.get(j, 0)), name(A.get(j, 0)),
                          {kk: (hex(v) if kk in ("id", "pending_id") else v) for kk, v in (t or {}).items()
                           if kk in ("id", "flags", "pending_id", "amount", "ledger", "code", "timestamp")}))
                print()
            return
        k += 1
    print("no mismatch")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), len(sys.argv) > 3)
