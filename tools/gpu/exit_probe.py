"""Teardown probe: which part of a profiled run faults in exit()?  (VERDICT r2 weak #4.)

Run under `rocprofv3 --kernel-trace --stats -- python3 tools/gpu/exit_probe.py MODE OUTDIR`:
  torch   torch only (a device tensor, a kernel)
  lib     libtbgpu only (an engine: init, one commit, close) — no torch import
  both    both, the engine closed explicitly
  leak    both, the engine left to the garbage collector at interpreter shutdown
  flow / register / events / pipelined   one feature of the bench's engine use each (bisection)
  bench / bench_torch   bench.py's engine lifetime in small
The process maps are written at Python exit (before the C atexit handlers run), so a PC in the
fault's backtrace can be matched to its library.
"""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


KEEP = []  # engines left to interpreter shutdown ("leak")


def main():
    mode, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    atexit.register(lambda: open(os.path.join(out, "maps_%s.txt" % mode), "w").write(open("/proc/self/maps").read()))
    if mode in ("torch", "both", "leak"):
        import torch
        x = torch.arange(1 << 20, device="cuda")
        print("torch sum", int((x * 2).sum().item()), flush=True)
    if mode in ("lib", "both", "leak"):
        from tigerbeetle_amd.state_machine import Engine, Options
        from tigerbeetle_amd.types import pack_account
        e = Engine(Options(accounts_max=1024, transfers_max=4096, pass_events_max=8192, pass_batches_max=4))
        assert e.commit(128, 10, pack_account(1, ledger=1, code=1)) == b""
        print("engine commit ok", flush=True)
        if mode == "leak":
            KEEP.append(e)  # left to interpreter shutdown
        else:
            e.close()
    if mode in ("flow", "register", "events", "pipelined"):
        import numpy as np
        from tigerbeetle_amd.state_machine import Engine, Options
        from tigerbeetle_amd.types import pack_account, pack_transfer
        e = Engine(Options(accounts_max=1024, transfers_max=4096, pass_events_max=8192, pass_batches_max=4,
                           profile=(mode == "events")))
        accts = pack_account(1, ledger=1, code=1) + pack_account(2, ledger=1, code=1)
        if mode == "pipelined":
            body = np.frombuffer(accts, dtype=np.uint8).copy()
            rb, _, _ = e.commit_pipelined(128, [10], [2], body)
            assert int(rb.sum()) == 0
        else:
            assert e.commit(128, 10, accts) == b""
        if mode == "flow":  # a create_transfers pass: tb_flow, a cooperative launch
            assert e.commit(129, 20, pack_transfer(5, 1, 2, 7, ledger=1, code=1)) == b""
        if mode == "register":
            buf = np.zeros(1 << 20, dtype=np.uint8)
            e.register_host(buf)
            e.unregister_host(buf)
        e.close()
        print("%s ok" % mode, flush=True)
    if mode in ("bench", "bench_torch"):
        # bench.py's engine lifetime in small: registered host prepares, pipelined commits, close.
        if mode == "bench_torch":
            import torch
            torch.zeros(1, device="cuda")
        import numpy as np
        from tests.harness.configs import batches, generate, timestamps
        from tigerbeetle_amd.state_machine import Engine, Options
        e = Engine(Options(accounts_max=10000, transfers_max=1 << 20, pass_events_max=64 * 8190, pass_batches_max=64,
                           profile=True))
        accts, xfers = generate(e, "c2", 10000, 500000, seed=1)
        a_lens, x_lens = batches(10000, 8190), batches(500000, 8190)
        a_ts, t = timestamps(a_lens, 10**9)
        x_ts, _ = timestamps(x_lens, t + 10)
        e.commit_pipelined(128, a_ts, a_lens, np.ascontiguousarray(accts), chunk_batches=64)
        host = np.ascontiguousarray(xfers)
        e.register_host(host)
        rb, _, _ = e.commit_pipelined(129, x_ts, x_lens, host, chunk_batches=16, latency=True)
        e.unregister_host(host)
        print("bench-like commit ok, failed bytes", int(rb.sum()), flush=True)
        e.close()
    print("probe %s done" % mode, flush=True)


if __name__ == "__main__":
    main()
