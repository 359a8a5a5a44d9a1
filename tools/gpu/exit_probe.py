"""Teardown probe: which part of a profiled run faults in exit()?  (VERDICT r2 weak #4.)

Run under `rocprofv3 --kernel-trace --stats -- python3 tools/gpu/exit_probe.py MODE OUTDIR`:
  torch   torch only (a device tensor, a kernel)
  lib     libtbgpu only (an engine: init, one commit, close) — no torch import
  both    both, the engine closed explicitly
  leak    both, the engine left to the garbage collector at interpreter shutdown
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
    print("probe %s done" % mode, flush=True)


if __name__ == "__main__":
    main()
