"""Time one rank's route plan (tb_route_classify / _offsets / _scatter, tbgpu_route_plan_build) on a
C2-sized pass (512 prepares of 8190 transfers, 1M accounts), once with no limit account in the
table and once with 10 % limit accounts (the classify kernel then probes both accounts of every
transfer).  Single process: no collective is involved.
usage (GPU box): python tools/gpu/route_probe.py [world]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tigerbeetle_amd.sharded import GpuShard  # noqa: E402
from tigerbeetle_amd.state_machine import Engine, Options  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    accounts, batch, nb = 1_000_000, 8190, 512
    n = batch * nb
    out = {"world": world, "events": n}
    for limit_permille in (0, 100):
        engine = Engine(Options(accounts_max=accounts, transfers_max=n + 8192, pass_events_max=n,
                                pass_batches_max=nb, device=0))
        acct = torch.empty((accounts, 128), dtype=torch.uint8, device="cuda")
        engine.generate_accounts(acct.data_ptr(), 0, accounts, limit_permille=limit_permille)
        lens = [batch] * (accounts // batch) + ([accounts % batch] if accounts % batch else [])
        ts, t = [], 1_000_000_000
        for L in lens:
            t += 1 + L
            ts.append(t)
        res = torch.empty(accounts * 2, dtype=torch.int32, device="cuda")
        rb = torch.empty(len(lens), dtype=torch.int32, device="cuda")
        engine.commit_device_async(128, ts, lens, acct.data_ptr(), res.data_ptr(), rb.data_ptr())
        engine.sync()
        events = torch.empty((n, 128), dtype=torch.uint8, device="cuda")
        engine.generate_transfers(events.data_ptr(), 0, n, accounts)
        engine.sync()
        shard = GpuShard(engine, world, events_max=n)
        pts = [t + (k + 1) * (batch + 1) for k in range(nb)]
        times = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            shard.plan(pts, [batch] * nb, events)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        out["plan_ms_limit_permille_%d" % limit_permille] = round(min(times[1:]), 4)
        engine.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
