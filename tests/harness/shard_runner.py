"""Per-rank body of the multi-rank sharding tests (tests/test_sharded.py, tests/test_gpu_sharded.py).

Every rank builds the same seeded scenario (tests/harness/workload.py), splits each pass's
prepares among the ranks (rank r gets a contiguous share, so the global order is rank-major), and
commits its share collectively through ShardedStateMachine.  Rank 0 collects every reply in global
order plus the merged tables, replays the scenario through one CPU oracle, and writes the verdict
to a JSON file.
"""
import json
import os
import traceback

import numpy as np
import torch
import torch.distributed as dist


def _passes(sc, max_prepares):
    """Group consecutive commits of one create operation into passes; setups stand alone."""
    out, cur = [], []
    for step in sc.steps:
        if step[0] == "setup" or (cur and (cur[0][1] != step[1] or len(cur) == max_prepares)):
            if cur:
                out.append(("commit", cur))
                cur = []
        if step[0] == "setup":
            out.append(("setup", step))
        else:
            cur.append(step)
    if cur:
        out.append(("commit", cur))
    return out


def run_rank(rank, world, port, kind, scenario_kw, max_prepares, result_path, dist_backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    if dist_backend == "nccl":  # RCCL: device tensors for every collective (one rank per GPU)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    verdict = {"ok": False}
    try:
        from tigerbeetle_amd.sharded import ShardedStateMachine
        from tests.harness.oracle import OracleEngine
        from tests.harness.workload import make_scenario, run_oracle

        if kind == "oracle":
            from tests.harness.shard_double import OracleShard
            backend = OracleShard(world)
        else:
            from tigerbeetle_amd.sharded import GpuShard
            from tigerbeetle_amd.state_machine import Engine, Options
            engine = Engine(Options(accounts_max=4096, transfers_max=1 << 16, pass_events_max=8192 * 8,
                                    pass_batches_max=64, device=0))
            backend = GpuShard(engine, world, events_max=8192 * 16, device=torch.device("cuda", 0))
        sm = ShardedStateMachine(backend)
        sc = make_scenario(**scenario_kw)
        replies = []
        for what, item in _passes(sc, max_prepares):
            if what == "setup":
                sm.test_set_balances(*item[1:])
                continue
            k = len(item)
            share = item[rank * k // world:(rank + 1) * k // world]
            bodies = [b"".join(s[3]) for s in share]
            raw = np.frombuffer(b"".join(bodies), dtype=np.uint8).reshape(-1, 128).copy()
            events = torch.from_numpy(raw).to(backend.device)
            res = sm.commit(item[0][1], [s[2] for s in share], [len(b) // 128 for b in bodies], events)
            mine = res.replies()
            parts = [None] * world if rank == 0 else None
            dist.gather_object(mine, parts, dst=0)
            if rank == 0:
                for p in parts:
                    replies.extend(p)
        sm.sync_commit_timestamp()
        # Owner partition: a rank holds balances only for the accounts it owns.
        local = backend.export_accounts()
        not_mine = ~sm._owner_mask(local)
        stray = sum(int(np.count_nonzero(local[f + w][not_mine])) for f in
                    ("debits_pending", "debits_posted", "credits_pending", "credits_posted") for w in ("_lo", "_hi"))
        stray_t = torch.tensor([stray], dtype=torch.int64, device=sm.comm_device)
        dist.all_reduce(stray_t)
        accounts = sm.export_accounts()
        transfers = sm.export_transfers()
        posted = sm.export_posted()
        if rank == 0:
            oracle = OracleEngine()
            expect = run_oracle(sc, oracle)
            problems = []
            if len(expect) != len(replies):
                problems.append("reply count %d != %d" % (len(replies), len(expect)))
            for i, (a, b) in enumerate(zip(replies, expect)):
                if a != b:
                    problems.append("prepare %d reply differs: got %s expected %s" % (
                        i, np.frombuffer(a, np.uint32).reshape(-1, 2)[:6].tolist(),
                        np.frombuffer(b, np.uint32).reshape(-1, 2)[:6].tolist()))
                    break
            if accounts.tobytes() != oracle.export_accounts().tobytes():
                problems.append("accounts differ")
            if transfers.tobytes() != oracle.export_transfers().tobytes():
                problems.append("transfers differ (%d vs %d)" % (len(transfers), len(oracle.export_transfers())))
            if posted.tobytes() != oracle.export_posted().tobytes():
                problems.append("posted differs")
            if int(stray_t.item()):
                problems.append("%d balance words held by a rank that does not own the account" % int(stray_t.item()))
            if sm.commit_timestamp != oracle.commit_timestamp:
                problems.append("commit_timestamp %d != %d" % (sm.commit_timestamp, oracle.commit_timestamp))
            verdict = {"ok": not problems, "problems": problems, "clean": sm.passes_clean, "dirty": sm.passes_dirty,
                       "split": sm.passes_split, "demoted": int(torch.tensor([sm.demoted]).sum()),
                       "prepares": len(replies), "transfers": int(len(transfers))}
    except Exception:
        verdict = {"ok": False, "problems": [traceback.format_exc()]}
    finally:
        if rank == 0:
            with open(result_path, "w") as f:
                json.dump(verdict, f)
        dist.destroy_process_group()
