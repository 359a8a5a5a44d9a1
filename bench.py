"""Headline benchmark: committed create_transfers per second, bit-exact, on MI355X.

Workload (BASELINE.json configs[1], "C2"): 1M accounts, 100M uniform-random transfers (dr != cr,
no flags), prepares of 8190 events, synthetic data generated on the GPU (tigerbeetle_amd
k_workload.h, shapes of the reference benchmark client src/benchmark.zig:223-327).

A step = committing all 100M transfers (12,211 prepares) from the post-account-creation state.
`value` is measured with the prepare bodies already resident in HBM when the timed region starts
(tbgpu_commit_device_async, passes of --pass-batches prepares; replies written to HBM): the engine's
own rate.  Between steps the transfer store and balances are restored (untimed), so every step
commits the same 100M transfers.  Each timed step is bracketed by a barrier + torch.cuda.synchronize();
value = transfers committed by all ranks / sum of step times (max over ranks).  `host_path` is the
same commit from registered host memory (tbgpu_commit_pipelined: chunk c+1 crosses PCIe while chunk c
commits, replies back in host memory): the replica's batched call, PCIe both ways inside its timing.

--gpus N: BASELINE.json configs[4] ("C5") on one tbgpu node engine over the N GPUs (run_node): 100M
accounts hash-partitioned by owner, 125M uniform transfers per GPU (1B over 8), the prepares resident
in their source GPU's HBM for `value` (host memory for `host_path`).  Per-GPU work is fixed as N
grows: scaling is weak.

The JSON line also carries:
  roofline      the dominant kernel's algorithmic bytes per launch / its average launch time
                (device clock, inside the timed steps) against 8 TB/s; `traffic` (HBM bytes per
                launch) comes from the PMC_FILE (rocprofv3 PMC passes), with rocprof's mean launch
                time of the same kernel beside it.
  cpu_baseline  the C oracle (reference semantics restated, single thread) timed on this host on
                a bounded prefix of the same workload.
  parity        the same prefix committed on the GPU from a fresh state through the timed path (and
                through the host path) and compared with the oracle byte for byte (replies, every
                account, every transfer); for the full run, every reply empty, no dependent event,
                debits == credits in total.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ctypes_u8 = ctypes.c_uint8
U64_ALL = np.uint64(0xFFFFFFFFFFFFFFFF)
METRIC = "transfers/sec committed (whole node, bit-exact results) + p99 batch latency"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
PCIE_PEAK_GBS = 63.0   # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s spec
# What one H2D stream reaches on this host link (tools/microbench_h2d: hipMemcpyAsync from pinned or
# registered memory on the copy engine, or a kernel pulling mapped host memory: 55.5-57.3 GB/s).
PCIE_MEASURED_GBS = 57.3
# Prepares per pipelined chunk.  C2 and C3 at 64 (C3's in-order sweep grows with the chunk); C4 at
# 128: its ordered run costs about (DAG depth x unit latency) per chunk whatever the chunk's size, so
# larger chunks amortise it (10M C4 transfers: 282M/s at 64, 352M/s at 128, 351M/s at 256, with
# p99 submit-to-reply 5.4 / 7.0 / 9.8 ms; tools/gpu/chunks.sh).
CHUNK_PREPARES = {"c2": 64, "c3": 64, "c3h": 64, "c4": 128}
# The node engine (--gpus N > 1): prepares per source block of a pass.  A node pass has fixed costs a
# single engine's has not (the route plan's host round trip, per-shard import, owner legs, replies,
# each a launch per shard): C2 on two logical shards of one GPU ran at 0.76 / 1.52 / 1.76 G/s in
# 64- / 256- / 512-prepare blocks (1024: 1.76; round 6, profiles/r06/node/lib_ab/).  Per GPU a
# 512-prepare block costs ~1 GB of send buffer and 2 GB of owner-leg regions at N = 8.
NODE_CHUNK_PREPARES = {"c2": 512, "c3": 64, "c3h": 64, "c4": 128}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--latency-steps", type=int, default=2,
                   help="headline steps run again after the timed ones with every pass timed (batch latency)")
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--accounts", type=int, default=None, help="default: 1M (N=1, C2); 100M (N>1, C5)")
    p.add_argument("--transfers", type=int, default=None,
                   help="transfers per GPU; default: 100M (N=1, C2); 125M (N>1, C5: 1B over 8 GPUs)")
    p.add_argument("--batch", type=int, default=8190)
    p.add_argument("--pass-batches", type=int, default=512, help="prepares per device pass (device-resident leg)")
    p.add_argument("--inplace", type=int, default=1,
                   help="1: the device-resident prepares are placed in the engine's log window and committed in "
                        "place (tbgpu_log_window, zero-copy); 0: committed from a separate HBM buffer")
    p.add_argument("--staged-steps", type=int, default=2,
                   help="steps of the same leg from a separate HBM buffer (the copy commit), reported beside it")
    p.add_argument("--chunk-prepares", type=int, default=None,
                   help="prepares per pipelined chunk (host memory -> PCIe -> commit -> reply); default per "
                        "workload: CHUNK_PREPARES")
    p.add_argument("--host-steps", type=int, default=3,
                   help="timed steps of the host path (prepares in registered host memory, PCIe inclusive; 0: skip)")
    p.add_argument("--secondary", type=int, default=10_000_000,
                   help="transfers of the C3 / C4 secondary lines (0: skip)")
    p.add_argument("--secondary-device", type=int, default=100_000_000,
                   help="transfers of the C3 / C4 secondary lines' device-resident leg (in place, as the headline; "
                        "BASELINE.md's 100M; 0: skip)")
    p.add_argument("--cpu-sample", type=int, default=12_285_000, help="transfers in the CPU baseline / parity sample (0: skip)")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--walk-merge", type=int, default=-1,
                   help="heavy limit-account segments the sweep walks merged on one wave at most (-1: the engine's "
                        "default; 0: a wave each)")
    p.add_argument("--workload", default="c2", choices=["c2", "c3", "c3h", "c4"],
                   help="BASELINE.json shape: c2 (headline, default), c3 Zipf + limit accounts, c4 chains + two-phase")
    p.add_argument("--profile", type=int, default=1, help="time kernels with HIP events (roofline)")
    p.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) or gloo (rehearsal on one GPU)")
    p.add_argument("--same-device", action="store_true", help="rehearsal: every rank on cuda:0")
    p.add_argument("--sharded", action="store_true",
                   help="run the multi-GPU protocol even at one rank (rehearses the RCCL code path on one GPU)")
    p.add_argument("--access-mix", type=int, default=1,
                   help="time the validate kernel's access pattern without its logic (roofline.access_mix)")
    p.add_argument("--host-prepares", type=int, default=600,
                   help="prepares committed one per tbgpu_commit call from host memory (the replica's call; 0: skip)")
    p.add_argument("--replica-prepares", type=int, default=2000,
                   help="ops of the replica call path through the C++ mirror (tb_replica_bench; 0: skip)")
    p.add_argument("--write-back", type=int, default=1,
                   help="time the groove write-back per bar at the full stored count and near empty")
    p.add_argument("--engine", default="node", choices=["node", "ranks"],
                   help="--gpus N > 1: 'node' = one tbgpu node engine over the N GPUs (include/tbgpu.h "
                        "tbgpu_config.devices: what a replica binds), 'ranks' = one process per GPU over RCCL "
                        "(tigerbeetle_amd/sharded.py)")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher rehearsal (CPU): every rank reports its place in the process group and exits "
                        "before touching a GPU")
    args = p.parse_args()
    if args.steps < 1:
        p.error("--steps must be at least 1 (the headline is measured over the timed steps)")
    return args


def batches(total, batch):
    q, r = divmod(total, batch)
    return [batch] * q + ([r] if r else [])


def timestamps(lens, start, gap_every=0):
    """Prepare timestamps: t_k = t_{k-1} + 1 + len_k (state_machine.zig:1483-1485), plus the C4
    expiry gaps (tests/harness/configs.py)."""
    from tests.harness.configs import timestamps as ts_gaps
    return ts_gaps(lens, start, gap_every)


def expected_unique(accounts, legs):
    """Expected number of distinct accounts touched by `legs` uniform draws."""
    return accounts * (1.0 - math.exp(-legs / accounts))


def ref_percentile(sorted_ms, p):
    """The reference's percentile pick (src/benchmark.zig:454-471): latencies[len * p / 100 -| 1]."""
    if len(sorted_ms) == 0:
        return float("nan")
    return float(sorted_ms[max(0, len(sorted_ms) * p // 100 - 1)])


def deciles(sorted_ms):
    out = {"p%02d" % (10 * d): round(ref_percentile(sorted_ms, 10 * d), 3) for d in range(11)}
    out["p99"] = round(ref_percentile(sorted_ms, 99), 3)
    return out


def run_host_commits(engine, args, events_dev, t_cursor):
    """The replica's own call pattern: one prepare per tbgpu_commit, body in host memory, reply
    bytes back in host memory (state_machine.zig:508-540 as replica.zig:3654 calls it).  The
    latency includes PCIe both ways; measured with the host clock around each call, first from
    pageable memory, then from memory registered once (tbgpu_register_host: the message pool)."""
    import ctypes
    from tigerbeetle_amd import _lib

    lib = engine.lib
    L = args.batch
    n = min(args.host_prepares, args.transfers // L)
    body = np.ascontiguousarray(engine.to_host(events_dev, n * L * 128))
    out = np.zeros(L * 8, dtype=np.uint8)
    out_len = ctypes.c_uint32(0)
    res = {"prepares": n, "events_per_prepare": L, "call": "tbgpu_commit (one prepare per call, host buffers)"}
    engine.profile_mask(0)  # no HIP event pairs around the kernels
    for mode in ("pageable", "registered"):
        if mode == "registered":
            _lib.check(lib.tbgpu_register_host(engine.h, body.ctypes.data, body.nbytes))
        engine.reset_transfers()
        engine.sync()
        lat = []
        for k in range(n):
            t_cursor += 1 + L
            t0 = time.perf_counter()
            _lib.check(lib.tbgpu_commit(engine.h, 129, t_cursor, ctypes.c_void_p(body.ctypes.data + k * L * 128),
                                        L * 128, out.ctypes.data, out.nbytes, ctypes.byref(out_len)))
            lat.append(time.perf_counter() - t0)
            assert out_len.value == 0, "C2 prepare returned errors"
        lat = np.array(lat[min(20, n // 10):]) * 1e3  # first calls warm the path
        res[mode] = {"transfers_per_s": round(L / (lat.mean() / 1e3), 1), "p50_ms": round(float(np.percentile(lat, 50)), 4),
                     "p99_ms": round(float(np.percentile(lat, 99)), 4), "p100_ms": round(float(lat.max()), 4)}
    # Per-kernel device time of the same calls (HIP event pairs: a separate, shorter run).
    engine.reset_transfers()
    engine.profile_mask(engine.PROF_ALL)
    engine.reset_stats()
    for k in range(min(n, 200)):
        t_cursor += 1 + L
        _lib.check(lib.tbgpu_commit(engine.h, 129, t_cursor, ctypes.c_void_p(body.ctypes.data + k * L * 128),
                                    L * 128, out.ctypes.data, out.nbytes, ctypes.byref(out_len)))
    st = engine.stats()
    res["device_ms_per_call"] = {name: round(st["ms_" + key] / max(1, st["launches_" + key]), 4)
                                 for name, key in (("validate", "validate"), ("resolve", "resolve"), ("apply_legs", "apply"),
                                                   ("flow", "replay"), ("pass_clear", "clear"))}
    _lib.check(lib.tbgpu_unregister_host(engine.h, body.ctypes.data))
    return res, t_cursor + 10


def run_write_back(engine, args, t_cursor, bars=4):
    """The durable replica's groove write-back per bar (tbgpu_checkpoint_delta after each bar of 64
    prepares, as the Zig wrapper's compact does, src/state_machine.zig:542-582): the current state
    is taken as written back (tbgpu_bench_checkpoint_mark), then each bar of fresh C2 transfers is
    committed from host memory and its write-back timed (host clock: device work, the D2H of the
    changed objects and their sort).  Its cost follows the bar's changes, not the stored objects:
    compare the entries taken at different stored counts."""
    L, bar = args.batch, 64
    n = bar * L
    dev = engine.alloc(n * 128)
    out = []
    engine.checkpoint_mark()
    stored = engine.stats()["transfers"]
    for k in range(bars):
        engine.generate_transfers(dev, 10 * args.transfers + k * n, n, args.accounts, seed=args.seed + 7)
        host = engine.to_host(dev, n * 128)
        lens = batches(n, L)
        ts, t_cursor = timestamps(lens, t_cursor + 10)
        rb, _, _ = engine.commit_pipelined(129, ts, lens, host, chunk_batches=bar)
        assert int(rb.sum()) == 0
        t0 = time.perf_counter()
        d = engine.checkpoint_delta(caps=(2 * n, n, n), copy=False)  # views of the registered buffers
        out.append({"ms": round((time.perf_counter() - t0) * 1e3, 3), "accounts": len(d.accounts),
                    "transfers": len(d.transfers)})
    engine.free(dev)
    steady = out[1:] if len(out) > 1 else out  # the first call allocates and registers the buffers
    return {"stored_transfers": int(stored), "bar_prepares": bar, "bars": out,
            "ms_per_bar": round(float(np.mean([b["ms"] for b in steady])), 3),
            "bytes_per_bar": int(np.mean([128 * b["transfers"] + 192 * b["accounts"] for b in steady]))}, t_cursor


def run_replica_path(args, device):
    """The replica's call path from C++ (tigerbeetle_amd/host/replica_bench.cpp, the tb::StateMachine
    mirror): per op, prepare -> prefetch (the body's DMA from the registered message pool starts)
    -> commit -> compact, serially, one C2 prepare of 8190 transfers each (src/vsr/replica.zig:
    3045-3102); without and with the groove write-back in compact: one bar behind (asynchronous), at each
    bar's last op (synchronous: the Zig wrapper's default), one bar behind with the bars of every
    checkpoint op and trigger synchronous (a 1024-slot journal, src/config.zig:136; the Zig wrapper
    with engine_write_back_behind), and one op / a chunk of 4 or 8 ops behind with every bar complete
    at its last op (the reference's one-bar table_mutable bound)."""
    import subprocess
    exe = os.path.join(ROOT, "tigerbeetle_amd", "host", "tb_replica_bench")
    out = {}
    # The write-back shapes call tbgpu_prefetch (--stage) as the replica does before every commit: with a
    # copy-out in flight it stages the body by DMA.
    for name, opts in (("in_memory", []), ("in_memory_staged", ["--stage"]), ("with_write_back", ["--write-back", "--stage"]),
                       ("with_write_back_sync", ["--write-back-sync", "--stage"]),
                       ("with_write_back_behind_checkpoints", ["--write-back", "--checkpoint-journal-slots", "1024", "--stage"]),
                       ("with_write_back_per_op", ["--write-back-per-op", "--stage"]),
                       ("with_write_back_every_4", ["--write-back-every", "4", "--stage"]),
                       ("with_write_back_every_8", ["--write-back-every", "8", "--stage"])):
        cmd = [exe, "--accounts", str(args.accounts), "--prepares", str(args.replica_prepares),
               "--device", str(device)] + opts
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            out[name] = {"error": (r.stdout + r.stderr)[-500:]}
            continue
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
    return out


def run_cpu_baseline(engine, args, acct_lens, acct_ts, events_dev, sample_lens, sample_ts):
    """Oracle (single thread) on the sample; returns (result dict, oracle engine, replies)."""
    from tests.harness.configs import SETTINGS
    from tests.harness.oracle import OracleEngine

    n_acct = args.accounts
    acct_dev = engine.alloc(n_acct * 128)
    wl = SETTINGS[args.workload]
    engine.generate_accounts(acct_dev, 0, n_acct, seed=args.seed, limit_permille=wl["limit_permille"],
                             account_count=n_acct, hot_limited=wl.get("hot_limited", 0))
    acct_events = engine.to_host(acct_dev, n_acct * 128)
    engine.free(acct_dev)
    n_sample = sum(sample_lens)
    events = engine.to_host(events_dev, n_sample * 128)

    oracle = OracleEngine(n_acct, n_sample)
    off = 0
    for L, ts in zip(acct_lens, acct_ts):
        r = oracle.commit(128, ts, acct_events[off * 128:(off + L) * 128].tobytes())
        assert r == b"", "account creation failed on the oracle"
        off += L
    replies = []
    off = 0
    lat = []
    t0 = time.perf_counter()
    for L, ts in zip(sample_lens, sample_ts):
        b0 = time.perf_counter()
        replies.append(oracle.commit(129, ts, events[off * 128:(off + L) * 128].tobytes()))
        lat.append(time.perf_counter() - b0)
        off += L
    dt = time.perf_counter() - t0
    lat = np.array(lat) * 1e3
    return {
        "value": n_sample / dt,
        "unit": "transfers/s",
        "cores": 1,
        "kind": "port",
        "sample": "first %d transfers (%d prepares of %d) of the same workload; C oracle oracle/tb_oracle.c "
                  "(reference semantics restated, in-memory hash-map grooves, no LSM/WAL/network), one thread, "
                  "%s" % (n_sample, len(sample_lens), args.batch, cpu_model()),
        "p99_batch_latency_ms": float(np.percentile(lat, 99)),
        "seconds": dt,
        "c1": run_cpu_c1(engine, args),
    }, oracle, replies


def run_secondary(args, kind, device):
    """BASELINE.json configs[2] (C3) / configs[3] (C4) at 1M accounts and args.secondary transfers,
    measured like the headline (prepares in registered host memory, pipelined chunks, PCIe
    inclusive), with its own roofline; parity: the first 1M transfers committed on a fresh engine
    and compared with the oracle byte for byte (replies, accounts, transfers, posted groove)."""
    from tests.harness.configs import KINDS, SETTINGS, generate, split
    from tests.harness.oracle import OracleEngine
    from tigerbeetle_amd.state_machine import Engine, Options

    wl = SETTINGS[kind]
    args = argparse.Namespace(**dict(vars(args), chunk_prepares=CHUNK_PREPARES[kind]))
    n_acct, n_xfer = 1_000_000, args.secondary
    eng = Engine(Options(accounts_max=n_acct, transfers_max=n_xfer, pass_events_max=args.chunk_prepares * args.batch,
                         pass_batches_max=args.chunk_prepares, device=device, profile=True))
    if args.walk_merge >= 0:
        eng.walk_merge_max(args.walk_merge)
    accts, xfers = generate(eng, kind, n_acct, n_xfer, seed=args.seed)
    a_lens, x_lens = batches(n_acct, args.batch), batches(n_xfer, args.batch)
    a_ts, t_end = timestamps(a_lens, 1_000_000_000)

    def create_accounts(e):
        rb, _, _ = e.commit_pipelined(128, a_ts, a_lens, accts, chunk_batches=args.chunk_prepares)
        assert int(rb.sum()) == 0, "account creation returned errors"

    create_accounts(eng)
    eng.register_host(xfers)
    replies = np.empty(n_xfer * 8, dtype=np.uint8)
    step_ms, t_cursor = [], t_end
    eng.profile_mask(eng.PROF_APPLY | eng.PROF_REPLAY)  # validate on the device clock (no event pair inside its span)
    for step in range(2):  # one warmup, one timed
        eng.reset_transfers()
        ts, t_cursor = timestamps(x_lens, t_cursor + 10, wl["gap_every"])
        if step == 1:
            eng.reset_stats()
        t0 = time.perf_counter()
        rb, _, _ = eng.commit_pipelined(129, ts, x_lens, xfers, chunk_batches=args.chunk_prepares, replies=replies)
        if step == 1:
            step_ms.append((time.perf_counter() - t0) * 1e3)
    stats = eng.stats()
    eng.unregister_host(xfers)
    eng.close()
    per_launch = n_xfer / max(1, stats["span_launches"][0] or stats["launches_validate"])
    # The ordered fallback (tb_flow) has no byte roofline (it is bound by its dependency rounds):
    # the roofline is the validate kernel's; tb_flow's time share is reported beside it.
    roof = roofline(stats, expected_unique(n_acct, 2 * per_launch) / per_launch, per_launch,
                    argparse.Namespace(transfers=n_xfer, steps=1), step_ms[0], None, kernel="tb_transfers_validate")
    roof["flow_ms_share"] = round(stats["ms_replay"] / step_ms[0], 4)

    # Parity: the first 1M transfers (the same prepares, same timestamps) on a fresh engine.
    n_par = min(n_xfer, 1_000_000)
    p_lens = batches(n_par, args.batch)
    p_ts, _ = timestamps(p_lens, t_end + 10, wl["gap_every"])
    oracle = OracleEngine(n_acct, n_par)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    expected = oracle.commit_many(129, p_ts, split(xfers[:n_par * 128], p_lens))
    eng = Engine(Options(accounts_max=n_acct, transfers_max=n_par, pass_events_max=args.chunk_prepares * args.batch,
                         pass_batches_max=args.chunk_prepares, device=device))
    create_accounts(eng)
    rb, rep, _ = eng.commit_pipelined(129, p_ts, p_lens, np.ascontiguousarray(xfers[:n_par * 128]),
                                      chunk_batches=args.chunk_prepares)
    got, off = [], 0
    for L, nb in zip(p_lens, rb):
        got.append(bytes(rep[off * 8:off * 8 + int(nb)]))
        off += L
    parity = {"sample_transfers": n_par, "replies_equal": got == expected,
              "accounts_equal": eng.export_accounts().tobytes() == oracle.export_accounts().tobytes(),
              "transfers_equal": eng.export_transfers().tobytes() == oracle.export_transfers().tobytes(),
              "posted_equal": bool(np.array_equal(eng.export_posted(), oracle.export_posted())),
              "failed_events": sum(len(r) for r in expected) // 8}
    eng.close()
    device_resident = None
    if args.secondary_device:
        device_resident = run_secondary_device(args, kind, device, accts, a_lens, a_ts, t_cursor, oracle, expected,
                                               p_lens, p_ts)
        parity["device_sample_equal"] = device_resident["parity"]["sample_equal"]
    return {"workload": WORKLOAD_TEXT[kind] % (n_acct, n_xfer, args.batch),
            "value": round(n_xfer / (step_ms[0] / 1e3), 1), "unit": "transfers/s", "ms_per_step": round(step_ms[0], 3),
            "input": "registered host memory, %d-prepare pipelined chunks, PCIe inclusive" % args.chunk_prepares,
            "dependent_events": stats["dependent_events"],
            "flow": {k: (round(stats[k], 3) if isinstance(stats[k], float) else stats[k])
                     for k in ("flow_units", "flow_runs", "flow_plan_ms", "flow_run_ms", "bounds_passes", "bounds_units",
                               "bounds_rounds", "bounds_skipped", "bounds_abandoned", "bounds_swept", "sweep_ms",
                               "sweep_loop_ms", "sweep_wait_ms", "walk_segments", "walk_heavy",
                               "walk_heavy_positions", "walk_heavy_windows", "walk_heavy_stops", "walk_heavy_blocks",
                               "walk_heavy_blocked_ms", "walk_longest", "walk_crit_windows",
                               "walk_crit_blocks", "walk_crit_wait_ms", "walk_crit_ms")},
            "flow_phases_ms": flow_phases(stats),
            "roofline": roof, "device_resident": device_resident, "parity": parity}


def run_secondary_device(args, kind, device, accts, a_lens, a_ts, t_cursor, oracle, expected, p_lens, p_ts):
    """The C3 / C4 line with its prepares resident in HBM, as the headline measures C2: BASELINE.md's
    100M transfers generated at their transfer-log positions (tbgpu_log_window, untimed) and committed
    in place with tbgpu_commit_device_async in passes of the line's chunk size; one warmup step and
    one timed step, validate on the device clock, tb_flow (the ordered fallback) timed beside it.
    Parity: the oracle's sample (the first 1M transfers, the same generator indices and timestamps)
    committed in place from the post-account-creation state on the same engine."""
    from tests.harness.configs import KINDS, SETTINGS
    from tigerbeetle_amd.state_machine import Engine, Options

    wl = SETTINGS[kind]
    n_acct, n = 1_000_000, args.secondary_device
    chunk = args.chunk_prepares
    eng = Engine(Options(accounts_max=n_acct, transfers_max=n, pass_events_max=chunk * args.batch,
                         pass_batches_max=chunk, device=device, profile=True))
    try:
        if args.walk_merge >= 0:
            eng.walk_merge_max(args.walk_merge)
        rb, _, _ = eng.commit_pipelined(128, a_ts, a_lens, accts, chunk_batches=chunk)
        assert int(rb.sum()) == 0, "account creation returned errors"
        ct_accounts = eng.commit_timestamp
        lens = batches(n, args.batch)
        res_dev = eng.alloc(n * 8)
        rb_dev = eng.alloc((len(lens) + 2) * 4)
        gen = dict(seed=args.seed, kind=KINDS[kind], limit_permille=wl["limit_permille"],
                   hot_limited=wl.get("hot_limited", 0))

        def place(count):
            eng.reset_transfers()
            window = eng.log_window(count)
            eng.generate_transfers(window, 0, count, n_acct, **gen)
            eng.sync()
            return window

        step_ms = []
        for step in range(2):  # one warmup, one timed
            window = place(n)
            ts, t_cursor = timestamps(lens, t_cursor + 10, wl["gap_every"])
            if step == 1:
                breakdown = eng.stats()
                eng.reset_stats()
                eng.profile_mask(eng.PROF_APPLY | eng.PROF_PASS | eng.PROF_REPLAY)
            else:
                eng.profile_mask(eng.PROF_ALL)
            t0 = time.perf_counter()
            eng.commit_device_async(129, ts, lens, window, res_dev, rb_dev)
            eng.sync()
            if step == 1:
                step_ms.append((time.perf_counter() - t0) * 1e3)
        stats = eng.stats()
        n_failed = int(eng.to_host(rb_dev, len(lens) * 4).view(np.uint32).sum()) // 8
        accs = eng.export_accounts()

        def total(field):
            return sum(int(x) for x in accs[field + "_lo"]) + (sum(int(x) for x in accs[field + "_hi"]) << 64)

        full_ok = bool(stats["transfers"] == n - n_failed and total("debits_posted") == total("credits_posted")
                       and total("debits_pending") == total("credits_pending"))
        n_val = (stats.get("span_launches") or [0])[0] or stats["launches_validate"]
        per_launch = n / max(1, n_val)
        roof = roofline(stats, expected_unique(n_acct, 2 * per_launch) / per_launch, per_launch,
                        argparse.Namespace(transfers=n, steps=1), step_ms[0], breakdown, kernel="tb_transfers_validate",
                        in_place=True)
        pass_lat = np.sort(np.array(eng.pass_latencies()))

        # Parity: the oracle's sample, in place, from the post-account-creation state.
        n_par = sum(p_lens)
        window = place(n_par)
        eng.set_commit_timestamp(ct_accounts)
        eng.commit_device_async(129, p_ts, p_lens, window, res_dev, rb_dev)
        eng.sync()
        rbp = eng.to_host(rb_dev, len(p_lens) * 4).view(np.uint32)
        results = eng.to_host(res_dev, n_par * 8)
        got, off = [], 0
        for L, nb in zip(p_lens, rbp):
            got.append(bytes(results[off * 8:off * 8 + int(nb)]))
            off += L
        sample_equal = bool(got == expected
                            and eng.export_accounts().tobytes() == oracle.export_accounts().tobytes()
                            and eng.export_transfers(cap=n_par).tobytes() == oracle.export_transfers().tobytes()
                            and np.array_equal(eng.export_posted(), oracle.export_posted()))
        for ptr in (res_dev, rb_dev):
            eng.free(ptr)
    finally:
        eng.close()
    return {"value": round(n / (step_ms[0] / 1e3), 1), "unit": "transfers/s", "ms_per_step": round(step_ms[0], 3),
            "transfers": n, "pass_prepares": chunk,
            "input": "prepares resident in HBM at their transfer-log positions, committed in place "
                     "(tbgpu_log_window + tbgpu_commit_device_async), %d-prepare passes" % chunk,
            "p99_batch_latency_ms": round(ref_percentile(pass_lat, 99), 3) if len(pass_lat) else None,
            "dependent_events": stats["dependent_events"], "failed_events": n_failed,
            "validate_ms": round(stats["span_ms"][0], 3) if stats.get("span_ms") else None,
            "tb_flow_ms": round(stats["ms_replay"], 3),
            "flow_ms_share": round(stats["ms_replay"] / step_ms[0], 4),
            "flow_phases_ms": flow_phases(stats),
            "roofline": roof,
            "parity": {"sample_transfers": n_par, "sample_equal": sample_equal, "full_run_properties": full_ok}}


def run_cpu_c1(engine, args):
    """BASELINE.json configs[0] (scripts/benchmark.sh, src/benchmark.zig:22-24): 10k accounts, 1M
    uniform transfers in prepares of 8190, committed by the oracle on one host core."""
    from tests.harness.configs import generate, split
    from tests.harness.oracle import OracleEngine

    n_acct, n_xfer = 10_000, 1_000_000
    accts, xfers = generate(engine, "c2", n_acct, n_xfer, seed=args.seed)
    a_lens, x_lens = batches(n_acct, args.batch), batches(n_xfer, args.batch)
    a_ts, t = timestamps(a_lens, 10**12)
    x_ts, _ = timestamps(x_lens, t + 10)
    oracle = OracleEngine(n_acct, n_xfer)
    assert all(r == b"" for r in oracle.commit_many(128, a_ts, split(accts, a_lens)))
    bodies = split(xfers, x_lens)
    lat = []
    t0 = time.perf_counter()
    for ts, body in zip(x_ts, bodies):
        b0 = time.perf_counter()
        assert oracle.commit(129, ts, body) == b"", "C1 transfer failed on the oracle"
        lat.append(time.perf_counter() - b0)
    dt = time.perf_counter() - t0
    lat = np.sort(np.array(lat) * 1e3)
    return {"value": round(n_xfer / dt, 1), "unit": "transfers/s", "cores": 1, "kind": "port",
            "sample": "C1 in full: 10000 accounts, 1000000 transfers, %d prepares of %d" % (len(x_lens), args.batch),
            "p99_batch_latency_ms": round(ref_percentile(lat, 99), 3)}


def bind_local_numa(device):
    """Run this process on the CPUs of its GPU's NUMA node (those it may use), before the prepare
    bodies are allocated in host memory: their pages then sit on the socket whose PCIe root the GPU
    hangs off, and with N ranks each rank's H2D reads its own socket's memory.  Returns the node, or
    None when the topology is not visible (nothing changes)."""
    import torch
    try:
        p = torch.cuda.get_device_properties(device)
        bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open("/sys/bus/pci/devices/%s/numa_node" % bdf) as f:
            node = int(f.read())
        if node < 0:
            return None
        cpus = set()
        with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        allowed = os.sched_getaffinity(0) & cpus
        if not allowed:
            return None
        os.sched_setaffinity(0, allowed)
        return node
    except (OSError, ValueError, RuntimeError, AttributeError, AssertionError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return "host CPU: %s, nproc %d" % (line.split(":", 1)[1].strip(), os.cpu_count())
    except OSError:
        pass
    return "nproc %d" % os.cpu_count()


# The rocprofv3 evidence behind `roofline.traffic` (tools/gpu/archive/r04_prof.sh -> tools/perf_pmc.py): per
# kernel, HBM bytes per committed transfer from FETCH_SIZE / WRITE_SIZE passes and rocprof's mean
# launch time, for the headline leg (64-prepare chunks from host memory) and for device-resident
# passes.  It lives outside profiles/ so it travels to the GPU box with the tree.
PMC_FILE = os.path.join("perf", "pmc_r06.json")


def load_pmc(leg, kernel, transfers_per_launch):
    """`traffic` fields of the roofline from PMC_FILE: HBM bytes per launch of `kernel` (raw FETCH_SIZE +
    WRITE_SIZE per transfer x this run's transfers per launch), the doubled-FETCH figure, and rocprof's
    mean launch time of the profiled launches.  Missing file or kernel: says so loudly (stderr and the
    `traffic_error` field) and leaves traffic null."""
    path = os.path.join(ROOT, PMC_FILE)
    try:
        d = json.load(open(path))
        k = d["legs"][leg]["kernels"][kernel]
        lt = d["legs"][leg]["launch_transfers"]
    except (OSError, ValueError, KeyError) as e:
        msg = "bench.py: no PMC traffic for %s/%s in %s (%s: %s)" % (leg, kernel, PMC_FILE, type(e).__name__, e)
        print(msg, file=sys.stderr, flush=True)
        return {"traffic": None, "traffic_error": msg}
    out = {"traffic": round(k["raw_per_transfer"] * transfers_per_launch),
           "traffic_fetch_x2": round(k["fetch_x2_per_transfer"] * transfers_per_launch),
           "traffic_per_transfer": k["raw_per_transfer"], "traffic_fetch_x2_per_transfer": k["fetch_x2_per_transfer"],
           "traffic_source": "%s legs.%s (rocprofv3 FETCH_SIZE + WRITE_SIZE, separate passes; %s)" % (
               PMC_FILE, leg, d.get("source", ""))}
    if k.get("rocprof_avg_ms"):
        out["rocprof_avg_launch_ms"] = k["rocprof_avg_ms"]
        out["rocprof_launch_transfers"] = lt
    return out


WORKLOAD_TEXT = {
    "c2": "C2 (BASELINE.json configs[1]): %d accounts, %d uniform transfers/GPU, no flags, prepares of %d",
    "c3": "C3 (BASELINE.json configs[2]): %d accounts (10%% debits_must_not_exceed_credits, funded by a bank "
          "account), %d transfers with Zipf(1.2) dr/cr, prepares of %d",
    "c3h": "C3, adversarial (BASELINE.json configs[2] with the hottest Zipf rank limited too): %d accounts (10%% "
           "debits_must_not_exceed_credits plus the hottest account, funded by a bank account), %d transfers with "
           "Zipf(1.2) dr/cr, prepares of %d",
    "c4": "C4 (BASELINE.json configs[3]): %d accounts, %d transfers: ~20%% in linked chains (5%% chain-breaking), "
          "30%% pending with 0..10 s timeouts, 15%% post/void of earlier transfers, 0.5%% balancing, a 2 s "
          "timestamp gap every 64 prepares; prepares of %d",
}


def launch_ranks(n):
    """`--gpus N` without a launcher around it: start N rank processes of this same command line
    (torch.distributed.run, rendezvous on 127.0.0.1) before any GPU call, and exit with their code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def launch_check(args, world, rank):
    """Every rank joins the process group (gloo, CPU) and rank 0 prints who came: the launcher's
    rehearsal, with no GPU call anywhere."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(got, torch.tensor([rank, world], dtype=torch.int64))
        ranks = sorted(int(g[0]) for g in got)
        worlds = sorted(set(int(g[1]) for g in got))
        dist.destroy_process_group()
    else:
        ranks, worlds = [0], [1]
    if rank == 0:
        print(json.dumps({"launch_check": True, "gpus": args.gpus, "engine": args.engine, "world": world,
                          "ranks": ranks, "worlds": worlds}), flush=True)


def main():
    args = parse()
    if args.chunk_prepares is None:
        node = args.gpus > 1 and args.engine == "node"
        args.chunk_prepares = (NODE_CHUNK_PREPARES if node else CHUNK_PREPARES)[args.workload]
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and args.engine == "ranks" and not launched:
        sys.exit(launch_ranks(args.gpus))
    if args.launch_check:
        return launch_check(args, world, rank)
    if launched and world > 1 and world != args.gpus:
        raise SystemExit("bench.py: launched with %d ranks but --gpus %d" % (world, args.gpus))
    if args.gpus > 1 and args.engine == "node":
        # The node engine keeps three streams per shard (copy, route, engine) and the sequencer's on the
        # first device: with HIP's default of 4 hardware queues per device the sequencer's stream shares
        # a queue with shard 0's engine stream and waits behind its routed part.  Read by the HIP
        # runtime when it starts (no HIP call has been made yet); an explicit setting is kept, except
        # below 8 for logical shards on one device (their streams all share that device's queues: C3
        # on two logical shards ran at 253 M/s with the box's exported 4, 356 with 8).
        cur = os.environ.get("GPU_MAX_HW_QUEUES")
        if cur is None or (args.same_device and cur.isdigit() and int(cur) < 8):
            os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch
    import torch.distributed as dist

    if args.accounts is None:
        args.accounts = 100_000_000 if max(world, args.gpus) > 1 else 1_000_000
    if args.transfers is None:
        args.transfers = 125_000_000 if max(world, args.gpus) > 1 else 100_000_000
    if args.gpus > 1 and args.engine == "node":
        return run_node(args, world, rank)
    if world > 1 or args.sharded:
        assert args.workload == "c2", "the multi-GPU bench runs the C5 shape (uniform, no flags)"
        if args.same_device:
            local_rank = 0
        torch.cuda.set_device(local_rank)
        args.numa_node = bind_local_numa(local_rank)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.dist_backend)
        return run_sharded(args, world, rank, local_rank)

    def barrier():
        if world > 1:
            dist.barrier()

    def allmax(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    from tests.harness.configs import KINDS, SETTINGS
    args.numa_node = bind_local_numa(local_rank)
    from tigerbeetle_amd.state_machine import Engine, Options

    wl = SETTINGS[args.workload]
    pass_events = args.pass_batches * args.batch
    engine = Engine(Options(accounts_max=args.accounts, transfers_max=args.transfers + 6 * 64 * args.batch,
                            pass_events_max=pass_events, pass_batches_max=args.pass_batches, device=local_rank,
                            profile=bool(args.profile)))
    if args.walk_merge >= 0:
        engine.walk_merge_max(args.walk_merge)
    seed = args.seed + 1000003 * rank  # each rank: its own ledger shard

    # -- accounts (create_accounts through the engine) --------------------------------------
    acct_lens = batches(args.accounts, args.batch)
    acct_ts, t_end = timestamps(acct_lens, 1_000_000_000)
    acct_dev = engine.alloc(args.accounts * 128)
    engine.generate_accounts(acct_dev, 0, args.accounts, seed=seed, limit_permille=wl["limit_permille"],
                             account_count=args.accounts, hot_limited=wl.get("hot_limited", 0))
    res_dev = engine.alloc(max(args.accounts, args.transfers) * 8)
    rb_dev = engine.alloc(max(len(acct_lens), args.transfers // args.batch + 2) * 4)
    engine.commit_device_async(128, acct_ts, acct_lens, acct_dev, res_dev, rb_dev)
    engine.sync()
    rb = engine.to_host(rb_dev, len(acct_lens) * 4).view(np.uint32)
    assert rb.sum() == 0, "account creation returned errors"
    engine.free(acct_dev)

    # -- transfers (synthetic, resident in HBM) ----------------------------------------------
    xfer_lens = batches(args.transfers, args.batch)
    events_dev = engine.alloc(args.transfers * 128)
    engine.generate_transfers(events_dev, 0, args.transfers, args.accounts, seed=seed, kind=KINDS[args.workload],
                              limit_permille=wl["limit_permille"], hot_limited=wl.get("hot_limited", 0))
    engine.sync()

    def place(dst, count=None):
        """The same prepares (same generator, same seed) at `dst`: the log window for an in-place
        commit (each committed record is stamped there, so every step places them afresh, untimed)."""
        engine.generate_transfers(dst, 0, count or args.transfers, args.accounts, seed=seed, kind=KINDS[args.workload],
                                  limit_permille=wl["limit_permille"], hot_limited=wl.get("hot_limited", 0))

    def headline_input(count=None):
        """Reset the transfer store; the prepares' device address for the next commit."""
        engine.reset_transfers()
        if not args.inplace:
            return events_dev
        window = engine.log_window(count or args.transfers)
        place(window, count)
        return window

    # -- headline: the prepares already resident in HBM (the measurement rule: inputs in HBM when
    # the timed region starts), tbgpu_commit_device_async in passes of pass_batches prepares — in
    # place: the prepares sit at their transfer-log positions (tbgpu_log_window), where a replica's
    # DMA or a peer would put them.  Each step commits all of them from the post-account-creation
    # state; bracketed by barrier + sync.
    step_ms, issue_ms, sync_ms = [], [], []
    t_cursor = t_end
    engine.profile_mask(engine.PROF_ALL)  # warmup: every kernel's HIP-event time (the breakdown)
    breakdown = None
    for step in range(args.warmup + args.steps):
        timed = step >= args.warmup
        src = headline_input()
        ts, t_cursor = timestamps(xfer_lens, t_cursor + 10, wl["gap_every"])
        if timed and step == args.warmup:
            if args.warmup:
                breakdown = engine.stats()
            engine.reset_stats()
            # The timed steps stamp validate's, resolve's and apply's launch spans on the device
            # clock and record no HIP event pair: a pair on the stream holds the next launch back by a
            # few microseconds (the bench's former pass / apply / flow pairs cost 3.8 % of a step,
            # tools/gpu/prof_cost.py, profiles/r06/prof_cost.log).
            # (C3 / C4: tb_flow's pair stays — its share of the step is part of the line.)
            engine.profile_mask(engine.PROF_SPANS | (engine.PROF_REPLAY if args.workload != "c2" else 0))
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        engine.commit_device_async(129, ts, xfer_lens, src, res_dev, rb_dev)
        t_issue = time.perf_counter()
        engine.sync()
        t_sync = time.perf_counter()
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        if timed:
            step_ms.append(allmax(dt * 1e3))
            issue_ms.append((t_issue - t0) * 1e3)
            sync_ms.append((t_sync - t0) * 1e3)
    stats = engine.stats()
    # The batch latency: the same steps again, each pass between a HIP event pair (not timed).
    engine.reset_stats()
    engine.profile_mask(engine.PROF_PASS)
    for _ in range(args.latency_steps):
        src = headline_input()
        ts, t_cursor = timestamps(xfer_lens, t_cursor + 10, wl["gap_every"])
        engine.commit_device_async(129, ts, xfer_lens, src, res_dev, rb_dev)
        engine.sync()
    pass_lat = engine.pass_latencies()
    rb = engine.to_host(rb_dev, len(xfer_lens) * 4).view(np.uint32)
    n_failed = int(rb.sum()) // 8

    # -- the same leg from a separate HBM buffer (the copy commit: kernel 1 stores each record) ------
    staged = None
    if args.inplace and args.staged_steps:
        s_ms = []
        engine.profile_mask(engine.PROF_APPLY | engine.PROF_PASS | engine.PROF_REPLAY)
        s_stats0 = engine.stats()
        for step in range(args.staged_steps):
            engine.reset_transfers()
            ts, t_cursor = timestamps(xfer_lens, t_cursor + 10, wl["gap_every"])
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            engine.commit_device_async(129, ts, xfer_lens, events_dev, res_dev, rb_dev)
            engine.sync()
            torch.cuda.synchronize()
            barrier()
            s_ms.append(allmax((time.perf_counter() - t0) * 1e3))
        s_stats = engine.stats()
        s_total = sum(s_ms)
        s_val = max(1, s_stats["span_launches"][0] - s_stats0["span_launches"][0]) if s_stats.get("span_launches") else 0
        staged = {"value": round(args.transfers * world * args.staged_steps / (s_total / 1e3), 1), "unit": "transfers/s",
                  "steps": args.staged_steps, "ms_per_step": round(s_total / args.staged_steps, 3),
                  "definition": "the same prepares committed from a separate HBM buffer (kernel 1 copies each record "
                                "into the log) instead of in place",
                  "validate_avg_launch_ms": round((s_stats["span_ms"][0] - s_stats0["span_ms"][0]) / s_val, 4)
                  if s_val else None,
                  "replies_equal_to_in_place": bool(int(engine.to_host(rb_dev, len(xfer_lens) * 4).view(np.uint32).sum())
                                                    // 8 == n_failed)}

    # -- the host path: the same prepares from registered host memory, PCIe both ways (the replica's
    # batched call, tbgpu_commit_pipelined: chunk c+1 crosses PCIe while chunk c commits) ---------
    host_path = None
    n_failed_host = n_failed
    if args.host_steps:
        host_events = engine.to_host(events_dev, args.transfers * 128)
        engine.register_host(host_events)
        replies = np.empty(args.transfers * 8, dtype=np.uint8)
        h_ms, lat_all = [], []
        engine.profile_mask(engine.PROF_ALL)
        h_breakdown = None
        for step in range(1 + args.host_steps):
            engine.reset_transfers()
            ts, t_cursor = timestamps(xfer_lens, t_cursor + 10, wl["gap_every"])
            if step == 1:
                h_breakdown = engine.stats()
                engine.reset_stats()
                engine.profile_mask(engine.PROF_APPLY | engine.PROF_REPLAY)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rb_h, _, lat = engine.commit_pipelined(129, ts, xfer_lens, host_events, chunk_batches=args.chunk_prepares,
                                                   latency=True, replies=replies)
            torch.cuda.synchronize()
            if step >= 1:
                h_ms.append((time.perf_counter() - t0) * 1e3)
                lat_all.append(lat)
        h_stats = engine.stats()
        n_failed_host = int(rb_h.sum()) // 8
        engine.unregister_host(host_events)
        del host_events
        h_total = sum(h_ms)
        h_lat = np.sort(np.concatenate(lat_all))
        n_val = (h_stats.get("span_launches") or [0])[0] or h_stats["launches_validate"]
        per_launch_h = args.transfers / max(1, n_val / args.host_steps)
        u_h = expected_unique(args.accounts, 2 * per_launch_h) / per_launch_h
        pcie_gbs = args.transfers * 128 * args.host_steps / (h_total / 1e3) / 1e9
        host_path = {
            "value": round(args.transfers * args.host_steps / (h_total / 1e3), 1), "unit": "transfers/s",
            "steps": args.host_steps, "warmup": 1, "ms_per_step": round(h_total / args.host_steps, 3),
            "chunk_prepares": args.chunk_prepares,
            "definition": "tbgpu_commit_pipelined from registered host memory (the replica's message pool): PCIe "
                          "H2D of the bodies and the reply D2H inside the timed region, %d-prepare chunks, 3 in flight"
                          % args.chunk_prepares,
            "p99_batch_latency_ms": round(ref_percentile(h_lat, 99), 3),
            "batch_latency_ms": dict(deciles(h_lat), definition=(
                "per prepare, submit to reply: from the start of its chunk's PCIe copy to its reply landing in host "
                "memory (device clock); percentiles by src/benchmark.zig:454-471")),
            "pcie": {"h2d_bytes_per_transfer": 128, "achieved": round(pcie_gbs, 2), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                     "frac": round(pcie_gbs / PCIE_PEAK_GBS, 4), "measured_ceiling": PCIE_MEASURED_GBS,
                     "frac_of_measured": round(pcie_gbs / PCIE_MEASURED_GBS, 4),
                     "note": "host link (PCIe Gen5 x16, MI355X_MICROARCH.md): the bound of this path"},
            "roofline": roofline(h_stats, u_h, per_launch_h, argparse.Namespace(transfers=args.transfers,
                                                                                steps=args.host_steps),
                                 h_total, h_breakdown, kernel="tb_transfers_validate", pmc_leg="headline"),
        }
    write_back = None
    if rank == 0 and world == 1 and args.write_back and args.workload == "c2":
        at_full, t_cursor = run_write_back(engine, args, t_cursor)
        engine.reset_transfers()
        at_empty, t_cursor = run_write_back(engine, args, t_cursor)
        write_back = {"definition": "tbgpu_checkpoint_delta per bar of 64 C2 prepares (524,160 transfers), host "
                                    "clock: device work + D2H of the changed objects into registered buffers; "
                                    "ms_per_bar over the bars after the first (which allocates the buffers)",
                      "at_stored": [at_full, at_empty]}

    # -- full-run checks (size-independent properties) of the last timed step ---------------------
    # (the write-back leg committed other transfers since: re-run one untimed step to check them)
    src = headline_input()
    ts, t_cursor = timestamps(xfer_lens, t_cursor + 10, wl["gap_every"])
    engine.commit_device_async(129, ts, xfer_lens, src, res_dev, rb_dev)
    engine.sync()
    rb = engine.to_host(rb_dev, len(xfer_lens) * 4).view(np.uint32)
    accts = engine.export_accounts()
    check_stats = engine.stats()

    def total(field):
        return sum(int(x) for x in accts[field + "_lo"]) + (sum(int(x) for x in accts[field + "_hi"]) << 64)

    dpost, cpost = total("debits_posted"), total("credits_posted")
    # C2: every transfer commits.  Every config: each committed transfer is one record; debits equal
    # credits in total, posted and pending.
    full_ok = bool(check_stats["transfers"] == args.transfers - n_failed and dpost == cpost and dpost > 0
                   and total("debits_pending") == total("credits_pending") and len(accts) == args.accounts
                   and (n_failed == 0 or args.workload != "c2") and int(rb.sum()) // 8 == n_failed
                   and n_failed_host == n_failed)

    total_ms = sum(step_ms)
    n_total = args.transfers * world * args.steps
    value = n_total / (total_ms / 1e3)

    # -- roofline: the dominant kernel of the timed steps (validate, device clock) ----------------
    n_val = (stats.get("span_launches") or [0])[0] or stats["launches_validate"]
    per_launch_transfers = args.transfers / max(1, n_val / max(1, args.steps))
    u_over_t = expected_unique(args.accounts, 2 * per_launch_transfers) / per_launch_transfers
    # The ordered fallback (tb_flow) has no byte roofline (its dependency rounds bound it): the
    # roofline is the validate kernel's, with tb_flow's share of the time beside it.
    roof = roofline(stats, u_over_t, per_launch_transfers, args, total_ms, breakdown, kernel="tb_transfers_validate",
                    pmc_leg="device", in_place=bool(args.inplace))
    if roof is not None and args.workload != "c2":
        roof["flow_ms_share"] = round(stats["ms_replay"] / total_ms, 4)

    # -- the validate kernel against its own access pattern, measured live (rank 0, N=1) ------
    if rank == 0 and world == 1 and args.access_mix and roof and roof["kernel"] == "tb_transfers_validate":
        roof["access_mix"] = access_mix(engine, per_launch_transfers, roof["avg_launch_ms"])
        if host_path and host_path["roofline"]:
            hr = host_path["roofline"]
            hr["access_mix"] = access_mix(engine, hr["transfers_per_launch"], hr["avg_launch_ms"])

    # -- CPU baseline + bit-exact sample parity (rank 0, N=1 only) ---------------------------
    cpu = None
    parity = {"full_run_properties": full_ok}
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        sample_lens = batches(min(args.cpu_sample, args.transfers), args.batch)
        sample_ts, t_cursor = timestamps(sample_lens, t_cursor + 10, wl["gap_every"])
        cpu, oracle, expected = run_cpu_baseline(engine, args, acct_lens, acct_ts, events_dev, sample_lens, sample_ts)
        n_sample = sum(sample_lens)

        def got_replies(rb, results):
            got, off = [], 0
            for L, nb in zip(sample_lens, rb):  # sparse replies at the prepare's event offset
                got.append(bytes(results[off * 8:off * 8 + int(nb)]))
                off += L
            return got

        # 1. The headline's own timed path: the sample resident in HBM, tbgpu_commit_device_async
        # (in place when the headline is).
        ct0 = engine.commit_timestamp
        src = headline_input(n_sample)
        engine.commit_device_async(129, sample_ts, sample_lens, src, res_dev, rb_dev)
        engine.sync()
        rb = engine.to_host(rb_dev, len(sample_lens) * 4).view(np.uint32)
        results = engine.to_host(res_dev, n_sample * 8)
        acc_equal = engine.export_accounts().tobytes() == oracle.export_accounts().tobytes()
        xfer_equal = engine.export_transfers(cap=n_sample).tobytes() == oracle.export_transfers().tobytes()
        parity.update({"sample_transfers": n_sample, "replies_equal": got_replies(rb, results) == expected,
                       "accounts_equal": acc_equal, "transfers_equal": xfer_equal,
                       "sample_path": "tbgpu_commit_device_async, %d-prepare passes%s (the timed path)" % (
                           args.pass_batches, ", in place (tbgpu_log_window)" if args.inplace else "")})
        # 2. The host path: tbgpu_commit_pipelined from registered host memory (the same timestamps:
        # the commit timestamp goes back to where the first run started, as a replica's would).
        engine.reset_transfers()
        engine.set_commit_timestamp(ct0)
        sample_host = engine.to_host(events_dev, n_sample * 128)
        engine.register_host(sample_host)
        rb, results, _ = engine.commit_pipelined(129, sample_ts, sample_lens, sample_host,
                                                 chunk_batches=args.chunk_prepares)
        engine.unregister_host(sample_host)
        del sample_host
        parity["host_path_sample_equal"] = bool(
            got_replies(rb, results) == expected
            and engine.export_accounts().tobytes() == oracle.export_accounts().tobytes()
            and engine.export_transfers(cap=n_sample).tobytes() == oracle.export_transfers().tobytes())
        cpu.pop("seconds")

    host = None
    if rank == 0 and world == 1 and args.host_prepares > 0:
        host, t_cursor = run_host_commits(engine, args, events_dev, t_cursor)

    # The C3/C4 lines run on an engine of their own: the headline engine (its 100M-transfer log and
    # index, the resident prepares) is released first, so they run on the same memory a standalone
    # `--workload c3|c4` run gets.
    for ptr in (events_dev, res_dev, rb_dev):
        engine.free(ptr)
    engine.close()
    replica_path = None
    if rank == 0 and world == 1 and args.replica_prepares > 0:
        replica_path = run_replica_path(args, local_rank)
    secondary = {}
    if rank == 0 and world == 1 and args.workload == "c2" and args.secondary:
        for kind in ("c3", "c3h", "c4"):
            secondary[kind] = run_secondary(args, kind, local_rank)

    pass_lat = np.sort(np.array(pass_lat)) if len(pass_lat) else np.array([float("nan")])
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "transfers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(total_ms / args.steps, 3),
        "step_ms": [round(x, 3) for x in step_ms], "issue_ms": [round(x, 3) for x in issue_ms],
        "engine_sync_ms": [round(x, 3) for x in sync_ms],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128",
        "data": "synthetic (generated on the GPU in the reference benchmark's shapes, resident in HBM before timing)",
        "config": {"workload": WORKLOAD_TEXT[args.workload] % (args.accounts, args.transfers, args.batch),
                   "prepares_per_step": len(xfer_lens), "pass_prepares": args.pass_batches,
                   "input": ("prepare bodies resident in HBM when the timed region starts, placed at their transfer-log "
                             "positions and committed in place (tbgpu_log_window + tbgpu_commit_device_async; the same "
                             "leg from a separate buffer is `device_resident_staged`)" if args.inplace else
                             "prepare bodies resident in HBM when the timed region starts (tbgpu_commit_device_async)")
                            + "; replies written to HBM; the PCIe-inclusive rate is `host_path`",
                   "host_numa_node": args.numa_node, "parallelism": "single"},
        "p99_batch_latency_ms": round(ref_percentile(pass_lat, 99), 3),
        "batch_latency_ms": dict(deciles(pass_lat), definition=(
            "per prepare, commit to reply: its device pass's duration (a prepare's reply is complete when its "
            "%d-prepare pass is; device clock, HIP events around each pass, in %d steps run after the timed "
            "ones so that no event pair sits among the timed launches); percentiles by "
            "src/benchmark.zig:454-471" % (args.pass_batches, args.latency_steps))),
        "host_path": host_path,
        "device_resident_staged": staged,
        "dependent_events": stats["dependent_events"],
        "flow": {k: (round(stats[k], 3) if isinstance(stats[k], float) else stats[k])
                 for k in ("flow_units", "flow_runs", "flow_run_units", "flow_plan_ms", "flow_run_ms", "bounds_passes",
                           "bounds_units", "bounds_rounds", "bounds_skipped", "bounds_abandoned", "bounds_swept",
                           "sweep_ms", "sweep_loop_ms", "sweep_wait_ms", "flow_exec_ms", "walk_segments",
                           "walk_heavy", "walk_heavy_positions", "walk_heavy_windows", "walk_heavy_stops",
                           "walk_heavy_blocks", "walk_heavy_blocked_ms", "walk_longest", "walk_crit_windows",
                           "walk_crit_blocks", "walk_crit_wait_ms", "walk_crit_ms")},
        "flow_phases_ms": flow_phases(stats),
        "failed_events": n_failed,
        "roofline": roof,
        "cpu_baseline": cpu,
        "host_commit": host,
        "replica_path": replica_path,
        "write_back": write_back,
        "secondary": secondary or None,
    }
    # Last, so the end of the line (what a log tail keeps) carries the verdicts.
    for kind, sec in (secondary or {}).items():
        sp = sec["parity"]
        parity[kind + "_sample_equal"] = bool(sp["replies_equal"] and sp["accounts_equal"] and sp["transfers_equal"]
                                              and sp["posted_equal"])
        if sec.get("device_resident"):
            parity[kind + "_device_sample_equal"] = sec["device_resident"]["parity"]["sample_equal"]
    line["parity"] = parity
    line["headline"] = {"value": line["value"], "unit": "transfers/s", "p99_batch_latency_ms": line["p99_batch_latency_ms"],
                        "roofline_frac": roof["frac"] if roof else None,
                        "roofline_frac_in_place_bytes": roof["in_place"]["frac"] if roof and "in_place" in roof else None,
                        "roofline_traffic": roof.get("traffic") if roof else None,
                        "host_path_value": host_path["value"] if host_path else None,
                        "staged_value": staged["value"] if staged else None}
    if rank == 0:
        print(json.dumps(line), flush=True)
    engine.close()
    if world > 1:
        dist.destroy_process_group()


def run_sharded(args, world, rank, local_rank):
    """N>1: BASELINE.json configs[4] ("C5"): 100M accounts hash-partitioned by owner, 1B transfers
    on 8 GPUs — every rank submits 125M (weak scaling: at N=8 the node commits C5's 1B per step).
    Each rank's prepares sit in its own pinned host memory (the replica's message pool); pass p+1
    crosses PCIe on a side stream while pass p is routed and committed: events to their home GPU
    (all-to-all over RCCL), the home's commit, the committed transfers' balance legs to the
    accounts' owners (all-to-all), the result codes back (all-to-all), the replies to host."""
    import torch
    import torch.distributed as dist

    from tigerbeetle_amd.sharded import GpuShard, ShardedStateMachine
    from tigerbeetle_amd.state_machine import Engine, Options

    dev = torch.device("cuda", local_rank)
    pass_events = args.pass_batches * args.batch
    # A home receives about 1/N of every rank's pass: size for imbalance.
    recv_max = int(pass_events * 1.25) + 8192
    engine = Engine(Options(accounts_max=args.accounts, transfers_max=int(args.transfers * 1.05) + recv_max,
                            pass_events_max=recv_max, pass_batches_max=recv_max // 8190 + 2, device=local_rank,
                            profile=bool(args.profile)))
    engine.profile_mask(engine.PROF_VALIDATE | engine.PROF_REPLAY)
    backend = GpuShard(engine, world, events_max=pass_events, device=dev)
    sm = ShardedStateMachine(backend)

    # Accounts: every rank commits the same create_accounts prepares (the immutable fields are
    # replicated; balances start at zero and live on their owners).
    acct_lens = batches(args.accounts, args.batch)
    acct_ts, t_end = timestamps(acct_lens, 1_000_000_000)
    chunk = 2048 * args.batch  # whole prepares per staging chunk (bounded staging for 100M accounts)
    for a0 in range(0, args.accounts, chunk):
        n_a = min(chunk, args.accounts - a0)
        acct = torch.empty((n_a, 128), dtype=torch.uint8, device=dev)
        engine.generate_accounts(acct.data_ptr(), a0, n_a, seed=args.seed)
        lens_a = batches(n_a, args.batch)
        k0 = a0 // args.batch
        res = torch.empty(n_a * 2, dtype=torch.int32, device=dev)
        rb = torch.empty(len(lens_a), dtype=torch.int32, device=dev)
        engine.commit_device_async(128, acct_ts[k0:k0 + len(lens_a)], lens_a, acct.data_ptr(), res.data_ptr(),
                                   rb.data_ptr())
        engine.sync()
        assert int(rb.sum().item()) == 0, "account creation returned errors"
        del acct, res, rb
    sm.commit_timestamp = engine.commit_timestamp

    # Transfers: this rank's share of the global sequence, in pinned host memory.
    gen = torch.empty((args.transfers, 128), dtype=torch.uint8, device=dev)
    engine.generate_transfers(gen.data_ptr(), rank * args.transfers, args.transfers, args.accounts, seed=args.seed)
    engine.sync()
    host = torch.empty((args.transfers, 128), dtype=torch.uint8, pin_memory=True)
    host.copy_(gen)
    del gen
    torch.cuda.synchronize(dev)
    lens = batches(args.transfers, args.batch)
    passes = [lens[i:i + args.pass_batches] for i in range(0, len(lens), args.pass_batches)]
    starts = np.concatenate([[0], np.cumsum([sum(p) for p in passes])]).astype(np.int64)
    bufs = [torch.empty((pass_events, 128), dtype=torch.uint8, device=dev) for _ in range(2)]
    copy_stream = torch.cuda.Stream(dev)
    copied = [torch.cuda.Event() for _ in range(2)]

    def h2d(p):
        n = int(starts[p + 1] - starts[p])
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_stream(torch.cuda.current_stream(dev))  # the buffer's previous pass is done
            bufs[p % 2][:n].copy_(host[starts[p]:starts[p + 1]], non_blocking=True)
            copied[p % 2].record(copy_stream)

    step_ms = []
    t_cursor = t_end
    errors = 0
    for step in range(args.warmup + args.steps):
        timed = step >= args.warmup
        engine.reset_transfers()
        if timed and step == args.warmup:
            engine.reset_stats()
            sm.passes_clean = sm.passes_dirty = 0
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        h2d(0)
        for p, plens in enumerate(passes):
            n = sum(plens)
            mine = None
            for r in range(world):  # rank-major global order of the pass
                ts, t_cursor = timestamps(plens, t_cursor)
                if r == rank:
                    mine = ts
            torch.cuda.current_stream(dev).wait_event(copied[p % 2])
            if p + 1 < len(passes):
                h2d(p + 1)
            out = sm.commit(129, mine, plens, bufs[p % 2][:n])
            errors += int(out.reply_bytes.sum().item())  # the pass's reply sizes back on the host
        torch.cuda.synchronize(dev)
        dist.barrier()
        dt = time.perf_counter() - t0
        if timed:
            t = torch.tensor([dt * 1e3], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            step_ms.append(float(t.item()))
        t_cursor += 10
    stats = engine.stats()

    # Full-run properties: every reply empty, every transfer stored once somewhere, debits ==
    # credits in total (summed over owners), no rank holding balances it does not own.
    local = backend.export_accounts()
    not_mine = ~sm._owner_mask(local)
    stray = sum(int(np.count_nonzero(local[f + w][not_mine])) for f in
                ("debits_pending", "debits_posted", "credits_pending", "credits_posted") for w in ("_lo", "_hi"))
    dpost = sum(int(x) for x in local["debits_posted_lo"]) + (sum(int(x) for x in local["debits_posted_hi"]) << 64)
    cpost = sum(int(x) for x in local["credits_posted_lo"]) + (sum(int(x) for x in local["credits_posted_hi"]) << 64)
    tot = torch.tensor([errors, stats["transfers"], stray], dtype=torch.int64, device=dev)
    dist.all_reduce(tot)
    sums = torch.tensor([[dpost & ((1 << 62) - 1), dpost >> 62], [cpost & ((1 << 62) - 1), cpost >> 62]],
                        dtype=torch.int64, device=dev)
    dist.all_reduce(sums)
    s = sums.cpu().tolist()
    d_all, c_all = s[0][0] + (s[0][1] << 62), s[1][0] + (s[1][1] << 62)
    full_ok = bool(int(tot[0]) == 0 and int(tot[1]) == args.transfers * world and int(tot[2]) == 0
                   and d_all == c_all and d_all > 0 and sm.passes_dirty == 0)

    total_ms = sum(step_ms)
    value = args.transfers * world * args.steps / (total_ms / 1e3)
    recv_per_launch = args.transfers / max(1, stats["launches_validate"] / max(1, args.steps))
    u_over_t = expected_unique(args.accounts, 2 * recv_per_launch) / recv_per_launch
    roof = roofline(stats, u_over_t, recv_per_launch, args, total_ms)
    pcie_gbs = args.transfers * 128 * args.steps / (total_ms / 1e3) / 1e9
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "transfers/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(total_ms / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128",
        "data": "synthetic (generated on the GPU in the reference benchmark's shapes, copied to pinned host memory "
                "before timing)",
        "config": {"workload": "C5 (BASELINE.json configs[4]): %d accounts owner-partitioned by hash(id) over %d GPUs, "
                               "%d uniform transfers submitted per GPU (%d in all), prepares of %d; transfer home = "
                               "hash(id), legs to account owners, all-to-all over RCCL"
                               % (args.accounts, world, args.transfers, args.transfers * world, args.batch),
                   "prepares_per_step": len(lens) * world, "pass_prepares_per_gpu": args.pass_batches,
                   "input": "prepare bodies in pinned host memory per rank; PCIe H2D inside the timed region, "
                            "overlapped with the previous pass",
                   "host_numa_node": args.numa_node,
                   "parallelism": "shard%d (events to home GPU, legs to owner GPU, RCCL all-to-all)" % world},
        "pcie": {"achieved_per_gpu": round(pcie_gbs, 2), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                 "frac": round(pcie_gbs / PCIE_PEAK_GBS, 4), "measured_ceiling": PCIE_MEASURED_GBS,
                 "frac_of_measured": round(pcie_gbs / PCIE_MEASURED_GBS, 4)},
        "passes": {"clean": sm.passes_clean, "dirty": sm.passes_dirty},
        "roofline": roof,
        "cpu_baseline": None,
        "parity": {"full_run_properties": full_ok},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    engine.close()
    dist.destroy_process_group()


def numa_cpus(device):
    """CPUs of the NUMA node a GPU hangs off (None when the topology is not visible)."""
    import torch
    try:
        p = torch.cuda.get_device_properties(device)
        bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open("/sys/bus/pci/devices/%s/numa_node" % bdf) as f:
            node = int(f.read())
        if node < 0:
            return None, None
        cpus = set()
        with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        return node, cpus or None
    except (OSError, ValueError, RuntimeError, AttributeError, AssertionError):
        return None, None


def run_node(args, procs, rank):
    """--gpus N (engine "node"): BASELINE.json configs[4] ("C5") on ONE tbgpu node engine over the N
    GPUs — the handle a replica binds (include/tbgpu.h tbgpu_config.devices, csrc/node.h): 100M
    accounts hash-partitioned by owner, 125M uniform transfers per GPU (1B over 8), every pass of N x
    chunk prepares routed across the GPUs inside the library (homes gather their transfers from the
    sources over xGMI, owners pull their balance legs, sources pull their result codes).

    `value`: the prepares resident in their source GPU's HBM when the timing starts (block d of every
    pass generated on GPU d, read in place by its route kernels), replies back in host memory.
    `host_path`: the same prepares from registered host memory on each GPU's NUMA node, PCIe inside.
    `parity`: one full pass (N x chunk prepares) committed from a fresh state through the timed path
    and compared byte for byte with the oracle, which holds exactly the accounts the sample touches
    (generator records with their create timestamps); then the full-run properties.

    Under torchrun (WORLD_SIZE = N, the driver's launch) rank 0 drives the node and the other ranks
    only take part in the step barriers and the max-over-ranks timing (gloo: they touch no GPU)."""
    import torch
    import torch.distributed as dist

    if procs > 1:
        dist.init_process_group("gloo")
    n_steps = args.warmup + args.steps

    def barrier():
        if procs > 1:
            dist.barrier()

    if rank != 0:  # followers: the barriers of every step, then the timing reduction
        for _ in range(n_steps):
            barrier()
            barrier()
        t = torch.zeros(args.steps, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.destroy_process_group()
        return

    from tests.harness.configs import KINDS, SETTINGS, split
    from tests.harness.oracle import OracleEngine
    from tigerbeetle_amd import _lib
    from tigerbeetle_amd.state_machine import Engine, Options
    from tigerbeetle_amd.types import ACCOUNT_DTYPE, TRANSFER_DTYPE

    wl = SETTINGS[args.workload]
    N = args.gpus
    devices = [0] * N if args.same_device else list(range(N))
    chunk = args.chunk_prepares
    T = args.transfers * N
    engine = Engine(Options(accounts_max=args.accounts, transfers_max=T, pass_events_max=chunk * args.batch,
                            pass_batches_max=chunk, devices=tuple(devices), profile=bool(args.profile)))
    shards = [engine.shard(d) for d in range(N)]
    gen_kw = dict(seed=args.seed, kind=KINDS[args.workload], limit_permille=wl["limit_permille"],
                  hot_limited=wl.get("hot_limited", 0))

    # Prepare k of pass p = k // (N chunk) belongs to source GPU d = (k mod N chunk) // chunk.
    lens = batches(T, args.batch)
    n_prep = len(lens)
    per_pass = N * chunk
    src_of = (np.arange(n_prep) % per_pass) // chunk
    starts = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)

    # The parity sample: the first pass, its transfers generated once on the host side.
    n_sample_prep = min(n_prep, per_pass) if args.cpu_sample > 0 else 0
    n_sample = int(starts[n_sample_prep])
    sample_x = None
    sample_idx = np.zeros(0, dtype=np.uint64)
    if n_sample:
        gen = engine.alloc(n_sample * 128)
        engine.generate_transfers(gen, 0, n_sample, args.accounts, **gen_kw)
        sample_x = engine.to_host(gen, n_sample * 128)
        engine.free(gen)
        x = sample_x.view(TRANSFER_DTYPE)
        # account ids are IdPermutation.inversion: maxInt(u128) - (index + 1), one high word (a post /
        # void may leave them 0: its pending transfer's accounts are used)
        ids_hi = np.concatenate([x["debit_account_id_hi"], x["credit_account_id_hi"]])
        ids_lo = np.concatenate([x["debit_account_id_lo"], x["credit_account_id_lo"]])
        named = (ids_hi | ids_lo) != 0
        assert (ids_hi[named] == U64_ALL).all()
        lo = np.unique(ids_lo[named])
        sample_idx = np.uint64(U64_ALL - 1) - lo

    # Accounts: generated on the first GPU in chunks, committed from host memory; the oracle gets the
    # sample's accounts as created (generator record + create timestamp).
    acct_lens = batches(args.accounts, args.batch)
    acct_ts, t_end = timestamps(acct_lens, 1_000_000_000)
    a_lens_arr, a_ts_arr = np.asarray(acct_lens, dtype=np.uint64), np.asarray(acct_ts, dtype=np.uint64)
    a_chunk = 2048 * args.batch
    dev_buf = engine.alloc(a_chunk * 128)
    oracle_accts = []
    for a0 in range(0, args.accounts, a_chunk):
        n_a = min(a_chunk, args.accounts - a0)
        engine.generate_accounts(dev_buf, a0, n_a, seed=args.seed, limit_permille=wl["limit_permille"],
                                 account_count=args.accounts, hot_limited=wl.get("hot_limited", 0))
        host = engine.to_host(dev_buf, n_a * 128)
        k0 = a0 // args.batch
        lens_a = batches(n_a, args.batch)
        rb, _, _ = engine.commit_pipelined(128, acct_ts[k0:k0 + len(lens_a)], lens_a, host, chunk_batches=chunk)
        assert int(rb.sum()) == 0, "account creation returned errors"
        sel = sample_idx[(sample_idx >= a0) & (sample_idx < a0 + n_a)]
        if len(sel):
            recs = host.view(ACCOUNT_DTYPE)[(sel - np.uint64(a0)).astype(np.int64)].copy()
            k = (sel // np.uint64(args.batch)).astype(np.int64)
            recs["timestamp"] = a_ts_arr[k] - a_lens_arr[k] + np.uint64(1) + sel % np.uint64(args.batch)
            oracle_accts.append(recs)
    engine.free(dev_buf)

    # Transfers: source d's prepares back to back in d's HBM (every pass's block d in turn), generated
    # there; the host path's copy on d's NUMA node, registered once (the replica's message pool).
    dptrs, hptrs = np.zeros(n_prep, dtype=np.uint64), np.zeros(n_prep, dtype=np.uint64)
    dbufs, hbufs, nodes = [], [], []
    for d in range(N):
        mine = np.nonzero(src_of == d)[0]
        n_ev = int(sum(lens[k] for k in mine))
        dbuf = shards[d].alloc(max(n_ev, 1) * 128)
        dbufs.append(dbuf)
        off, i = 0, 0
        while i < len(mine):  # runs of consecutive prepares (one block of a pass) in one launch
            j = i + 1
            while j < len(mine) and mine[j] == mine[j - 1] + 1:
                j += 1
            k0, k1 = int(mine[i]), int(mine[j - 1]) + 1
            for k in range(k0, k1):
                dptrs[k] = dbuf + (off + int(starts[k] - starts[k0])) * 128
            shards[d].generate_transfers(dbuf + off * 128, int(starts[k0]), int(starts[k1] - starts[k0]), args.accounts,
                                         **gen_kw)
            off += int(starts[k1] - starts[k0])
            i = j
        if args.host_steps:
            node, cpus = numa_cpus(devices[d])
            nodes.append(node)
            old_aff = os.sched_getaffinity(0)
            if cpus:
                os.sched_setaffinity(0, cpus)
            buf = np.empty(max(n_ev, 1) * 128, dtype=np.uint8)
            buf[::4096] = 0  # first touch from this GPU's NUMA node
            if cpus:
                os.sched_setaffinity(0, old_aff)
            _lib.check(engine.lib.tbgpu_copy_to_host(shards[d].h, buf.ctypes.data, ctypes.c_void_p(dbuf), n_ev * 128))
            hbufs.append(buf)
            hptrs[np.nonzero(src_of == d)[0]] = dptrs[src_of == d] - np.uint64(dbuf) + np.uint64(buf.ctypes.data)
    replies = np.empty(T * 8, dtype=np.uint8)

    def run_steps(ptrs, warmup, steps, t_cursor):
        ms, lat_all, rb = [], [], None
        for step in range(warmup + steps):
            timed = step >= warmup
            engine.reset_transfers()
            ts, t_cursor = timestamps(lens, t_cursor + 10, wl["gap_every"])
            if step == 0:
                engine.profile_mask(engine.PROF_ALL)
            if timed and step == warmup:
                engine.reset_stats()
                engine.profile_mask(engine.PROF_APPLY | engine.PROF_REPLAY)  # validate on the device clock
            barrier()
            t0 = time.perf_counter()
            rb, lat = engine.commit_pipelined_ptrs(129, ts, lens, ptrs, replies, chunk_batches=chunk, latency=True)
            dt = time.perf_counter() - t0
            barrier()
            if timed:
                ms.append(dt * 1e3)
                lat_all.append(lat)
        return ms, np.sort(np.concatenate(lat_all)) if lat_all else np.array([float("nan")]), rb, t_cursor

    # -- value: device-resident prepares --------------------------------------------------------
    step_ms, lat, rb, t_cursor = run_steps(dptrs, args.warmup, args.steps, t_end)
    stats = engine.stats()
    t = torch.tensor(step_ms, dtype=torch.float64)
    if procs > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step_ms = [float(v) for v in t.tolist()]
    n_failed = int(rb.sum()) // 8
    summ = engine.ledger_summary()
    full_ok = bool((n_failed == 0 or args.workload != "c2") and stats["transfers"] == T - n_failed
                   and summ["debits_posted"] == summ["credits_posted"] and summ["debits_posted"] > 0
                   and summ["debits_pending"] == summ["credits_pending"] and summ["stray"] == 0
                   and summ["accounts"] == args.accounts)
    total_ms = sum(step_ms)
    value = T * args.steps / (total_ms / 1e3)
    n_val = (stats.get("span_launches") or [0])[0] or stats["launches_validate"]
    per_launch = T / max(1, n_val / max(1, args.steps))
    u_over_t = expected_unique(args.accounts, 2 * per_launch) / per_launch
    roof = roofline(stats, u_over_t, per_launch, argparse.Namespace(transfers=T, steps=args.steps), total_ms,
                    kernel="tb_transfers_validate")
    passes = {"clean": stats["node_passes_clean"], "split": stats["node_passes_split"],
              "whole": stats["node_passes_whole"], "sequenced_events": stats["node_sequenced_events"]}

    # -- host path: the same prepares from registered host memory -------------------------------
    host_path = None
    if args.host_steps:
        for buf in hbufs:
            engine.register_host(buf)
        h_ms, h_lat, h_rb, t_cursor = run_steps(hptrs, 1, args.host_steps, t_cursor)
        h_stats = engine.stats()
        for buf in hbufs:
            engine.unregister_host(buf)
        h_summ = engine.ledger_summary()
        full_ok = full_ok and int(h_rb.sum()) == int(rb.sum()) and h_summ == summ
        h_total = sum(h_ms)
        pcie_gbs = T * 128 * args.host_steps / (h_total / 1e3) / 1e9
        n_hv = (h_stats.get("span_launches") or [0])[0] or h_stats["launches_validate"]
        per_launch_h = T / max(1, n_hv / args.host_steps)
        host_path = {
            "value": round(T * args.host_steps / (h_total / 1e3), 1), "unit": "transfers/s", "steps": args.host_steps,
            "warmup": 1, "ms_per_step": round(h_total / args.host_steps, 3),
            "definition": "the same prepares in registered host memory on each GPU's NUMA node (%s), PCIe H2D and "
                          "replies inside the timed region" % nodes,
            "p99_batch_latency_ms": round(ref_percentile(h_lat, 99), 3),
            "pcie": {"achieved_per_gpu": round(pcie_gbs / N, 2), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                     "frac": round(pcie_gbs / N / PCIE_PEAK_GBS, 4), "measured_ceiling": PCIE_MEASURED_GBS,
                     "frac_of_measured": round(pcie_gbs / N / PCIE_MEASURED_GBS, 4)},
            "roofline": roofline(h_stats, expected_unique(args.accounts, 2 * per_launch_h) / per_launch_h, per_launch_h,
                                 argparse.Namespace(transfers=T, steps=args.host_steps), h_total,
                                 kernel="tb_transfers_validate"),
        }

    # -- parity: one full pass through the timed path against the oracle --------------------------
    parity = {"full_run_properties": full_ok, "ledger": {k: str(v) for k, v in summ.items()}}
    if n_sample:
        oracle_accts = np.concatenate(oracle_accts)
        assert len(oracle_accts) == len(sample_idx)
        s_lens = lens[:n_sample_prep]
        s_ts, t_cursor = timestamps(s_lens, t_cursor + 10, wl["gap_every"])
        oracle = OracleEngine(len(oracle_accts) + 16, n_sample)
        oracle.upsert_accounts(oracle_accts)
        expected = oracle.commit_many(129, s_ts, split(sample_x, s_lens))
        engine.reset_transfers()
        rb_s, _ = engine.commit_pipelined_ptrs(129, s_ts, s_lens, dptrs[:n_sample_prep], replies, chunk_batches=chunk)
        got, off = [], 0
        for L, nb in zip(s_lens, rb_s):
            got.append(bytes(replies[off * 8:off * 8 + int(nb)]))
            off += L
        ids = np.stack([oracle_accts["id_lo"], oracle_accts["id_hi"]], axis=1)
        mine, found = engine.fetch_accounts(ids)
        theirs, _ = oracle.fetch_accounts(ids)
        parity.update({
            "sample_transfers": n_sample, "sample_prepares": n_sample_prep,
            "sample_path": "one full pass (%d sources x %d prepares) from device-resident prepares (the timed path)"
                           % (N, chunk),
            "replies_equal": got == expected,
            "accounts_equal": bool(found.all()) and mine.tobytes() == theirs.tobytes(),
            "transfers_equal": engine.export_transfers(cap=n_sample).tobytes() == oracle.export_transfers().tobytes(),
            "sample_failed_events": sum(len(r) for r in expected) // 8,
        })
    for dbuf, sh in zip(dbufs, shards):
        sh.free(dbuf)

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "transfers/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(total_ms / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u128",
        "data": "synthetic (generated on the GPUs in the reference benchmark's shapes, resident in each source GPU's "
                "HBM before timing)",
        "config": {"workload": ("C5 (BASELINE.json configs[4]): %d accounts hash-partitioned by owner over %d GPUs, %d "
                                "uniform transfers per GPU (%d in all), prepares of %d"
                                % (args.accounts, N, args.transfers, T, args.batch)) if args.workload == "c2" else
                               ("%s on %d GPUs: " % (args.workload, N)) + WORKLOAD_TEXT[args.workload] % (
                                   args.accounts, T, args.batch),
                   "prepares_per_step": n_prep, "chunk_prepares_per_gpu": chunk,
                   "engine": "one tbgpu node engine (include/tbgpu.h tbgpu_config.devices = %s), driven by one "
                             "process; %d process(es) launched" % (devices, procs),
                   "input": "prepare bodies resident in their source GPU's HBM (block d of every pass on GPU d); "
                            "replies into host memory; the PCIe-inclusive rate is `host_path`",
                   "parallelism": "shard%d (transfer home = hash(id), balance legs to owner GPUs, peer reads over "
                                  "xGMI inside the library)" % N},
        "p99_batch_latency_ms": round(ref_percentile(lat, 99), 3),
        "batch_latency_ms": dict(deciles(lat), definition=(
            "per prepare, submit to reply: from the start of its pass on its source GPU to its reply landing in host "
            "memory (device clock of its source GPU); percentiles by src/benchmark.zig:454-471")),
        "failed_events": n_failed,
        "passes": passes,
        "roofline": roof,
        "host_path": host_path,
        "cpu_baseline": None,
        "parity": parity,
    }
    line["headline"] = {"value": line["value"], "unit": "transfers/s", "p99_batch_latency_ms": line["p99_batch_latency_ms"],
                        "roofline_frac": roof["frac"] if roof else None,
                        "host_path_value": host_path["value"] if host_path else None}
    print(json.dumps(line), flush=True)
    engine.close()
    if procs > 1:
        dist.destroy_process_group()


FLOW_PHASES = ("plan", "sort", "link", "bounds_setup", "bounds_rounds", "sweep", "run_or_apply", "replies_wg0")


def flow_phases(stats):
    """tb_flow's wall time by phase (device clock, workgroup 0), ms over the measured steps."""
    return {n: round(v, 3) for n, v in zip(FLOW_PHASES, stats["flow_phase_ms"])}


def access_mix(engine, transfers, kernel_ms):
    """tb_transfers_validate's memory accesses without its logic (tbgpu_bench_access_mix: stream the
    event in and the record + per-event results out, two random account-row reads, one random CAS
    into an index sized like the engine's), timed on this GPU for one launch's transfers: the
    practical bound of the kernel's access pattern.  frac = that time / the kernel's launch time."""
    parts = engine.access_mix(int(transfers))
    return {"ms": round(parts["all"], 4), "kernel_ms": round(kernel_ms, 4), "frac": round(parts["all"] / kernel_ms, 3),
            "parts_ms": {k: round(v, 4) for k, v in parts.items()}, "transfers": int(transfers),
            "source": "tbgpu_bench_access_mix (k_workload.h tb_access_mix), measured in this run"}


def roofline(stats, u_over_t, per_launch_transfers, args, total_ms, breakdown=None, steps=None, kernel=None,
             pmc_leg=None, in_place=False):
    """The dominant kernel of the timed steps against the HBM peak; `kernels` = every kernel's mean
    launch time (from the warmup steps when given: the timed steps time only validate, replay/flow
    and whole passes).  `in_place`: the prepares were committed at their transfer-log positions, so
    validate stamps each record's 8-B timestamp instead of writing the 128-B record; the line then
    also carries `in_place` (the same launch priced at the bytes that kernel must move)."""
    def kernel_table(stats):
        return {
            "tb_transfers_validate": (stats["ms_validate"], stats["launches_validate"]),
            "tb_resolve<129>": (stats["ms_resolve"], stats["launches_resolve"]),
            # the ordered fallback of create_transfers passes: tb_flow (or tb_replay<129> when disabled)
            "tb_flow": (stats["ms_replay"], stats["launches_replay"]),
            "tb_pass_clear": (stats["ms_clear"], stats["launches_clear"]),
            "tb_apply_legs": (stats["ms_apply"], stats["launches_apply"]),
        }

    kernels = kernel_table(stats)
    dom = kernel or max(kernels, key=lambda k: kernels[k][0])
    ms_dom, n_dom = kernels[dom]
    # The launch's own duration on the device clock (tbgpu_stats.span_ms; validate: from the end of
    # the kernel before it to the start of the one after it, pass.h), what rocprofv3's kernel trace
    # measures too.  The timed steps put no HIP event pair around validate (an event record between
    # the kernels would sit inside its span): its HIP-event mean comes from the warmup steps.
    span_idx = {"tb_transfers_validate": 0, "tb_resolve<129>": 1, "tb_apply_legs": 2}.get(dom)
    has_span = bool(span_idx is not None and stats.get("span_launches") and stats["span_launches"][span_idx])
    # B = 296 + 256·U/T per transfer, split by where the work happens:
    # validate reads the event (128), probes + claims the id (32), writes the record (128) and reads
    # each touched account once (128·U/T); resolve writes the result slot (8) and each touched
    # account back (128·U/T) — or, with the legs path, tb_apply_legs writes the accounts back.
    legs = (breakdown or stats)["launches_apply"] > 0
    b_validate = 288 + 128 * u_over_t
    b_resolve = 8 + (0 if legs else 128 * u_over_t)
    b_apply = 128 * u_over_t if legs else 0.0
    alg_bytes = {"tb_transfers_validate": b_validate, "tb_resolve<129>": b_resolve, "tb_flow": 0.0,
                 "tb_pass_clear": 0.0,
                 "tb_apply_legs": b_apply}[dom] * per_launch_transfers
    if not n_dom and not has_span:
        return None
    hms, hn = (kernels if n_dom else kernel_table(breakdown) if breakdown else kernels)[dom]
    hip_avg = hms / hn if hn else None
    avg_ms, timing = hip_avg, "HIP events on the engine stream around every launch of the kernel in the timed steps"
    if has_span:
        avg_ms = stats["span_ms"][span_idx] / stats["span_launches"][span_idx]
        timing = ("device clock (s_memrealtime), every launch of the kernel in the timed steps: validate from the end of "
                  "tb_pass_clear to the start of tb_resolve, the others from the first workgroup's start to the last "
                  "one's end")
    avg_s = avg_ms / 1e3
    achieved = alg_bytes / avg_s / 1e9
    src = kernel_table(breakdown) if breakdown else kernels
    per_kernel = {k: {"launches": int(n), "avg_launch_ms": round(ms / n, 4)} for k, (ms, n) in src.items() if n}
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": dom,
           "avg_launch_ms": round(avg_ms, 4), "avg_launch_ms_hip_events": round(hip_avg, 4) if hip_avg else None,
           "transfers_per_launch": round(per_launch_transfers, 1),
           "alg_bytes_per_transfer": round(alg_bytes / per_launch_transfers, 1), "timing": timing}
    if dom == "tb_transfers_validate":
        # One build's validate mean moves with the box it lands on (each gpurun call gets a fresh one):
        # round 5's driver runs of unchanged kernels read frac 0.276-0.285, round 4's same-build A/B
        # lines 0.59-0.70 ms.  The frac above is this box's.
        out["frac_box_spread"] = "about +-8% box to box for one build (DESIGN.md §4); this line is one box"
        if in_place:
            # §8(d)'s figure counts the groove insert's 128-B record write; committed in place the record
            # is already at its log position (placed before the timed region, as a replica's receive DMA
            # would) and the kernel writes only its timestamp: 128 - 8 = 120 B fewer per transfer.
            b_ip = b_validate - 120
            out["in_place"] = {"alg_bytes_per_transfer": round(b_ip, 1),
                               "achieved": round(b_ip * per_launch_transfers / avg_s / 1e9, 1),
                               "frac": round(b_ip * per_launch_transfers / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                               "definition": "the in-place launch's own minimum: event read 128, id probe + claim "
                                             "32, timestamp stamp 8, each touched account read once (128 U/T)"}
    if pmc_leg:  # the C2 launches the PMC runs profiled (not the C3/C4 lines)
        out.update(load_pmc(pmc_leg, dom, per_launch_transfers))
    if out.get("rocprof_avg_launch_ms"):
        # The same definition from the committed rocprof summary: algorithmic bytes per transfer x the
        # profiled launches' mean transfers / rocprof's mean launch duration.
        rp = out["rocprof_avg_launch_ms"] / 1e3
        out["frac_rocprof"] = round(alg_bytes / per_launch_transfers * out["rocprof_launch_transfers"] / rp / 1e9
                                    / HBM_PEAK_GBS, 4)
    out.update({"kernels": per_kernel, "kernels_timed_in": "warmup steps (every kernel)" if breakdown else "timed steps",
                "path_bytes_per_transfer": round(296 + 256 * u_over_t, 1),
                "path_achieved_GBs": round((296 + 256 * u_over_t) * args.transfers * (steps or args.steps)
                                           / (total_ms / 1e3) / 1e9, 1)})
    return out

if __name__ == "__main__":
    main()
