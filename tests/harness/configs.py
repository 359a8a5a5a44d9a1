"""BASELINE.json workload shapes (C2 uniform, C3 Zipf + limit accounts, C4 chains / two-phase /
balancing), generated on the GPU by the engine's own generator (csrc/k_workload.h) and copied to
the host, so the oracle and the engine commit byte-identical prepares.  Shared by the GPU parity
tests and bench.py."""
import numpy as np

KINDS = {"c2": 0, "c3": 1, "c3h": 1, "c4": 2}
# Per-config generator settings.
SETTINGS = {
    "c2": dict(limit_permille=0, gap_every=0),
    "c3": dict(limit_permille=100, gap_every=0),
    # C3 with the hottest Zipf rank limited too (the adversarial case: ~18 % of the debits check one
    # account whose balance hovers at its limit).
    "c3h": dict(limit_permille=100, gap_every=0, hot_limited=1),
    # C4: a 2 s timestamp gap every 64 prepares, so 1..10 s pending timeouts expire across gaps.
    "c4": dict(limit_permille=0, gap_every=64),
}
GAP_NS = 2_000_000_000


def batches(total, batch):
    q, r = divmod(total, batch)
    return [batch] * q + ([r] if r else [])


def timestamps(lens, start, gap_every=0, gap_ns=GAP_NS):
    """Prepare timestamps: t_k = t_{k-1} + 1 + len_k (state_machine.zig:1483-1485), plus an
    optional gap before every `gap_every`-th prepare (C4 expiry)."""
    ts, t = [], start
    for k, L in enumerate(lens):
        if gap_every and k and k % gap_every == 0:
            t += gap_ns
        t += 1 + L
        ts.append(t)
    return ts, t


def generate(engine, config, n_accounts, n_transfers, seed, first_transfer=0):
    """Device-generate the config's accounts and transfers; returns host uint8 arrays."""
    st = SETTINGS[config]
    acct_dev = engine.alloc(n_accounts * 128)
    hot = st.get("hot_limited", 0)
    engine.generate_accounts(acct_dev, 0, n_accounts, seed=seed, limit_permille=st["limit_permille"],
                             account_count=n_accounts, hot_limited=hot)
    xfer_dev = engine.alloc(max(n_transfers, 1) * 128)
    engine.generate_transfers(xfer_dev, first_transfer, n_transfers, n_accounts, seed=seed, kind=KINDS[config],
                              limit_permille=st["limit_permille"], hot_limited=hot)
    engine.sync()
    accts = engine.to_host(acct_dev, n_accounts * 128)
    xfers = engine.to_host(xfer_dev, n_transfers * 128)
    engine.free(acct_dev)
    engine.free(xfer_dev)
    return np.asarray(accts), np.asarray(xfers)


def split(events, lens):
    out, off = [], 0
    for L in lens:
        out.append(events[off * 128:(off + L) * 128].tobytes())
        off += L
    return out
