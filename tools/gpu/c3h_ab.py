"""C3h (bench.py's secondary.c3h line: 1M accounts, 10M transfers from registered host memory, 1M
parity sample) on the builds named on the command line, alternating: `cur` is the in-tree library,
any other name loads tigerbeetle_amd/libtbgpu_<name>.so (TBGPU_AB_LIB, set per child process).
usage (GPU box): python tools/gpu/c3h_ab.py [rounds] variant..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import json, sys
sys.argv = ["bench.py", "--secondary", "10000000"]
import bench
from tigerbeetle_amd.state_machine import Engine
seen = {}
_stats = Engine.stats
def stats(self):
    s = _stats(self)
    seen["walk_dbg"] = s.get("walk_dbg")
    return s
Engine.stats = stats
d = bench.run_secondary(bench.parse(), "c3h", 0)
d["flow"]["walk_dbg"] = seen.get("walk_dbg")
print(json.dumps(d))
"""


def main():
    rounds = int(sys.argv[1])
    variants = sys.argv[2:] or ["cur"]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            env.pop("TBGPU_AB_LIB", None)
            if v != "cur":
                env["TBGPU_AB_LIB"] = os.path.join(ROOT, "tigerbeetle_amd", "libtbgpu_%s.so" % v)
            p = subprocess.run([sys.executable, "-u", "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                               timeout=400)
            if p.returncode != 0:
                print("FAIL", v, p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            f = d["flow"]
            print(json.dumps({"variant": v, "round": r, "value_M": round(d["value"] / 1e6, 2), "ms": d["ms_per_step"],
                              "parity": all(d["parity"][k] for k in ("replies_equal", "accounts_equal",
                                                                      "transfers_equal", "posted_equal")),
                              **{k: f[k] for k in ("sweep_ms", "walk_crit_ms", "walk_crit_windows", "walk_crit_blocks",
                                                   "walk_crit_wait_ms", "walk_heavy_stops", "walk_heavy_blocks",
                                                   "walk_heavy_blocked_ms", "walk_dbg")}}), flush=True)


if __name__ == "__main__":
    main()
