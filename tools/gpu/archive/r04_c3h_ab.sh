#!/bin/bash
# C3h (bench --workload c3h, 1M accounts, 10M transfers from host memory) on two builds, alternating.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04
mkdir -p $O
for v in ${AB_VARIANTS:-norefresh cur}; do
  if [ $v = cur ]; then unset TBGPU_AB_LIB; else export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload c3h --accounts 1000000 --transfers 10000000 --steps 2 --warmup 1 \
    --cpu-sample 0 --host-prepares 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0 --device-steps 0 \
    > $O/c3h_$v.json 2> $O/c3h_$v.err || { echo FAIL $v; tail -5 $O/c3h_$v.err; exit 1; }
  python - $O/c3h_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
f = d.get("flow", {})
print(sys.argv[2], "value %.1f M/s" % (d["value"] / 1e6), "ms/step", d.get("ms_per_step"),
      {k: f.get(k) for k in ("sweep_ms", "walk_crit_ms", "walk_crit_wait_ms", "walk_heavy_stops", "walk_crit_windows", "walk_crit_blocks")},
      "parity", d.get("parity", {}).get("replies_equal"))
PY
done
