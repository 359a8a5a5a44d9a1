#!/bin/bash
# A/B of the launch-span stamps: the headline and device-resident legs with and without them.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04
mkdir -p $O
ARGS="--steps 2 --cpu-sample 0 --host-prepares 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0"
TBGPU_NO_KCLOCK=1 timeout -k 10 300 python -u bench.py $ARGS > $O/ab_nokclock.json 2> $O/ab_nokclock.err || exit 1
timeout -k 10 300 python -u bench.py $ARGS > $O/ab_kclock.json 2> $O/ab_kclock.err || exit 1
TBGPU_NO_KCLOCK=1 timeout -k 10 300 python -u bench.py $ARGS > $O/ab_nokclock2.json 2> $O/ab_nokclock2.err || exit 1
for f in ab_nokclock ab_kclock ab_nokclock2; do
python - $O/$f.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; dr = d.get("device_resident", {}).get("roofline", {})
print(sys.argv[1], "value", round(d["value"] / 1e6, 1), "head", r["kernels"], "dev", dr.get("kernels"), dr.get("avg_launch_ms"))
PY
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/replica_wb -o run --output-format csv -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 400 --write-back
