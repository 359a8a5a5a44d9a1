#!/bin/bash
# Same-box A/B of host-side features (env switches of the current build) on the headline and
# device-resident legs.  usage: bash tools/gpu/r04_ab_env.sh
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04
mkdir -p $O
ARGS="--steps 2 --cpu-sample 0 --host-prepares 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0"
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $ARGS > $O/abe_$name.json 2> $O/abe_$name.err || { echo FAIL $name; tail -5 $O/abe_$name.err; exit 1; }
  python - $O/abe_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; dr = d.get("device_resident", {}).get("roofline", {})
k = r["kernels"]; dk = dr.get("kernels", {})
print(sys.argv[2], "value %.1f" % (d["value"] / 1e6), "head validate %.4f apply %.4f" % (
    k.get("tb_transfers_validate", {}).get("avg_launch_ms", 0), k.get("tb_apply_legs", {}).get("avg_launch_ms", 0)),
    "dev validate", dk.get("tb_transfers_validate"), "dev value %.2f G/s" % (d.get("device_resident", {}).get("value", 0) / 1e9))
PY
}
run cur X=1
run nowb TBGPU_AB_NO_WB=1
run noprobe TBGPU_AB_NO_PROBE=1
run nopool TBGPU_AB_NO_POOL=1
run all TBGPU_AB_NO_WB=1 TBGPU_AB_NO_PROBE=1 TBGPU_AB_NO_POOL=1
run r3 TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_4b43286.so
