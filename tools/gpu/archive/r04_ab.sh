#!/bin/bash
# Same-box A/B of older engine builds (tigerbeetle_amd/libtbgpu_<name>.so) against the current one,
# headline + device-resident legs only.  usage: AB_VARIANTS="4b43286 cur" bash tools/gpu/r04_ab.sh
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04
mkdir -p $O
ARGS="--steps 2 --cpu-sample 0 --host-prepares 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0"
for v in ${AB_VARIANTS:-cur}; do
  unset TBGPU_NO_KCLOCK
  case $v in
    cur) unset TBGPU_AB_LIB ;;
    knobs_nokc) export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_knobs.so TBGPU_NO_KCLOCK=1 ;;
    *) export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_$v.so ;;
  esac
  timeout -k 10 300 python -u bench.py $ARGS > $O/ab_$v.json 2> $O/ab_$v.err || { echo AB_FAIL $v; tail -5 $O/ab_$v.err; exit 1; }
  python - $O/ab_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]; dr = d.get("device_resident", {}).get("roofline", {})
k = r["kernels"]; dk = dr.get("kernels", {})
print(sys.argv[2], "value %.1f" % (d["value"] / 1e6), "head validate %.4f resolve %.4f apply %.4f" % (
    k["tb_transfers_validate"]["avg_launch_ms"], k.get("tb_resolve<129>", {}).get("avg_launch_ms", 0),
    k.get("tb_apply_legs", {}).get("avg_launch_ms", 0)), "dev validate", dk.get("tb_transfers_validate"),
    "dev resolve/apply", dk.get("tb_resolve<129>"), dk.get("tb_apply_legs"),
    "dev value %.2f G/s" % (d.get("device_resident", {}).get("value", 0) / 1e9))
PY
done
