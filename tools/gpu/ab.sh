# Same-box A/B of the headline bench: the current build against older builds of the engine
# (tigerbeetle_amd/libtbgpu_<name>.so, made by hand), alternating, so box-to-box variance cancels.
# usage (GPU box): [AB_VARIANTS="base cur"] bash tools/gpu/ab.sh [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in $(seq 1 "${1:-2}"); do
  for v in ${AB_VARIANTS:-base cur}; do
    if [ $v = cur ]; then unset TBGPU_AB_LIB; else export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_$v.so; fi
    timeout -k 10 300 python -u bench.py --cpu-sample 0 --host-prepares 0 --steps 2 > gpurun_out/ab_${v}_$r.log 2>&1 || { echo AB_FAIL $v; tail -5 gpurun_out/ab_${v}_$r.log; exit 1; }
    python tools/gpu/summ.py gpurun_out/ab_${v}_$r.log "$v#$r"
  done
done
