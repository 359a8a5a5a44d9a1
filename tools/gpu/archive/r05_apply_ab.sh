#!/bin/bash
# Device-resident headline leg on several builds (cur = in-tree; NAME = tigerbeetle_amd/libtbgpu_NAME.so),
# alternating, printing value, validate frac and the per-kernel device-clock times.
# usage (GPU box): bash tools/gpu/r05_apply_ab.sh ROUNDS NAME...
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
mkdir -p gpurun_out/r05
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset TBGPU_AB_LIB; else export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_$v.so; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --secondary 0 --replica-prepares 0 --host-prepares 0 \
      --write-back 0 --cpu-sample 0 --host-steps 0 --access-mix 0 --staged-steps 0 > gpurun_out/r05/ab_${v}_$r.json 2> gpurun_out/r05/ab_${v}_$r.err \
      || { echo "FAIL $v"; tail -5 gpurun_out/r05/ab_${v}_$r.err; exit 1; }
    python tools/gpu/summ.py gpurun_out/r05/ab_${v}_$r.json "$v#$r"
  done
done
