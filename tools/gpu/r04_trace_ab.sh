#!/bin/bash
# Kernel traces (and FETCH/WRITE counters) of the device-resident leg: current build vs round 3's.
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r04/trace_ab
mkdir -p $O
ARGS="--steps 1 --warmup 0 --cpu-sample 0 --host-prepares 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0 --transfers 20971200"
for v in cur r3; do
  if [ $v = cur ]; then unset TBGPU_AB_LIB; else export TBGPU_AB_LIB=$R/tigerbeetle_amd/libtbgpu_4b43286.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o kt --output-format csv -- python3 $R/bench.py $ARGS > $O/$v.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/${v}_fetch -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $O/${v}_f.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/${v}_hit -o pmc --output-format csv -- python3 $R/bench.py $ARGS > $O/${v}_h.log 2>&1 || exit 1
done
