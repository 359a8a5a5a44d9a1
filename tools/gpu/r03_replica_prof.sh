#!/bin/bash
# Timeline of the replica call path: kernel + memory-copy trace of tb_replica_bench (300 ops).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r03c/rp_trace -o run -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 300 --warmup 20 > $R/gpurun_out/r03c/rp_trace.log 2>&1
echo "rc=$?"; grep call_path $R/gpurun_out/r03c/rp_trace.log
find $R/gpurun_out/r03c/rp_trace -name "*.csv" | head
