#!/bin/bash
# SQ counters of the replica call path's kernels (one --pmc pass, tb_replica_bench, 100 calls).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
  --output-format csv -d $R/gpurun_out/r03c/rp_pmc -o run -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 100 --warmup 10 > $R/gpurun_out/r03c/rp_pmc.log 2>&1
echo "pmc rc=$?"
