#!/bin/bash
# Teardown SIGSEGV bisection: one engine feature per profiled process (rocprofv3 csv, as the crash).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for mode in flow register events pipelined; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03/pb_$mode -o run -- \
    python3 $R/tools/gpu/exit_probe.py $mode $R/gpurun_out/r03 > $R/gpurun_out/r03/pb_$mode.log 2>&1
  echo "probe $mode rc=$?"
done
timeout -k 10 60 python3 $R/tools/gpu/exit_probe.py flow $R/gpurun_out/r03 > $R/gpurun_out/r03/pb_flow_noprof.log 2>&1
echo "flow without profiler rc=$?"
exit 0
