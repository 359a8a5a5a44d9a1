#!/bin/bash
# Round 3: the pipelined panic test, then teardown probes under rocprofv3 with CSV output (as the
# round-2 profiles that ended in SIGSEGV), up to a small bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py::test_pipelined_stops_at_device_panic > gpurun_out/r03/pytest_panic.log 2>&1
echo "panic test rc=$?"; grep -E "PASSED|FAILED|^E " gpurun_out/r03/pytest_panic.log | head
for mode in lib bench bench_torch; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03/pc_$mode -o run -- \
    python3 $R/tools/gpu/exit_probe.py $mode $R/gpurun_out/r03 > $R/gpurun_out/r03/pc_$mode.log 2>&1
  echo "csv probe $mode rc=$?"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03/pc_benchpy -o run -- \
  python3 $R/bench.py --accounts 100000 --transfers 4000000 --cpu-sample 0 --host-prepares 0 --device-steps 0 \
  --secondary 0 --steps 1 --warmup 1 > $R/gpurun_out/r03/pc_benchpy.log 2>&1
echo "csv bench rc=$?"
tail -25 $R/gpurun_out/r03/pc_benchpy.log | grep -v "^W2026\|^E2026" | head -30
exit 0
