#!/bin/bash
# Round 3: C5 tests, apply-split, panic test; node bench rehearsal; teardown probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py::test_pipelined_stops_at_device_panic tests/test_gpu_apply_split.py tests/test_gpu_c5.py \
  > gpurun_out/r03/pytest_c5.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r03/pytest_c5.log | head; grep -E "^E " gpurun_out/r03/pytest_c5.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 2 --same-device --accounts 10000000 --transfers 20000000 --steps 2 --warmup 1 \
  > gpurun_out/r03/bench_node2_same.log 2>&1
echo "bench node rc=$?"; tail -c 1500 gpurun_out/r03/bench_node2_same.log
for mode in lib both leak; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/probe_$mode -o run -- \
    python3 tools/gpu/exit_probe.py $mode gpurun_out/r03 > gpurun_out/r03/probe_$mode.log 2>&1
  echo "probe $mode rc=$?"
done
exit $rc
