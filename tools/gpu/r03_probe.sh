#!/bin/bash
# Round 3, first GPU call: the new parity tests, then the teardown probes under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_client_known_answers.py tests/test_gpu_pipeline.py::test_pipelined_stops_at_device_panic \
  tests/test_gpu_apply_split.py > gpurun_out/r03/pytest_new.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/pytest_new.log; exit 1; }
tail -3 gpurun_out/r03/pytest_new.log
for mode in lib torch both leak; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/probe_$mode -o run -- \
    python3 tools/gpu/exit_probe.py $mode gpurun_out/r03 > gpurun_out/r03/probe_$mode.log 2>&1
  echo "probe $mode rc=$?"
done
exit 0
