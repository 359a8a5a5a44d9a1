#!/bin/bash
# Round 3: panic-path debug, the node-engine tests (logical shards on one GPU), write-back tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 120 python3 tools/gpu/dbg_panic.py > gpurun_out/r03/dbg_panic.log 2>&1; echo "dbg rc=$?"
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_node.py \
  tests/test_gpu_checkpoint.py tests/test_client_known_answers.py tests/test_gpu_pipeline.py::test_pipelined_stops_at_device_panic \
  > gpurun_out/r03/pytest_node.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r03/pytest_node.log | sed 's/.*:://' | sort | uniq -c | sort -rn | head -5
grep -E "FAILED|Error|error" gpurun_out/r03/pytest_node.log | head -30; tail -5 gpurun_out/r03/pytest_node.log
exit $rc
