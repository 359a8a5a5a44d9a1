#!/bin/bash
# Round 3: panic-path debug, then the node-engine tests (logical shards on one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 120 python3 tools/gpu/dbg_panic.py > gpurun_out/r03/dbg_panic.log 2>&1; echo "dbg rc=$?"
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_node.py \
  > gpurun_out/r03/pytest_node.log 2>&1
rc=$?
echo "node tests rc=$rc"; tail -40 gpurun_out/r03/pytest_node.log
exit $rc
