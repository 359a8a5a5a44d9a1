#!/bin/bash
# Write-back rewrite: checkpoint + node tests, then the bench's write-back leg alone.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_checkpoint.py \
  tests/test_gpu_node.py tests/test_gpu_c5.py::test_c5_node_full_size > gpurun_out/r03/pytest_wb.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r03/pytest_wb.log; grep -E "^E " gpurun_out/r03/pytest_wb.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 \
  --access-mix 0 > gpurun_out/r03/bench_wb.log 2>&1
echo "bench rc=$?"
exit 0
