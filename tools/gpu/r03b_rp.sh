#!/bin/bash
# The replica call path after the done-word spin: its tests, the C++ replica bench, the walker tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_host_path.py \
  tests/test_host_cpp.py tests/test_gpu_pipeline.py tests/test_gpu_tables.py tests/test_gpu_walk.py tests/test_gpu_checkpoint.py \
  > gpurun_out/r03b/pytest_rp.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r03b/pytest_rp.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_rp.log | head -30; exit $rc; fi
for opt in "" "" "" "--stage"; do
  timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --prepares 2000 $opt > gpurun_out/r03b/replica.json 2> gpurun_out/r03b/replica.err
  echo "replica [$opt] rc=$?"; cat gpurun_out/r03b/replica.json
done
