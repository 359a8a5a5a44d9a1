#!/bin/bash
# Replica call path: the C++ bench (staged / read-through, in-memory / with write-back), then the tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for opt in "" "--no-stage" "--write-back" "--write-back --no-stage"; do
  timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --prepares 2000 $opt > gpurun_out/r03/replica.json 2> gpurun_out/r03/replica.err
  echo "replica [$opt] rc=$?"; cat gpurun_out/r03/replica.json; tail -2 gpurun_out/r03/replica.err
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  tests/test_gpu_host_path.py tests/test_host_cpp.py tests/test_gpu_flow.py tests/test_gpu_tables.py tests/test_gpu_differential.py \
  tests/test_gpu_edges.py > gpurun_out/r03/pytest_rp.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r03/pytest_rp.log; grep -E "^E " gpurun_out/r03/pytest_rp.log | head
