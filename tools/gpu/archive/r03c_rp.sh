#!/bin/bash
# Replica call path: parity tests, a kernel trace of tb_replica_bench, then three timed runs.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_host_path.py \
  tests/test_host_cpp.py tests/test_gpu_pipeline.py tests/test_gpu_tables.py tests/test_gpu_checkpoint.py ${EXTRA_TESTS} \
  > gpurun_out/r03c/pytest_rp.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r03c/pytest_rp.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03c/pytest_rp.log | head -30; exit $rc; fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03c/rp_trace -o run -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 300 --warmup 20 > $R/gpurun_out/r03c/rp_trace.log 2>&1
echo "trace rc=$?"
cd $R
for opt in "" "" ""; do
  timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --prepares 2000 $opt > gpurun_out/r03c/replica.json 2> gpurun_out/r03c/replica.err
  echo "replica [$opt] rc=$?"; cat gpurun_out/r03c/replica.json
done
