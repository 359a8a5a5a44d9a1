#!/bin/bash
# Walker parity first (C3 shapes, mixed limit flags, the adversarial C3), then the whole suite and the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_walk.py \
  tests/test_gpu_configs.py > gpurun_out/r03b/pytest_walk.log 2>&1
rc=$?
echo "walk tests rc=$rc"; tail -5 gpurun_out/r03b/pytest_walk.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_walk.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py --workload c3h --accounts 1000000 --transfers 10000000 --steps 1 --warmup 1 \
  --cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 --replica-prepares 0 > gpurun_out/r03b/bench_c3h.log 2>&1
echo "c3h bench rc=$?"; tail -c 1200 gpurun_out/r03b/bench_c3h.log
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03b/pytest_all.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -4 gpurun_out/r03b/pytest_all.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_all.log | head -30; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r03b/bench_default.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r03b/bench_default.log
exit $rc
