#!/bin/bash
# Walker parity (quick), then the adversarial C3 (merged heavy walk, and a wave per heavy segment) and C3.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_walk.py \
  > gpurun_out/r03b/pytest_walk.log 2>&1
rc=$?
echo "walk tests rc=$rc"; tail -3 gpurun_out/r03b/pytest_walk.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_walk.log | head -30; exit $rc; fi
B="--accounts 1000000 --transfers 10000000 --steps 1 --warmup 1 --cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 --replica-prepares 0 --access-mix 0"
for v in "c3h -1" "c3 -1"; do
  set -- $v
  timeout -k 10 300 python -u bench.py --workload $1 --walk-merge $2 $B > gpurun_out/r03b/bench_$1_m$2.log 2>&1
  rc=$?
  echo "$1 merge=$2 bench rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
