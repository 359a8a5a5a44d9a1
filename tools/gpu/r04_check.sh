#!/bin/bash
# Round-4 GPU checks: the new convention / determinism / write-back tests first (fast feedback),
# then the whole -m gpu suite, then the replica call path with the asynchronous write-back.
# Usage: bash tools/gpu/r04_check.sh [quick]
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
run() { echo "== $*"; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_alloc.py tests/test_gpu_determinism.py tests/test_gpu_checkpoint.py tests/test_gpu_node.py > $O/new.log 2>&1
rc=$?; echo "new tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/new.log | tail -40
[ $rc -ne 0 ] && { grep -E "^E " $O/new.log | head -60; exit $rc; }
[ "$1" = quick ] && exit 0
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/suite.log | head -30; exit $rc; }
for mode in "" "--write-back"; do
  timeout -k 10 300 ./tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 $mode || exit 1
done
