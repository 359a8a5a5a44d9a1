#!/bin/bash
# The default bench on the final code (its secondary lines include the replica call path).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u bench.py > gpurun_out/r03c/bench_default.log 2>&1
rc=$?
echo "bench rc=$rc"
exit $rc
