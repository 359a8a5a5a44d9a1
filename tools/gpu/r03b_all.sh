#!/bin/bash
# The walker script, then the whole -m gpu suite and the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/r03b_c3h.sh || exit $?
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03b/pytest_all.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r03b/pytest_all.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_all.log | head -30; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r03b/bench_default.log 2>&1
rc=$?
echo "bench rc=$rc"
exit $rc
