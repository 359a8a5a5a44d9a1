#!/bin/bash
# The whole -m gpu suite, then the replica call path's trace and timed runs (r03c_rp.sh steps).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03c/pytest_all.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -2 gpurun_out/r03c/pytest_all.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03c/pytest_all.log | head -30; exit $rc; fi
bash tools/gpu/r03c_rp.sh
