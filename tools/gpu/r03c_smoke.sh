#!/bin/bash
# smoke() on the final code.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03c/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r03c/smoke.log
exit $rc
