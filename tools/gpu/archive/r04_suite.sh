#!/bin/bash
# The whole -m gpu suite and smoke() of the current tree.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/suite.log | head -30; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; exit $rc
