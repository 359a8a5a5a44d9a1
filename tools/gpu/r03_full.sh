#!/bin/bash
# The whole -m gpu suite, then the teardown probes that faulted under rocprofv3 (csv output).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 1000 python -u -m pytest -q -x --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r03/pytest_all.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -4 gpurun_out/r03/pytest_all.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03/pytest_all.log | head -30; exit $rc; fi
for mode in flow bench; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03/pf_$mode -o run -- \
    python3 $R/tools/gpu/exit_probe.py $mode $R/gpurun_out/r03 > $R/gpurun_out/r03/pf_$mode.log 2>&1
  echo "probe $mode rc=$?"
done
exit 0
