#!/bin/bash
# Round 6, last build: the -m gpu suite, the driver's bench command, the profiling-cost check.
# Every step under its own limit; the first failure ends the script.
set -o pipefail
O=gpurun_out/r06/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q -rf --maxfail=5 --timeout 240 --timeout-method thread -m gpu tests \
  > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; [ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/gpu/prof_cost.py 1 > $O/prof_cost.log 2>&1
rc=$?; echo "prof_cost rc=$rc"; exit $rc
