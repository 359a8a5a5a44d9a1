#!/bin/bash
# Round-4 measurement call: targeted tests, the replica call path with and without the asynchronous
# write-back, then the default bench line.  Usage: bash tools/gpu/r04_run.sh [tests...]
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
T=${*:-tests/test_gpu_determinism.py tests/test_gpu_alloc.py tests/test_gpu_checkpoint.py}
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu $T > $O/run_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/run_tests.log | tail -15
[ $rc -ne 0 ] && { grep -E "^E " $O/run_tests.log | head -40; exit $rc; }
for mode in "" "--write-back"; do
  timeout -k 10 300 ./tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 $mode || exit 1
done
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 $O/bench_default.json; tail -5 $O/bench_default.err
exit $rc
