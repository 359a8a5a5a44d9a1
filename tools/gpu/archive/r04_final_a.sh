#!/bin/bash
# Final-round call A: the round's GPU tests, the replica path both ways with a kernel trace of the
# write-back run, then the default bench line.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04final
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_alloc.py \
  tests/test_gpu_determinism.py tests/test_gpu_checkpoint.py tests/test_gpu_node.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -30; exit $rc; }
for mode in "" "--write-back"; do
  timeout -k 10 300 ./tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 $mode > $O/replica$mode.json || exit 1
  cat $O/replica$mode.json
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/replica_wb -o run --output-format csv -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 400 --write-back > /dev/null 2>&1 || exit 1
cd $R
timeout -k 10 700 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench_default.json; tail -3 $O/bench_default.err
exit $rc
