#!/bin/bash
# Round 5: the -m gpu suite (stop at the first failure), a short default bench and a node rehearsal
# (two logical shards on the box's one GPU).  Usage: r05_run.sh [suite|bench|node]...
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r05
mkdir -p $O
for what in "$@"; do
  case $what in
    suite)
      timeout -k 10 1000 python -u -m pytest -q -rf --maxfail=25 --timeout 240 --timeout-method thread -m gpu tests \
        > $O/suite.log 2>&1
      rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR" $O/suite.log | head -40; exit $rc; } ;;
    node_tests)
      timeout -k 10 900 python -u -m pytest -q -rf --maxfail=25 --timeout 240 --timeout-method thread -m gpu \
        tests/test_gpu_node.py tests/test_gpu_alloc.py tests/test_gpu_c5.py > $O/node_tests.log 2>&1
      rc=$?; echo "node tests rc=$rc"; tail -3 $O/node_tests.log
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR" $O/node_tests.log | head -40; exit $rc; } ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --secondary 0 --replica-prepares 0 --host-prepares 0 \
        --write-back 0 --cpu-sample 2000000 > $O/bench.json 2> $O/bench.err
      rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench.json; tail -5 $O/bench.err; [ $rc -ne 0 ] && exit $rc ;;
    benchfull)
      timeout -k 10 900 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err
      rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench_full.json; tail -5 $O/bench_full.err; [ $rc -ne 0 ] && exit $rc ;;
    node)
      timeout -k 10 600 python -u bench.py --gpus 2 --same-device --accounts 2000000 --transfers 8000000 --steps 2 \
        --warmup 1 --host-steps 1 > $O/node.json 2> $O/node.err
      rc=$?; echo "node rc=$rc"; tail -c 2500 $O/node.json; tail -5 $O/node.err; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done
exit 0
