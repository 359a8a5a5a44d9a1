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
    evict)
      timeout -k 10 600 python -u -m pytest -q -rf --timeout 400 --timeout-method thread -m gpu tests/test_gpu_evict.py \
        > $O/evict.log 2>&1
      rc=$?; echo "evict rc=$rc"; tail -15 $O/evict.log; [ $rc -ne 0 ] && exit $rc ;;
    inplace)
      timeout -k 10 600 python -u -m pytest -q -rf --timeout 400 --timeout-method thread -m gpu tests/test_gpu_inplace.py \
        > $O/inplace.log 2>&1
      rc=$?; echo "inplace rc=$rc"; tail -15 $O/inplace.log; [ $rc -ne 0 ] && exit $rc ;;
    race)  # the node engine with every stream on its own hardware queue (as on N GPUs): node tests, C3 twice
      export GPU_MAX_HW_QUEUES=8
      timeout -k 10 600 python -u -m pytest -q -rf --maxfail=5 --timeout 240 --timeout-method thread -m gpu \
        tests/test_gpu_node.py -k "dirty or clean or differential or device_resident" > $O/race_tests.log 2>&1
      rc=$?; echo "race tests rc=$rc"; tail -3 $O/race_tests.log
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|^E  " $O/race_tests.log | head -40; exit $rc; }
      for k in 1 2; do
        timeout -k 10 300 python -u bench.py --gpus 2 --same-device --accounts 1000000 --transfers 4000000 --steps 2 \
          --warmup 1 --host-steps 0 --workload c3 > $O/race_c3_$k.json 2> $O/race_c3_$k.err
        rc=$?; echo "race c3 $k rc=$rc"; grep -o '"parity": {[^}]*}' $O/race_c3_$k.json; [ $rc -ne 0 ] && exit $rc
      done
      unset GPU_MAX_HW_QUEUES ;;
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
    replica)  # the replica call path (C++ mirror) with each write-back shape
      for m in --write-back --write-back-sync "--write-back --checkpoint-journal-slots 1024" --write-back-per-op "--write-back-every 4" "--write-back-every 8"; do
        timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 --device 0 $m \
          > "$O/replica$m.json" 2> "$O/replica$m.err"
        rc=$?; echo "replica $m rc=$rc"; cat "$O/replica$m.json"; [ $rc -ne 0 ] && { tail -3 "$O/replica$m.err"; exit $rc; }
      done ;;
    driver)  # the driver's own command line
      timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
      rc=$?; echo "bench rc=$rc"; tail -c 1200 $O/bench_driver.json; tail -5 $O/bench_driver.err; [ $rc -ne 0 ] && exit $rc ;;
    benchfull)
      timeout -k 10 900 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err
      rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench_full.json; tail -5 $O/bench_full.err; [ $rc -ne 0 ] && exit $rc ;;
    node)
      timeout -k 10 600 python -u bench.py --gpus 2 --same-device --accounts 2000000 --transfers 8000000 --steps 2 \
        --warmup 1 --host-steps 1 > $O/node.json 2> $O/node.err
      rc=$?; echo "node rc=$rc"; tail -c 2500 $O/node.json; tail -5 $O/node.err; [ $rc -ne 0 ] && exit $rc ;;
    passab)  # device-resident passes of 512 vs 1024 prepares
      for pb in 512 1024; do
        timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --secondary 0 --replica-prepares 0 --host-prepares 0 \
          --write-back 0 --cpu-sample 0 --host-steps 0 --access-mix 0 --pass-batches $pb > $O/passab_$pb.json 2> $O/passab_$pb.err
        rc=$?; echo "pass $pb rc=$rc"; python -c "import json,sys;d=json.loads(open('$O/passab_$pb.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],{k:v['avg_launch_ms'] for k,v in d['roofline']['kernels'].items()})"
        [ $rc -ne 0 ] && { tail -5 $O/passab_$pb.err; exit $rc; }
      done ;;
    nodec3)
      timeout -k 10 600 python -u bench.py --gpus 2 --same-device --accounts 1000000 --transfers 4000000 --steps 2 \
        --warmup 1 --host-steps 1 --workload c3 > $O/node_c3.json 2> $O/node_c3.err
      rc=$?; echo "node c3 rc=$rc"; tail -c 2500 $O/node_c3.json; tail -5 $O/node_c3.err; [ $rc -ne 0 ] && exit $rc ;;
    nodec3c)  # C3 on the node with 128-prepare blocks
      timeout -k 10 600 python -u bench.py --gpus 2 --same-device --accounts 1000000 --transfers 4000000 --steps 2 \
        --warmup 1 --host-steps 0 --workload c3 --chunk-prepares 128 > $O/node_c3_128.json 2> $O/node_c3_128.err
      rc=$?; echo "node c3/128 rc=$rc"; grep -o '"headline": {[^}]*}' $O/node_c3_128.json; tail -3 $O/node_c3_128.err; [ $rc -ne 0 ] && exit $rc ;;
    nodec4)
      timeout -k 10 600 python -u bench.py --gpus 2 --same-device --accounts 1000000 --transfers 4000000 --steps 2 \
        --warmup 1 --host-steps 0 --workload c4 > $O/node_c4.json 2> $O/node_c4.err
      rc=$?; echo "node c4 rc=$rc"; tail -c 1500 $O/node_c4.json; tail -5 $O/node_c4.err; [ $rc -ne 0 ] && exit $rc ;;
    node1)  # one C2 prepare per tbgpu_commit: node (2 logical shards) and single engine
      GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/gpu/node_one_prepare.py 400 2 > $O/node1.jsonl 2> $O/node1.err
      rc=$?; echo "node1 rc=$rc"; cat $O/node1.jsonl; tail -5 $O/node1.err; [ $rc -ne 0 ] && exit $rc ;;
    prof_*)  # a tools/gpu/profile.sh mode
      bash tools/gpu/profile.sh ${what#prof_}; rc=$?; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done
exit 0
