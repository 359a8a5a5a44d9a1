#!/bin/bash
# Round 6: the -m gpu suite (stop at the first failure), a short default bench and a node rehearsal
# (two logical shards on the box's one GPU).  Usage: r05_run.sh [suite|bench|node]...
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r06
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
    tests)  # selected test files: TESTS="tests/a.py tests/b.py" r06_run.sh tests
      timeout -k 10 900 python -u -m pytest -v -rf --maxfail=5 --timeout 400 --timeout-method thread -m gpu $TESTS \
        > $O/tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; grep -E "GPU_MAX_HW_QUEUES|passed|failed" $O/tests.log | tail -5
      [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|^E  " $O/tests.log | head -40; exit $rc; } ;;
    nodeab)  # same box: single engine vs a 2-shard node at equal accounts and pass size (C2, device-resident)
      LEGS="--secondary 0 --replica-prepares 0 --host-prepares 0 --write-back 0 --cpu-sample 0 --host-steps 0 --access-mix 0"
      for pb in ${NODEAB_CHUNKS:-64 512}; do
        timeout -k 10 400 python -u bench.py --accounts 2000000 --transfers 8000000 --steps 3 --warmup 1 $LEGS \
          --staged-steps 0 --pass-batches $((2 * pb)) > $O/ab_single_$pb.json 2> $O/ab_single_$pb.err
        rc=$?; echo "single pass $((2 * pb)) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/ab_single_$pb.err; exit $rc; }
        python -c "import json;d=json.loads(open('$O/ab_single_$pb.json').read().strip().splitlines()[-1]);print('single',d['value'],d['ms_per_step'])"
        timeout -k 10 400 python -u bench.py --gpus 2 --same-device --accounts 2000000 --transfers 4000000 --steps 3 \
          --warmup 1 $LEGS --chunk-prepares $pb > $O/ab_node_$pb.json 2> $O/ab_node_$pb.err
        rc=$?; echo "node chunk $pb rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/ab_node_$pb.err; exit $rc; }
        python -c "import json;d=json.loads(open('$O/ab_node_$pb.json').read().strip().splitlines()[-1]);print('node',d['value'],d['ms_per_step'],d.get('parity'))"
      done ;;
    resab)  # resolve variants on device-resident C2 passes, rocprofv3 kernel trace each: base (libtbgpu_base.so),
            # cur, cur with TBGPU_NO_LEAN=1
      export TMPDIR=/tmp
      for v in ${RESAB_VARIANTS:-base cur nolean}; do
        unset TBGPU_AB_LIB TBGPU_NO_LEAN
        [ $v = base ] && export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_base.so
        [ $v = nolean ] && export TBGPU_NO_LEAN=1
        [ $v = spill ] && export TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_spill.so
        rm -rf $O/rk_$v
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rk_$v -o run -- \
          python3 tools/gpu/device_pass.py 100000000 > $O/rk_$v.log 2>&1
        rc=$?; echo "resab $v rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/rk_$v.log; exit $rc; }
        python3 tools/gpu/kstats.py $(find $O/rk_$v -name '*kernel_stats.csv' | head -1) tb_transfers_validate tb_resolve tb_apply_legs tb_flow tb_pass_clear
      done
      unset TBGPU_AB_LIB TBGPU_NO_LEAN ;;
    mbj)  # the sort + join microbenchmark, with a kernel trace (per-phase times)
      export TMPDIR=/tmp
      rm -rf $O/mbj_kt
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mbj_kt -o run -- tools/bin/microbench_join \
        > $O/mbj.json 2> $O/mbj.err
      rc=$?; echo "mbj rc=$rc"; cat $O/mbj.json; [ $rc -ne 0 ] && { tail -5 $O/mbj.err; exit $rc; }
      python3 tools/gpu/kstats.py $(find $O/mbj_kt -name "*kernel_stats.csv" | head -1) cas hist bucket_totals scan_totals bucket_runs scatter bucket_sort dups probe append ;;
    nodeq)  # C2 on two logical shards with NODEQ hardware queues (bench.py keeps an explicit setting >= 8)
      GPU_MAX_HW_QUEUES=${NODEQ:-16} timeout -k 10 400 python -u bench.py --gpus 2 --same-device --accounts 2000000 \
        --transfers 4000000 --steps 3 --warmup 1 --secondary 0 --replica-prepares 0 --host-prepares 0 --write-back 0 \
        --cpu-sample 0 --host-steps 0 --access-mix 0 --chunk-prepares ${NODEQ_CHUNK:-64} > $O/nodeq_${NODEQ:-16}.json 2> $O/nodeq.err
      rc=$?; echo "nodeq ${NODEQ:-16} rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/nodeq.err; exit $rc; }
      python -c "import json;d=json.loads(open('$O/nodeq_${NODEQ:-16}.json').read().strip().splitlines()[-1]);print('node q${NODEQ:-16}',d['value'],d['ms_per_step'])" ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      rc=$?; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --secondary 0 --replica-prepares 0 --host-prepares 0 \
        --write-back 0 --cpu-sample 2000000 > $O/bench.json 2> $O/bench.err
      rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench.json; tail -5 $O/bench.err; [ $rc -ne 0 ] && exit $rc ;;
    nodelib)  # same box: node C2 (2 logical shards) with library builds in turn (NODELIB_VARIANTS: cur or a
      # tigerbeetle_amd/libtbgpu_<name>.so), NODELIB_CHUNKS prepare blocks
      LEGS="--secondary 0 --replica-prepares 0 --host-prepares 0 --write-back 0 --cpu-sample 0 --host-steps 0 --access-mix 0"
      for v in ${NODELIB_VARIANTS:-r06a cur r06a cur}; do
        lib=""; [ "$v" != cur ] && lib="$R/tigerbeetle_amd/libtbgpu_$v.so"
        for pb in ${NODELIB_CHUNKS:-64 512}; do
          TBGPU_AB_LIB=$lib timeout -k 10 400 python -u bench.py --gpus 2 --same-device --accounts 2000000 --transfers 4000000 \
            --steps 3 --warmup 1 $LEGS --chunk-prepares $pb > $O/nodelib_${v}_$pb.json 2> $O/nodelib_${v}_$pb.err
          rc=$?; [ $rc -ne 0 ] && { echo "nodelib $v $pb rc=$rc"; tail -5 $O/nodelib_${v}_$pb.err; exit $rc; }
          python -c "import json;d=json.loads(open('$O/nodelib_${v}_$pb.json').read().strip().splitlines()[-1]);print('nodelib $v $pb',round(d['value']/1e6,1),'M/s',d['ms_per_step'],'ms')"
        done
      done ;;
    flowab)  # same box: the C3 / C3h / C4 lines (host 10M + device-resident 100M) with library builds in turn
      for v in ${FLOWAB_VARIANTS:-preadm cur preadm cur}; do
        lib=""; [ "$v" != cur ] && lib="$R/tigerbeetle_amd/libtbgpu_$v.so"
        TBGPU_AB_LIB=$lib timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --host-prepares 0 --replica-prepares 0 \
          --write-back 0 --cpu-sample 0 --host-steps 0 --access-mix 0 --staged-steps 0 > $O/flowab_$v.json 2> $O/flowab_$v.err
        rc=$?; [ $rc -ne 0 ] && { echo "flowab $v rc=$rc"; tail -5 $O/flowab_$v.err; exit $rc; }
        python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('flowab', sys.argv[2], ' '.join('%s %.1f/%.1f' % (k, v['value']/1e6, v['device_resident']['value']/1e6) for k, v in d['secondary'].items()))
" $O/flowab_$v.json $v
      done ;;
    wblib)  # same box: the replica's write-back shapes with library builds in turn (WBLIB_VARIANTS: cur, or a
      # directory tigerbeetle_amd/<name>/ holding a libtbgpu.so the bench's RUNPATH is overridden to)
      for v in ${WBLIB_VARIANTS:-ab_wbprev cur ab_wbprev cur}; do
        ld=""; [ "$v" != cur ] && ld="$R/tigerbeetle_amd/$v"
        for m in "--write-back-every 4" "--write-back-every 8" --write-back; do
          f="$O/wblib_${v}_$(echo $m | tr -d ' -')"
          LD_LIBRARY_PATH=$ld timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 \
            --device 0 $m --stage > "$f.json" 2> "$f.err"
          rc=$?; [ $rc -ne 0 ] && { echo "wblib $v $m rc=$rc"; tail -3 "$f.err"; exit $rc; }
          python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('wblib',sys.argv[2],sys.argv[3],round(d['transfers_per_s']/1e6,1),'M/s p99',d['p99_ms'])" "$f.json" "$v" "$m"
        done
      done ;;
    wbab)  # write-back copy-out A/B on one box: counts-sized vs bound-sized, read through vs staged bodies
      for v in ${WBAB_VARIANTS:-base bound stage both}; do
        case $v in
          base) env_="TBGPU_WB_BOUND=0 TBGPU_WB_STAGE=0"; st="" ;;
          bound) env_="TBGPU_WB_BOUND=1 TBGPU_WB_STAGE=0"; st="" ;;
          stage) env_="TBGPU_WB_BOUND=0 TBGPU_WB_STAGE=1"; st="--stage" ;;
          both) env_="TBGPU_WB_BOUND=1 TBGPU_WB_STAGE=1"; st="--stage" ;;
        esac
        for m in ${WBAB_SHAPES:-"--write-back-every 4" "--write-back-every 8" --write-back --write-back-per-op}; do
          f="$O/wbab_${v}_$(echo $m | tr -d ' -')"
          env $env_ timeout -k 10 300 tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 --device 0 \
            $m $st > "$f.json" 2> "$f.err"
          rc=$?; [ $rc -ne 0 ] && { echo "wbab $v $m rc=$rc"; tail -3 "$f.err"; exit $rc; }
          python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('wbab',sys.argv[2],sys.argv[3],round(d['transfers_per_s']/1e6,1),'M/s p99',d['p99_ms'],'compact',d['compact_ms_per_op'])" "$f.json" "$v" "$m"
        done
      done ;;
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
