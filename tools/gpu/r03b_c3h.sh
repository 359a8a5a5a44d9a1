#!/bin/bash
# Walker parity (quick), then the adversarial C3 and C3 alone on the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_walk.py \
  > gpurun_out/r03b/pytest_walk.log 2>&1
rc=$?
echo "walk tests rc=$rc"; tail -3 gpurun_out/r03b/pytest_walk.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/r03b/pytest_walk.log | head -30; exit $rc; fi
for w in c3h c3; do
  timeout -k 10 300 python -u bench.py --workload $w --accounts 1000000 --transfers 10000000 --steps 1 --warmup 1 \
    --cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 --replica-prepares 0 --access-mix 0 > gpurun_out/r03b/bench_$w.log 2>&1
  rc=$?
  echo "$w bench rc=$rc"; tail -c 3000 gpurun_out/r03b/bench_$w.log | tr ',' '\n' | grep -E '"value"|sweep|walk|bounds_swept|"ms_per_step"|run_or_apply|rounds'
  [ $rc -eq 0 ] || exit $rc
done
# The replica call path's timeline (kernel trace of tb_replica_bench, 300 ops).
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03b/rp_trace -o run -- \
  $GRAFT_REPO_ROOT/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 300 --warmup 20 \
  > $GRAFT_REPO_ROOT/gpurun_out/r03b/rp_trace.log 2>&1
echo "replica trace rc=$?"
exit 0
