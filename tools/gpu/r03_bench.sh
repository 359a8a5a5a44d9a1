#!/bin/bash
# Default bench (C2 headline + legs), then the node bench rehearsed with 2 logical shards.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u bench.py > gpurun_out/r03/bench_default.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r03/bench_default.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --accounts 10000000 --transfers 30000000 --steps 2 --warmup 1 \
  > gpurun_out/r03/bench_node2_same.log 2>&1
echo "node bench rc=$?"
exit 0
