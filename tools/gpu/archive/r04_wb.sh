#!/bin/bash
# The replica call path with the asynchronous write-back: its tests, the bench both ways, a kernel
# trace of the write-back run; then the validate A/B against round 3's kernel.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_alloc.py tests/test_gpu_checkpoint.py tests/test_gpu_determinism.py > $O/wb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/wb_tests.log | tail -8
[ $rc -ne 0 ] && { grep -E "^E " $O/wb_tests.log | head -30; exit $rc; }
for mode in "" "--write-back"; do
  timeout -k 10 300 ./tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 2000 $mode || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/replica_wb2 -o run --output-format csv -- \
  $R/tigerbeetle_amd/host/tb_replica_bench --accounts 1000000 --prepares 400 --write-back > /dev/null 2>&1 || exit 1
cd $R && AB_VARIANTS="${AB:-cur}" bash tools/gpu/r04_ab.sh
