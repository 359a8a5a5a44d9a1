# rocprofv3 evidence for the headline bench (MI355X_MICROARCH.md HBM recipe): a kernel-trace +
# stats run of the headline leg of the default bench command (pipelined C2 commits from host
# memory; the HBM-resident leg, the C3/C4 lines, the CPU sample and the one-prepare host leg are
# switched off so every traced launch is a headline launch), and FETCH_SIZE / WRITE_SIZE in
# separate --pmc passes (they do not fit in one pass on gfx950) over a shorter run of the same
# configuration (same chunk size, so the same launch shape).  One mode per call:
#   bash tools/gpu/profile.sh kt|fetch|write      -> gpurun_out/prof/<mode>/
#   bash tools/gpu/profile.sh dfetch|dwrite       -> FETCH_SIZE / WRITE_SIZE of device-resident C2 passes
#     (tools/gpu/device_pass.py: 512-prepare passes, no host copy in flight)
#   bash tools/gpu/profile.sh dkt                 -> kernel trace + stats of the same run
#   bash tools/gpu/profile.sh hkt|hfetch|hwrite   -> the same for the host path (tools/gpu/host_pass.py:
#     pipelined 64-prepare chunks from registered host memory)
#   bash tools/gpu/profile.sh mc                  -> memory-copy + kernel trace of one headline step
#     (the copy engine's timeline: body copies, their gaps, the per-chunk metadata copies)
#   bash tools/gpu/profile.sh nkt|nc3             -> kernel trace of the node rehearsal (2 logical shards, C2 / C3)
#   bash tools/gpu/profile.sh nkt1                -> the same C2 trace on one hardware queue (kernels serialised)
#   bash tools/gpu/profile.sh n1kt                -> kernel + copy trace of one-prepare node calls
#   bash tools/gpu/profile.sh c3|c3h|c4           -> kernel trace of `bench.py --workload c3|c3h|c4`
#     (1M accounts, 10M transfers, one timed step from host memory: tb_flow's bounds / sweep / run)
# (rocprofv3 has written its CSVs when the profiled python exits; a crash after that, in process
# teardown, leaves them complete and is reported, not hidden.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
MODE=${1:-kt}
OUT=$R/gpurun_out/prof
mkdir -p "$OUT"; rm -rf "$OUT/$MODE"
cd /tmp && export TMPDIR=/tmp
# The headline (round 5): device-resident passes; the host path (PCIe) is its own leg (--host-steps).
LEG="--cpu-sample 0 --host-prepares 0 --host-steps 0 --secondary 0 --write-back 0 --replica-prepares 0"
case $MODE in
  kt) timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" $LEG \
        > "$OUT/bench_kt.log" 2>&1; rc=$? ;;
  mc) timeout -k 10 420 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d "$OUT/mc" -o run -- \
        python3 "$R/bench.py" $LEG --access-mix 0 --steps 1 --warmup 1 > "$OUT/bench_mc.log" 2>&1; rc=$? ;;
  dfetch|dwrite) C=FETCH_SIZE; [ "$MODE" = dwrite ] && C=WRITE_SIZE
      timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$MODE" -o run -- python3 "$R/tools/gpu/device_pass.py" 100000000 \
        > "$OUT/$MODE.log" 2>&1; rc=$? ;;
  dkt) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dkt" -o run -- \
        python3 "$R/tools/gpu/device_pass.py" 100000000 > "$OUT/dkt.log" 2>&1; rc=$? ;;
  fetch|write) C=FETCH_SIZE; [ "$MODE" = write ] && C=WRITE_SIZE
      timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$MODE" -o run -- python3 "$R/bench.py" $LEG \
        --steps 1 --warmup 0 > "$OUT/$MODE.log" 2>&1; rc=$? ;;
  nkt) export GPU_MAX_HW_QUEUES=8  # as bench.py sets for the node engine (the profiler starts HIP first)
      timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nkt" -o run -- python3 "$R/bench.py" \
        --gpus 2 --same-device --accounts 2000000 --transfers 8000000 --steps 1 --warmup 1 $LEG --access-mix 0 \
        > "$OUT/bench_nkt.log" 2>&1; rc=$? ;;
  nkt1) export GPU_MAX_HW_QUEUES=1  # every stream on one hardware queue: each kernel's duration its own
      timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nkt1" -o run -- python3 "$R/bench.py" \
        --gpus 2 --same-device --accounts 2000000 --transfers 8000000 --steps 1 --warmup 1 $LEG --access-mix 0 \
        --chunk-prepares ${NKT_CHUNK:-512} > "$OUT/bench_nkt1.log" 2>&1; rc=$? ;;
  nc3) export GPU_MAX_HW_QUEUES=8
      timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nc3" -o run -- python3 "$R/bench.py" \
        --gpus 2 --same-device --workload c3 --accounts 1000000 --transfers 4000000 --steps 1 --warmup 1 $LEG --access-mix 0 \
        > "$OUT/bench_nc3.log" 2>&1; rc=$? ;;
  hfetch|hwrite) C=FETCH_SIZE; [ "$MODE" = hwrite ] && C=WRITE_SIZE
      timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$MODE" -o run -- python3 "$R/tools/gpu/host_pass.py" \
        > "$OUT/$MODE.log" 2>&1; rc=$? ;;
  hkt) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/hkt" -o run -- \
        python3 "$R/tools/gpu/host_pass.py" > "$OUT/hkt.log" 2>&1; rc=$? ;;
  n1kt) export GPU_MAX_HW_QUEUES=8  # one C2 prepare per tbgpu_commit on a 2-shard node (and a single engine)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/n1kt" -o run -- \
        python3 "$R/tools/gpu/node_one_prepare.py" 120 2 > "$OUT/n1kt.log" 2>&1; rc=$? ;;
  c3|c3h|c4) timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$MODE" -o run -- python3 "$R/bench.py" \
        --workload $MODE --accounts 1000000 --transfers 10000000 --steps 1 --warmup 0 $LEG --access-mix 0 \
        > "$OUT/bench_$MODE.log" 2>&1; rc=$? ;;
esac
echo "rc=$rc"
find "$OUT/$MODE" -name "*.csv" | sort
exit $rc
