# rocprofv3 evidence for the headline bench (MI355X_MICROARCH.md HBM recipe): one kernel-trace +
# stats run of the default bench command, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (they do not fit in one pass on gfx950) over a shorter run of the same configuration.
# usage (on the GPU box): bash tools/gpu/profile.sh      -> gpurun_out/prof/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 "$R/bench.py" --cpu-sample 0 --host-prepares 0 \
    > "$OUT/bench_kt.log" 2>&1 || { echo KT_FAIL; tail -20 "$OUT/bench_kt.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" --cpu-sample 0 --host-prepares 0 \
    --steps 1 --warmup 0 --transfers 20000000 > "$OUT/fetch.log" 2>&1 || { echo FETCH_FAIL; tail -20 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" --cpu-sample 0 --host-prepares 0 \
    --steps 1 --warmup 0 --transfers 20000000 > "$OUT/write.log" 2>&1 || { echo WRITE_FAIL; tail -20 "$OUT/write.log"; exit 1; }
find "$OUT" -name "*.csv" | sort
tail -1 "$OUT/bench_kt.log" | cut -c1-300
