# One GPU iteration: parity tests, then the headline bench (and optional A/B runs with TBGPU_ABLATE).
# usage: bash tools/gpu/iter.sh [ablate-mask ...]      (SKIP_TESTS=1 skips pytest)
# Ablation masks act only on a timing build: build one on the CPU first with
#   TBGPU_TIMING_KNOBS=1 hipcc ... -o tigerbeetle_amd/libtbgpu_knobs.so   (see tigerbeetle_amd/build.py)
# and the runs below load it through TBGPU_AB_LIB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
summ() { python tools/gpu/summ.py "$1" "$2"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
summ gpurun_out/bench.log default
for m in "$@"; do
  TBGPU_AB_LIB=$PWD/tigerbeetle_amd/libtbgpu_knobs.so TBGPU_ABLATE=$m timeout -k 10 300 python -u bench.py --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/bench_ablate_$m.log 2>&1 || { echo ABL_FAIL $m; tail -5 gpurun_out/bench_ablate_$m.log; exit 1; }
  summ gpurun_out/bench_ablate_$m.log "ablate=$m"
done
