#!/bin/bash
# Round-4 roofline evidence: kernel trace + FETCH_SIZE + WRITE_SIZE runs of the headline leg and of
# device-resident passes (tools/gpu/profile.sh modes kt fetch write dkt dfetch dwrite), summarised
# into gpurun_out/prof/pmc_r04.json (tools/perf_pmc.py; commit it as perf/pmc_r04.json, the file
# bench.py reads).  Usage: bash tools/gpu/r04_prof.sh [tests]   (tests: run the -m gpu suite first)
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/prof/pytest_all.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/prof/pytest_all.log
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/prof/pytest_all.log | head -30; exit $rc; }
fi
for m in kt fetch write dkt dfetch dwrite; do
  bash "$R/tools/gpu/profile.sh" $m || { echo "profile $m failed"; exit 1; }
done
P=gpurun_out/prof
f() { find "$P/$1" -name "$2" | head -1; }
python3 "$R/tools/perf_pmc.py" "$P/pmc_r04.json" r04 \
  headline "$(f kt '*kernel_stats.csv')" "$(f fetch '*counter_collection.csv')" "$(f write '*counter_collection.csv')" \
           100000000 523560 \
  device "$(f dkt '*kernel_stats.csv')" "$(f dfetch '*counter_collection.csv')" "$(f dwrite '*counter_collection.csv')" \
           100000000 4166667
