#!/bin/bash
# Round-5 roofline evidence: kernel trace + FETCH_SIZE + WRITE_SIZE runs of the headline leg
# (device-resident passes committed in place: tools/gpu/device_pass.py) and of the host path
# (tools/gpu/host_pass.py), summarised into gpurun_out/prof/pmc_r05.json by tools/perf_pmc.py
# (commit it as perf/pmc_r05.json, the file bench.py reads).  Leg names as bench.py reads them:
# `device` (the headline) and `headline` (kept for the host path's roofline).
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for m in ${MODES:-dkt dfetch dwrite hkt hfetch hwrite}; do
  bash "$R/tools/gpu/profile.sh" $m || { echo "profile $m failed"; exit 1; }
done
P=gpurun_out/prof
f() { find "$P/$1" -name "$2" | head -1; }
python3 "$R/tools/perf_pmc.py" "$P/pmc_r05.json" r05 \
  headline "$(f hkt '*kernel_stats.csv')" "$(f hfetch '*counter_collection.csv')" "$(f hwrite '*counter_collection.csv')" \
           20962400 523560 \
  device "$(f dkt '*kernel_stats.csv')" "$(f dfetch '*counter_collection.csv')" "$(f dwrite '*counter_collection.csv')" \
           100000000 4166667
