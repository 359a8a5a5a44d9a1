#!/bin/bash
# SQ counters of the pass kernels on the headline leg (one --pmc pass, 8 SQ counters).
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r04sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LEG="--cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 --write-back 0 --replica-prepares 0 --access-mix 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY \
  --output-format csv -d $O/sq -o run -- python3 $R/bench.py $LEG --steps 1 --warmup 0 > $O/sq.log 2>&1 || exit 1
python3 - $O/sq/run_counter_collection.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); calls = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:32]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": calls[k] += 1
for k, d in agg.items():
    if calls[k] < 10: continue
    n = calls[k]
    print("%-32s %5d" % (k, n), {c: round(v / n) for c, v in sorted(d.items())})
PY
