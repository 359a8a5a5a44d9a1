#!/bin/bash
# Node-engine rehearsal on one GPU (2 logical shards): bench.py --gpus 2 --same-device for C2, C3, C4.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
O=gpurun_out/r04node
mkdir -p $O
for w in c3 c4 c2; do
  timeout -k 10 400 python -u bench.py --gpus 2 --same-device --workload $w --accounts 1000000 --transfers 4000000 \
    --steps 1 --warmup 1 --cpu-sample 0 > $O/node_$w.json 2> $O/node_$w.err || { echo FAIL $w; tail -20 $O/node_$w.err; exit 1; }
  python - $O/node_$w.json $w <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.1f M/s" % (d["value"] / 1e6), "passes", d.get("passes"), "parity", d.get("parity"))
PY
done
