# C3 / C4 standalone (10M transfers, 1M accounts, from registered host memory) at several chunk
# sizes: the ordered path's per-chunk latency (planning barriers, dependency depth) is amortised
# over more transfers as chunks grow.  usage: bash tools/gpu/chunks.sh "64 128 256" [c3 c4]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
sizes=${1:-"64 128 256"}
shift
kinds=${*:-"c3 c4"}
for k in $kinds; do
  for c in $sizes; do
    timeout -k 10 300 python -u bench.py --workload $k --accounts 1000000 --transfers 10000000 --steps 2 --warmup 1 \
      --chunk-prepares $c --cpu-sample 0 --host-prepares 0 --device-steps 0 --secondary 0 --access-mix 0 \
      > gpurun_out/chunks_${k}_$c.log 2>&1 || { echo FAIL $k $c; tail -5 gpurun_out/chunks_${k}_$c.log; exit 1; }
    python - "$k" "$c" <<'EOF'
import json, sys
d = json.loads(open("gpurun_out/chunks_%s_%s.log" % (sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
print(sys.argv[1], "chunk", sys.argv[2], "value %.1fM" % (d["value"] / 1e6), "ms/step", d["ms_per_step"],
      "p99", d["p99_batch_latency_ms"], "phases", d["flow_phases_ms"],
      {k: v["avg_launch_ms"] for k, v in (d["roofline"] or {}).get("kernels", {}).items()})
EOF
  done
done
