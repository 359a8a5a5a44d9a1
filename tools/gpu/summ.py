"""One-line summary of a bench.py JSON line (debug aid for GPU runs)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"] or {}
print(sys.argv[2] if len(sys.argv) > 2 else "", d["value"], "ms/step", d["ms_per_step"], "frac", r.get("frac"),
      {k: v["avg_launch_ms"] for k, v in r.get("kernels", {}).items()}, "dep", d.get("dependent_events"),
      "parity", d.get("parity"))
