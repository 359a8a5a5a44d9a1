"""Copy-engine timeline of a `profile.sh mc` run: per-chunk H2D body copies of the last step, their
duration, the gaps between them and the rate they imply (debug aid for the PCIe-bound headline)."""
import csv
import statistics as st
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/mc/run_memory_copy_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
h2d = [r for r in rows if r["Direction"].endswith("HOST_TO_DEVICE")]
by_stream = {}
for r in h2d:
    by_stream.setdefault(r["Stream_Id"], []).append(r)
body = max(by_stream.values(), key=len)  # the copy stream
gaps = [(int(body[i + 1]["Start_Timestamp"]) - int(body[i]["End_Timestamp"])) / 1e6 for i in range(len(body) - 1)]
cut = max(range(len(gaps)), key=lambda i: gaps[i]) + 1  # the last step starts after the longest gap
last = body[cut:]
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in last]
g = [(int(last[i + 1]["Start_Timestamp"]) - int(last[i]["End_Timestamp"])) / 1e6 for i in range(len(last) - 1)]
span = (int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])) / 1e6
print("copies per stream", {k: len(v) for k, v in by_stream.items()}, "last step copies", len(last))
print("copy ms median %.4f  gap ms median %.4f mean %.4f  span %.2f ms, busy %.1f%%"
      % (st.median(durs), st.median(g), st.mean(g), span, 100 * sum(durs) / span))
