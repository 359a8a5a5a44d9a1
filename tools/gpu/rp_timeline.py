"""Per-call kernel timeline of a tb_replica_bench kernel trace (rocprofv3 --kernel-trace CSV):
median duration of each kernel of a one-prepare commit and the gap before it."""
import collections, csv, statistics as st, sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ops, cur = [], None
for r in rows:
    k = r['Kernel_Name'].split('(')[0]
    if k.startswith('tb_pass_clear'):
        cur = []
        ops.append(cur)
    if cur is not None:
        cur.append((k, int(r['Start_Timestamp']), int(r['End_Timestamp'])))
ops = ops[-250:]
dur, gap, span, between = collections.defaultdict(list), collections.defaultdict(list), [], []
prev_end = None
for op in ops:
    for i, (k, s, e) in enumerate(op):
        dur[k].append(e - s)
        gap[k].append(s - op[i - 1][2] if i else 0)
    span.append(op[-1][2] - op[0][1])
    if prev_end:
        between.append(op[0][1] - prev_end)
    prev_end = op[-1][2]
for k in dur:
    print(f"{k[:40]:40s} dur {st.median(dur[k]) / 1e3:7.2f} us  gap-before {st.median(gap[k]) / 1e3:6.2f} us  n={len(dur[k])}")
print(f"span (first kernel start to last kernel end) median {st.median(span) / 1e3:.2f} us; "
      f"between calls median {st.median(between) / 1e3:.2f} us")
