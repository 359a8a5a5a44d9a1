"""Print the calls, mean and total duration of the kernels whose names start with the given
prefixes, from a rocprofv3 --stats kernel_stats.csv.  usage: kstats.py <csv> <prefix>..."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for pre in sys.argv[2:]:
    for r in rows:
        name = r["Name"].replace("void ", "")
        if name.startswith(pre):
            print("  %-40s calls %5s  mean %9.2f us  total %9.3f ms" % (name[:40], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                                      float(r["TotalDurationNs"]) / 1e6))
